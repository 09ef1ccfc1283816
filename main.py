"""SimCLR pre-training entry point (reference: /root/reference/main.py).

    python main.py [hydra-style overrides]                  # single process
    python launch.py --nproc_per_node=8 -m main [overrides]  # one process per GPU (RCCL)
"""
from simclr_amd.config import hydra_main
from simclr_amd.train.pretrain import pretrain


@hydra_main(config_path="conf", config_name="config")
def main(cfg):
    return pretrain(cfg)


if __name__ == "__main__":
    main()
