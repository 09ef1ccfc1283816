"""Supervised baseline entry point (reference: /root/reference/supervised.py).

    python launch.py --nproc_per_node=8 -m supervised parameter.epochs=200
"""
from simclr_amd.config import hydra_main
from simclr_amd.train.supervised import supervised


@hydra_main(config_path="conf", config_name="supervised_config")
def main(cfg):
    return supervised(cfg)


if __name__ == "__main__":
    main()
