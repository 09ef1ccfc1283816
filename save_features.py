"""Feature export entry point (reference: /root/reference/save_features.py).

    python save_features.py experiment.target_dir=PATH [parameter.use_full_encoder=true]
"""
from simclr_amd.config import hydra_main
from simclr_amd.evaluation.features import save_features


@hydra_main(config_path="conf", config_name="eval")
def main(cfg):
    return save_features(cfg)


if __name__ == "__main__":
    main()
