"""Downstream evaluation entry point (reference: /root/reference/eval.py).

    python eval.py experiment.target_dir=PATH [parameter.classifier={centroid,linear,nonlinear}]
                   [parameter.use_full_encoder=true]
"""
from simclr_amd.config import hydra_main
from simclr_amd.evaluation.features import evaluate


@hydra_main(config_path="conf", config_name="eval")
def main(cfg):
    return evaluate(cfg)


if __name__ == "__main__":
    main()
