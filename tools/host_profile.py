"""Host-side (Python) cost of issuing one training step: cProfile over a few eager steps."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from simclr_amd.config import compose, task_config, CONF_DIR
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    from simclr_amd.parallel import state as pstate
    from simclr_amd.train.pretrain import Trainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = pstate.get()
    st.device = dev
    cfg = task_config(compose(str(CONF_DIR), "config", [
        "experiment.base_cnn=resnet50", "model.cifar_stem=true", "experiment.batches=512",
        "data.synthetic=true", "parameter.epochs=10"]))
    tr = Trainer(cfg, st, 50000)
    loader = ContrastiveLoader(synthetic_dataset(4096, 10), 512, dev, seed=7)
    it = iter(loader)
    xs = [next(it)[0] for _ in range(6)]
    for x in xs[:2]:
        tr.step(x)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for x in xs[2:]:
        tr.step(x)
    pr.disable()
    torch.cuda.synchronize()
    st_ = pstats.Stats(pr).sort_stats("tottime")
    st_.print_stats(35)


if __name__ == "__main__":
    main()
