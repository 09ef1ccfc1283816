"""Program for a rocprofv3 --pmc run measuring the HBM traffic of whole training steps: 3
warm-up steps (autotuning), a marker kernel (torch.cumsum over a 3-element int tensor, absent
from the step), then --steps timed-shape steps.  tools/step_bytes_summary.py sums the counters
of every dispatch after the marker.  Usage (GPU box):
  tools/pmc.sh fetch "FETCH_SIZE" -- python3 tools/step_bytes.py --steps 2"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
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
    loader = ContrastiveLoader(synthetic_dataset(8192, 10), 512, dev, seed=7)
    it = iter(loader)
    xs = [next(it)[0] for _ in range(args.steps + 3)]
    for x in xs[:3]:
        tr.step(x)
    torch.cuda.synchronize()
    torch.cumsum(torch.arange(3, device=dev), 0)  # marker
    torch.cuda.synchronize()
    for x in xs[3:]:
        tr.step(x)
    torch.cuda.synchronize()
    print(f"[step_bytes] {args.steps} steps after the marker")


if __name__ == "__main__":
    main()
