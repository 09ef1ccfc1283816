"""Pure host cost of issuing one eager training step: each step is issued onto an idle GPU
(synchronize before), so no launch can block on a full queue; compared with the step's wall
time to the next synchronize.  Usage: python tools/issue_cost.py [--steps 6] [r50|r18]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--model", default="resnet50")
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
        f"experiment.base_cnn={args.model}", "model.cifar_stem=true", "experiment.batches=512",
        "data.synthetic=true", "parameter.epochs=10"]))
    tr = Trainer(cfg, st, 50000)
    loader = ContrastiveLoader(synthetic_dataset(8192, 10), 512, dev, seed=7)
    it = iter(loader)
    xs = [next(it)[0] for _ in range(args.steps + 3)]
    for x in xs[:3]:
        tr.step(x)
    torch.cuda.synchronize()
    hs, ws = [], []
    for x in xs[3:]:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step(x)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        hs.append((t1 - t0) * 1e3)
        ws.append((t2 - t0) * 1e3)
    print(f"issue_ms={sorted(hs)[len(hs) // 2]:.3f} wall_ms={sorted(ws)[len(ws) // 2]:.3f} "
          f"(medians over {len(hs)} steps; issue onto an idle GPU)")


if __name__ == "__main__":
    main()
