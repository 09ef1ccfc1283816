"""Per-step wall time of the reference-semantics torch path (runtime.backend=torch, fp32) of the
Trainer on the GPU — prints every step (diagnoses a slow first step, e.g. MIOpen solver search)."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(base="resnet18", batch=512, steps=6):
    from simclr_amd.config import compose, task_config, CONF_DIR
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    from simclr_amd.ops import registry
    from simclr_amd.parallel import state as pstate
    from simclr_amd.train.pretrain import Trainer
    import os
    registry.set_backend("torch")
    if os.environ.get("PROBE_CUDNN_DET") == "1":  # what seed_everything does (main.py:150-151)
        torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False
    cfg = task_config(compose(str(CONF_DIR), "config", [
        f"experiment.base_cnn={base}", f"experiment.batches={batch}", "data.synthetic=true",
        "runtime.precision=fp32", "runtime.backend=torch"]))
    st = pstate.get()
    st.device = torch.device("cuda", 0)
    tr = Trainer(cfg, st, 50000, precision="fp32")
    ld = ContrastiveLoader(synthetic_dataset(4096, 10), batch, st.device, seed=7)
    it = iter(ld)
    for i in range(steps):
        x, _ = next(it)
        torch.cuda.synchronize()
        t = time.perf_counter()
        loss = tr.step(x)
        torch.cuda.synchronize()
        print(f"step {i} {1000 * (time.perf_counter() - t):.1f} ms loss {float(loss):.4f}",
              flush=True)


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["resnet18"]), *[int(a) for a in sys.argv[2:]])
