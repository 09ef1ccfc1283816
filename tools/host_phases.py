"""Host wall time of each phase of an eager training step while the GPU runs ahead (the bench
loop's situation): a phase that takes far longer than its pure issue cost (tools/issue_cost.py)
is blocked in the HIP runtime (full queue or a synchronising call)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(steps=8):
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
    for _ in range(3):
        tr.step(next(it)[0])
    torch.cuda.synchronize()
    names = ["batch", "forward", "loss", "backward", "finish", "optimizer"]
    acc = {n: 0.0 for n in names}
    t_all = time.perf_counter()
    for _ in range(steps):
        t = [time.perf_counter()]
        x = next(it)[0]
        t.append(time.perf_counter())
        z = tr.model(x, segments=2)
        t.append(time.perf_counter())
        loss = tr.loss_fn(z)
        t.append(time.perf_counter())
        loss.backward()
        t.append(time.perf_counter())
        tr.store.finish()
        t.append(time.perf_counter())
        tr.opt.step()
        t.append(time.perf_counter())
        for i, n in enumerate(names):
            acc[n] += t[i + 1] - t[i]
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_all) / steps * 1e3
    print("per-step host ms: " + " ".join(f"{n}={acc[n] / steps * 1e3:.2f}" for n in names) +
          f" | wall/step {wall:.2f}", flush=True)


if __name__ == "__main__":
    main()
