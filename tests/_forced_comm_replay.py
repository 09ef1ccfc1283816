"""Worker of tests/test_gpu_forced_comm.py (run as its own process: it owns a 1-rank RCCL
process group, which the pytest process must not inherit).

Every collective of the N > 1 training step — bucketed gradient all-reduces on the comm stream,
the BatchNorm-statistics all-reduces on their own communicator, the z all-gather / column
reduce-scatter of the global-negatives loss — is issued on a 1-rank RCCL group, and the same
step is run three ways from the same weights on the same batches:

* eager issue (Python, per-op);
* the captured step replayed by ``hipGraphLaunch``;
* the captured step replayed by the native multi-stream executor with the capture-order plan
  over 4 streams (the N > 1 default of ``Trainer.capture``).

Losses, fp32 master, LARS momentum, the device step counter and every BatchNorm buffer must
agree bitwise after 4 steps.  Prints one JSON line per loss variant.
"""
from __future__ import annotations

import datetime
import json
import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _trainer(st, gather: bool, batch: int):
    from simclr_amd.config import compose, task_config, CONF_DIR
    from simclr_amd.train.pretrain import Trainer
    ov = ["experiment.base_cnn=resnet50", f"experiment.batches={batch}", "data.synthetic=true",
          "model.cifar_stem=true", "parameter.epochs=10", "parameter.warmup_epochs=1",
          f"loss.gather={'true' if gather else 'false'}"]
    cfg = task_config(compose(str(CONF_DIR), "config", ov))
    torch.manual_seed(0)
    return Trainer(cfg, st, 512, precision="bf16")


def _state(t):
    bufs = [b.detach().clone() for b in t.model.buffers()]
    return (t.store.master.detach().clone(), t.opt.mom.detach().clone(),
            t.opt.step_t.detach().clone(), bufs)


def run(st, gather: bool, batch: int, xs) -> dict:
    from simclr_amd.parallel import invariant as inv
    t0 = _trainer(st, gather, batch)
    t0.step(xs[0])  # eager: the autotuner settles every shape's tile (process-wide cache)
    arms = {}
    for name in ("eager", "graph", "streams"):
        t = _trainer(st, gather, batch)
        with torch.no_grad():
            t.store.master.copy_(t0.store.master)
            t.store.refresh_shadow()
            for u, v in zip(t.model.buffers(), t0.model.buffers()):
                u.copy_(v)
        arms[name] = t
    for name in ("graph", "streams"):
        t = arms[name]
        t.capture(xs[0], warmup=0)
        t.replay_mode = name
    sr = arms["streams"].sreplay
    assert sr is not None, "multi-stream executor refused the captured step"
    stats = sr.stats()
    losses = {n: [] for n in arms}
    for x in xs[1:]:
        for n, t in arms.items():
            losses[n].append(float(t.step(x).item()))
    torch.cuda.synchronize()
    ref = _state(arms["eager"])
    res = {"gather": gather, "batch": batch, "losses": losses, "stream_stats": stats,
           "equal": {}}
    for n in ("graph", "streams"):
        s = _state(arms[n])
        res["equal"][n] = {
            "loss": losses[n] == losses["eager"],
            "master": bool(torch.equal(s[0], ref[0])),
            "momentum": bool(torch.equal(s[1], ref[1])),
            "step": bool(torch.equal(s[2], ref[2])),
            "buffers": all(torch.equal(a, b) for a, b in zip(s[3], ref[3])),
            "fingerprint": bool(torch.equal(
                inv.fingerprint(arms[n].store, arms[n].opt, arms[n].model),
                inv.fingerprint(arms["eager"].store, arms["eager"].opt,
                                arms["eager"].model))),
        }
    res["learned"] = losses["eager"][-1] == losses["eager"][-1]
    for t in arms.values():
        if t.sreplay is not None:
            t.sreplay.close()
    return res


def zgather_overlap(st, dev) -> dict:
    """Global negatives at a batch the fused head takes (256 rows per view): z all-gathered
    view by view under the head's GEMM 2 (models/head_fused.py _gemm2_pregather) against the
    loss's one-shot all-gather, eagerly and as a captured step replayed by the multi-stream
    executor — losses and fp32 master bitwise equal over 3 steps."""
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    from simclr_amd.models import head_fused
    batch = 256
    loader = ContrastiveLoader(synthetic_dataset(1024, 10), batch, dev, seed=11)
    xs = [x.clone() for x, _ in loader][:4]
    out = {"zgather": True}
    arms = {}
    for name, flag in (("oneshot", "0"), ("overlap", "1"), ("overlap_streams", "1")):
        os.environ["SIMCLR_ZGATHER_OVERLAP"] = flag
        t = _trainer(st, True, batch)
        c0 = head_fused.PREGATHER_CALLS[0]
        t.step(xs[0])  # eager, every arm: the head's weight-transpose plan exists before capture
        if name == "overlap_streams":
            t.capture(xs[0], warmup=0)
            t.replay_mode = "streams"
        ls = [float(t.step(x).item()) for x in xs[1:]]
        torch.cuda.synchronize()
        arms[name] = (ls, t.store.master.detach().clone(), head_fused.PREGATHER_CALLS[0] - c0)
        if t.sreplay is not None:
            t.sreplay.close()
    os.environ.pop("SIMCLR_ZGATHER_OVERLAP", None)
    ref = arms["oneshot"]
    out["losses"] = {k: v[0] for k, v in arms.items()}
    out["pregather_calls"] = {k: v[2] for k, v in arms.items()}
    out["equal"] = {k: {"loss": v[0] == ref[0], "master": bool(torch.equal(v[1], ref[1]))}
                    for k, v in arms.items() if k != "oneshot"}
    return out


def main() -> int:
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", sys.argv[1] if len(sys.argv) > 1 else "29541")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev,
                            timeout=datetime.timedelta(seconds=120))
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    from simclr_amd.parallel import state as pstate
    st = pstate.set_state(rank=0, world_size=1, local_rank=0, group=dist.group.WORLD,
                          backend="nccl", force_comm=True)
    st.device = dev
    pstate.make_stat_group(st)
    assert st.comm, "forced 1-rank group did not enable the collectives"
    batch = int(os.environ.get("FORCED_BATCH", "64"))
    loader = ContrastiveLoader(synthetic_dataset(512, 10), batch, dev, seed=7)
    xs = [x.clone() for x, _ in loader][:5]
    for gather in (False, True):
        print(json.dumps(run(st, gather, batch, xs)), flush=True)
    print(json.dumps(zgather_overlap(st, dev)), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
