"""End-to-end GPU checks: a full SimCLR step on the HIP path runs, is finite, and tracks the
reference-semantics torch path (fp32) over the first steps."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(base="resnet18", batch=32, cifar_stem=None, precision="bf16"):
    from simclr_amd.config import compose, task_config, CONF_DIR
    ov = [f"experiment.base_cnn={base}", f"experiment.batches={batch}", "data.synthetic=true",
          f"model.cifar_stem={'true' if cifar_stem else 'null'}", f"runtime.precision={precision}",
          "parameter.epochs=10", "parameter.warmup_epochs=1"]
    return task_config(compose(str(CONF_DIR), "config", ov))


def _trainer(cfg, precision):
    from simclr_amd.parallel import state as pstate
    from simclr_amd.train.pretrain import Trainer
    pstate.reset()
    st = pstate.get()
    st.device = torch.device("cuda", 0)
    torch.manual_seed(0)
    return Trainer(cfg, st, 512, precision=precision)


@pytest.mark.parametrize("base,stem", [("resnet18", None), ("resnet50", True), ("resnet50", None)])
def test_hip_step_runs(base, stem):
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    cfg = _cfg(base, 32, stem)
    tr = _trainer(cfg, "bf16")
    assert tr.hip
    ds = synthetic_dataset(256, 10)
    loader = ContrastiveLoader(ds, 32, torch.device("cuda", 0), seed=7)
    losses = []
    for i, (x, _) in enumerate(loader):
        losses.append(float(tr.step(x).item()))
        if i == 3:
            break
    assert all(torch.isfinite(torch.tensor(losses)))
    assert torch.isfinite(tr.store.master).all()


def test_hip_matches_fp32_first_step():
    """Loss of step 0 (before any update) on the bf16 HIP path vs the fp32 torch path."""
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    cfg = _cfg("resnet18", 32)
    ds = synthetic_dataset(64, 10)
    loader = ContrastiveLoader(ds, 32, torch.device("cuda", 0), seed=7)
    x, _ = next(iter(loader))
    t_hip = _trainer(cfg, "bf16")
    t_ref = _trainer(cfg, "fp32")
    with torch.no_grad():
        t_ref.store.master.copy_(t_hip.store.master)
    l_hip = float(t_hip.step(x).item())
    l_ref = float(t_ref.step(x).item())
    assert abs(l_hip - l_ref) < 0.05, (l_hip, l_ref)


@pytest.mark.parametrize("base,stem,max_d,mean_d,learns", [("resnet18", None, 0.03, 0.01, True),
                                                          ("resnet50", True, 0.12, 0.04, False)])
def test_golden_trajectory_20_steps(base, stem, max_d, mean_d, learns):
    """SURVEY §4.5 golden run: fixed seed, synthetic data, 20 optimizer steps of the bf16 HIP
    path against the fp32 reference-semantics torch path from the same initial weights and the
    same augmented views.  The loss trajectories must agree step by step (bf16 rounding drifts
    the weights apart slowly, so the bound is loose but still far below the loss's own motion)
    and ResNet-18 must visibly train within the 20 warmup steps (ResNet-50 at batch 32 does not
    yet, on either path).  Measured on MI355X: max |Δ| 0.005 (r18), 0.066 (r50 CIFAR stem)."""
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    cfg = _cfg(base, 32, stem)
    ds = synthetic_dataset(640, 10)
    loader = ContrastiveLoader(ds, 32, torch.device("cuda", 0), seed=7)
    xs = [x.clone() for x, _ in loader][:20]
    assert len(xs) == 20
    t_hip = _trainer(cfg, "bf16")
    t_ref = _trainer(cfg, "fp32")
    assert t_hip.hip and not t_ref.hip
    with torch.no_grad():
        t_ref.store.master.copy_(t_hip.store.master)
    l_hip = [float(t_hip.step(x).item()) for x in xs]
    l_ref = [float(t_ref.step(x).item()) for x in xs]
    diffs = [abs(a - b) for a, b in zip(l_hip, l_ref)]
    print("hip", [round(v, 4) for v in l_hip])
    print("ref", [round(v, 4) for v in l_ref])
    assert max(diffs) < max_d and sum(diffs) / len(diffs) < mean_d, (diffs, l_hip, l_ref)
    if learns:
        assert sum(l_hip[-5:]) < sum(l_hip[:5]) - 0.5 and sum(l_ref[-5:]) < sum(l_ref[:5]) - 0.5


def test_hip_graph_replay_matches_eager():
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    cfg = _cfg("resnet18", 32)
    ds = synthetic_dataset(256, 10)
    loader = ContrastiveLoader(ds, 32, torch.device("cuda", 0), seed=7)
    xs = [x for x, _ in loader][:5]
    a = _trainer(cfg, "bf16")
    b = _trainer(cfg, "bf16")
    with torch.no_grad():
        b.store.master.copy_(a.store.master)
        b.store.refresh_shadow()
    b.capture(xs[0], warmup=0)  # capture only: no warmup updates, so both start equal
    la = [float(a.step(x).item()) for x in xs]
    lb = [float(b.step(x).item()) for x in xs]
    for u, v in zip(la, lb):
        assert abs(u - v) < 2e-2 * max(1.0, abs(u)), (la, lb)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("tuned", [False, True])
def test_golden_trajectory_resnet50_batch128_60_steps(tuned, monkeypatch):
    """The flagship model trains on the bf16 HIP path: ResNet-50 (CIFAR stem), batch 128, 60
    optimizer steps (warmup + cosine, LARS) against the fp32 reference-semantics torch path
    from identical weights and views.  Both losses must fall by >= 0.3 (measured: 5.54 -> 4.8
    on both paths) and the trajectories must agree:

    * ``tuned=False``: the tiles pinned (autotuner off, fixed default variants, the
      ``runtime.deterministic`` policy) and the tight bounds — a numerics change in a kernel
      shows here without the tile choice moving underneath it;
    * ``tuned=True``: the autotuner ON (the tiles production selects on this box, including the
      weight-gradient variants 20-26) with looser running-mean bounds, since the chosen tiles'
      summation orders vary from box to box."""
    from simclr_amd.ops import tuning
    monkeypatch.setattr(tuning, "ENABLED", tuning.ENABLED)  # both restored after the test
    monkeypatch.setattr(tuning, "_CACHE", {})
    tuning.set_enabled(tuned)
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    from simclr_amd.config import compose, task_config, CONF_DIR
    ov = ["experiment.base_cnn=resnet50", "experiment.batches=128", "data.synthetic=true",
          "model.cifar_stem=true", "parameter.epochs=8", "parameter.warmup_epochs=1"]
    cfg = task_config(compose(str(CONF_DIR), "config", ov))
    ds = synthetic_dataset(1024, 10)
    dev = torch.device("cuda", 0)
    xs = []
    for ep in range(1, 9):
        loader = ContrastiveLoader(ds, 128, dev, seed=7)
        loader.set_epoch(ep)
        xs += [x.clone() for x, _ in loader]
    xs = xs[:60]
    assert len(xs) == 60

    def trainer(precision):
        from simclr_amd.parallel import state as pstate
        from simclr_amd.train.pretrain import Trainer
        pstate.reset()
        st = pstate.get()
        st.device = dev
        torch.manual_seed(0)
        return Trainer(cfg, st, len(ds), precision=precision)
    t_hip = trainer("bf16")
    t_ref = trainer("fp32")
    assert t_hip.hip and not t_ref.hip
    with torch.no_grad():
        t_ref.store.master.copy_(t_hip.store.master)
    # the PRODUCTION path: autotuner on (the tiles training and bench.py select on this box).
    # The fp32 reference runs stock MIOpen convolutions whose algorithm choice also varies from
    # box to box, and the bf16-vs-fp32 rounding difference grows chaotically over the steps, so
    # step-wise agreement is only demanded while the weights are still nearly identical (first
    # 5 steps); afterwards the trajectories are compared as 10-step running means (the
    # per-batch losses jump ±0.1).  Calibration (MI355X, 6 runs, pinned and autotuned tiles):
    # first-5 max |d| <= 0.013; 10-step running-mean |d| max 0.033-0.153, mean 0.012-0.061.
    l_hip = [float(t_hip.step(x).item()) for x in xs]
    l_ref = [float(t_ref.step(x).item()) for x in xs]
    diffs = [abs(a - b) for a, b in zip(l_hip, l_ref)]
    print("hip", [round(v, 3) for v in l_hip])
    print("ref", [round(v, 3) for v in l_ref])
    print("max |d|", max(diffs), "mean |d|", sum(diffs) / len(diffs))
    first_h, last_h = sum(l_hip[:10]) / 10, sum(l_hip[-10:]) / 10
    first_r, last_r = sum(l_ref[:10]) / 10, sum(l_ref[-10:]) / 10
    assert last_h < first_h - 0.3 and last_r < first_r - 0.3, (first_h, last_h, first_r, last_r)
    if not tuned:
        # pinned tiles (the round-3 bounds): step-wise over 20 steps, 5-step running means
        assert max(diffs[:20]) < 0.06, diffs[:20]
        rm = [abs(sum(l_hip[i:i + 5]) - sum(l_ref[i:i + 5])) / 5 for i in range(len(xs) - 4)]
        print("5-step running-mean |d| max", max(rm), "mean", sum(rm) / len(rm))
        assert max(rm) < 0.12 and sum(rm) / len(rm) < 0.05, rm
        return
    assert max(diffs[:5]) < 0.04, diffs[:5]
    rm = [abs(sum(l_hip[i:i + 10]) - sum(l_ref[i:i + 10])) / 10 for i in range(len(xs) - 9)]
    print("10-step running-mean |d| max", max(rm), "mean", sum(rm) / len(rm))
    assert max(rm) < 0.2 and sum(rm) / len(rm) < 0.08, rm
