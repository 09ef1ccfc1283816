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
