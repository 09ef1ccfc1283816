"""Native multi-stream replay of a captured step (csrc/graphexec.cpp, runtime/graph_exec.py)
against the HIP graph executor: identical results, bitwise, on a hand-built two-stream DAG and on
whole SimCLR training steps."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sched", ["capture", "list"])
def test_stream_replay_two_stream_dag(sched):
    from simclr_amd.runtime.graph_exec import StreamReplay
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    static = torch.randn(1 << 20, device=dev)
    side = torch.cuda.Stream(device=dev)
    g = torch.cuda.CUDAGraph(keep_graph=True)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):  # warm the allocator / kernels outside the capture
        _ = static * 2
    torch.cuda.current_stream(dev).wait_stream(s)
    with torch.cuda.graph(g):
        a = static * 2
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            b = torch.sin(static) * 3
            b.add_(1)
        c = a + 1
        c.mul_(c)
        torch.cuda.current_stream(dev).wait_stream(side)
        out = c - b
        snap = out * 1.0
        zeros = torch.zeros(4096, device=dev)
    g.instantiate()
    r = StreamReplay(g, max_streams=3, sched=sched)
    st = r.stats()
    assert st["kernels"] >= 5 and st["streams"] >= 2, st
    assert r.pending == (sched == "list")
    for k in range(3):
        static.copy_(torch.randn(1 << 20, device=dev))
        ref = (static * 2 + 1) ** 2 - (torch.sin(static) * 3 + 1)
        if k % 2:
            g.replay()
        else:
            r.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref) and torch.equal(snap, ref)
        assert not bool(zeros.any())
    if sched == "list":  # planned from the timed replay: one duration per node, a valid order
        assert not r.pending and len(r.durations) == len(r.schedule())
        assert all(d >= 0.0 for d in r.durations)
    # a long run of back-to-back replays drains (no event / stream leak or hang)
    for _ in range(200):
        r.replay()
    torch.cuda.synchronize()
    r.close()


def test_stream_replay_memcpy_nodes_as_subgraphs():
    """A D2D copy captured from hipMemcpyAsync is a 1-D memcpy node whose parameters HIP does
    not expose: the executor replays it as a one-node graph cut from a clone, in order with the
    kernels around it on its stream."""
    from simclr_amd.runtime.graph_exec import StreamReplay
    dev = torch.device("cuda", 0)
    a = torch.randn(1 << 16, device=dev)
    b = torch.empty_like(a)
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        a2 = a + 1
        b.copy_(a2)
        c = b * 2
    g.instantiate()
    r = StreamReplay(g, max_streams=2)
    st = r.stats()
    assert st["subgraphs"] >= 1 and st["kernels"] >= 2, st
    for _ in range(3):
        a.normal_()
        r.replay()
        torch.cuda.synchronize()
        assert torch.equal(b, a + 1) and torch.equal(c, (a + 1) * 2)


def _trainer(base, stem, batch):
    from simclr_amd.config import compose, task_config, CONF_DIR
    from simclr_amd.parallel import state as pstate
    from simclr_amd.train.pretrain import Trainer
    ov = [f"experiment.base_cnn={base}", f"experiment.batches={batch}", "data.synthetic=true",
          f"model.cifar_stem={'true' if stem else 'null'}", "parameter.epochs=10",
          "parameter.warmup_epochs=1"]
    cfg = task_config(compose(str(CONF_DIR), "config", ov))
    pstate.reset()
    st = pstate.get()
    st.device = torch.device("cuda", 0)
    torch.manual_seed(0)
    return Trainer(cfg, st, 512, precision="bf16")


def test_early_stage_updates_match_single_update(monkeypatch):
    """ResNet-50 CIFAR trainers with and without the per-stage early optimizer updates issued
    from the fused backward (Trainer._early_updates): the same kernels on the same data, so the
    losses, master weights and momenta agree bitwise over captured, stream-replayed steps."""
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    dev = torch.device("cuda", 0)
    loader = ContrastiveLoader(synthetic_dataset(512, 10), 64, dev, seed=9)
    xs = [x.clone() for x, _ in loader][:4]
    monkeypatch.setenv("SIMCLR_EARLY_UPDATE", "0")
    a = _trainer("resnet50", True, 64)
    monkeypatch.setenv("SIMCLR_EARLY_UPDATE", "1")
    b = _trainer("resnet50", True, 64)
    assert a.opt._rest is None and b.opt._rest is not None and len(b.opt._groups) == 3
    with torch.no_grad():
        b.store.master.copy_(a.store.master)
        b.store.refresh_shadow()
        for (_, u), (_, v) in zip(b.model.named_buffers(), a.model.named_buffers()):
            u.copy_(v)
    la = [float(a.step(xs[0]).item())]
    lb = [float(b.step(xs[0]).item())]
    assert b.opt.early_issued == 3 and b.opt._issued == set()  # issued by the backward
    for t in (a, b):
        t.capture(xs[0], warmup=0)
        t.replay_mode = "streams"
    la += [float(a.step(x).item()) for x in xs[1:]]
    lb += [float(b.step(x).item()) for x in xs[1:]]
    torch.cuda.synchronize()
    assert la == lb, (la, lb)
    assert torch.equal(a.store.master, b.store.master)
    assert torch.equal(a.opt.mom, b.opt.mom)


@pytest.mark.parametrize("base,stem,batch,sched", [("resnet18", None, 32, "capture"),
                                                    ("resnet50", True, 64, "capture"),
                                                    ("resnet50", True, 64, "list")])
def test_stream_replay_matches_graph_replay(base, stem, batch, sched, monkeypatch):
    """Two trainers from the same weights, one replaying its captured step with hipGraphLaunch,
    the other with the native multi-stream executor: the same kernels on the same data, so the
    losses, the fp32 master weights and the BatchNorm running statistics agree bitwise.  With
    ``sched="list"`` the executor's first replay is its timed serial planning step and the later
    ones follow the list schedule (gexec_reschedule)."""
    monkeypatch.setenv("SIMCLR_REPLAY_SCHED", sched)
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    dev = torch.device("cuda", 0)
    loader = ContrastiveLoader(synthetic_dataset(512, 10), batch, dev, seed=7)
    xs = [x.clone() for x, _ in loader][:5]
    a = _trainer(base, stem, batch)
    a.step(xs[0])  # eager: the autotuner settles every shape's tile (process-wide cache)
    b = _trainer(base, stem, batch)
    c = _trainer(base, stem, batch)
    with torch.no_grad():
        for t in (b, c):
            t.store.master.copy_(a.store.master)
            t.store.refresh_shadow()
            for (_, u), (_, v) in zip(t.model.named_buffers(), a.model.named_buffers()):
                u.copy_(v)
    b.capture(xs[0], warmup=0)
    c.capture(xs[0], warmup=0)
    assert c.sreplay is not None, "multi-stream executor refused the captured step"
    c.replay_mode = "streams"
    stats = c.sreplay.stats()
    print("stream replay", stats)
    # (ResNet-18 at batch 32 runs the per-module path: one stream)
    assert stats["kernels"] > 100 and stats["streams"] >= (2 if base == "resnet50" else 1), stats
    lb = [float(b.step(x).item()) for x in xs[1:]]
    lc = [float(c.step(x).item()) for x in xs[1:]]
    torch.cuda.synchronize()
    assert lb == lc, (lb, lc)
    if sched == "list":
        assert not c.sreplay.pending and c.sreplay.durations is not None
    assert torch.equal(b.store.master, c.store.master)
    for (n, u), (_, v) in zip(b.model.named_buffers(), c.model.named_buffers()):
        assert torch.equal(u, v), n
