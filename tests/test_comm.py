"""Host-side logic of the IPC BatchNorm statistics exchange (comm/ipc.py): deterministic site
allocation (every rank must place a BatchNorm's region at the same arena offset) and the
fallback decision without GPUs.  The exchange itself runs in tests/test_gpu_distributed.py."""
import pytest

from simclr_amd.comm.ipc import SiteTable, region_words, setup_stats_exchange


def test_site_table_is_first_call_order_and_stable():
    a, b = SiteTable(8, 1 << 20, 1024), SiteTable(8, 1 << 20, 1024)
    keys = [("bn1", "fwd", 2, 64), ("bn2", "fwd", 2, 256), ("bn2", "bwd", 2, 256)]
    offs_a = [a.get(k[:2], k[2], k[3]) for k in keys]
    offs_b = [b.get(k[:2], k[2], k[3]) for k in keys]
    assert offs_a == offs_b
    assert offs_a[0] == (0, 0, 1)
    assert offs_a[1] == (region_words(8, 2, 64), 1, 4)
    assert a.get(("bn1", "fwd"), 2, 64) == offs_a[0]  # stable on reuse
    # the same module name at another shape (another model built in this process) gets a new
    # region; the old one stays where the peers expect it
    other = a.get(("bn1", "fwd"), 2, 128)
    assert other[0] >= offs_a[2][0] + region_words(8, 2, 256)
    assert a.get(("bn1", "fwd"), 2, 64) == offs_a[0]


def test_site_keys_are_module_names_and_survive_rebuild():
    """IPC sites are keyed by qualified module name (not id()): a model rebuilt in the same
    process maps onto the same arena regions instead of leaking new ones."""
    from simclr_amd.models.contrastive import ContrastiveModel, SupervisedModel
    from simclr_amd.parallel.state import site_key
    t = SiteTable(2, 1 << 22, 1 << 12)

    def alloc(m):
        return [t.get(site_key(bn, d), 2, bn.num_features)
                for bn in m.modules() if hasattr(bn, "running_mean") for d in ("fwd", "bwd")]
    m1 = ContrastiveModel("resnet18")
    a1 = alloc(m1)
    used = t.next_word
    a2 = alloc(ContrastiveModel("resnet18"))
    assert a1 == a2 and t.next_word == used
    assert site_key(m1.f.layer2[0].downsample[1], "fwd") == ("f.layer2.0.downsample.1", "fwd")
    assert site_key(SupervisedModel("resnet18").f.bn1, "bwd") == ("f.bn1", "bwd")


class _FakeIpc:
    def __init__(self):
        import torch
        self.err = torch.zeros(1, dtype=torch.int32)


class _FakeSt:
    comm, rank, group = True, 0, None

    def __init__(self):
        self.ipc = _FakeIpc()


def test_step_guard_tuning_steps_detach_ipc(monkeypatch):
    from simclr_amd.comm import ipc as ipcmod
    from simclr_amd.ops import tuning
    monkeypatch.setattr(tuning, "sync_from_rank0", lambda group=None: 0)
    st = _FakeSt()
    g = ipcmod.StepGuard(st)
    seen = [g.run(lambda: st.ipc is None) for _ in range(ipcmod.TUNING_STEPS + 2)]
    assert seen == [True] * ipcmod.TUNING_STEPS + [False, False]
    assert st.ipc is not None


def test_step_guard_raises_on_exchange_timeout():
    """A timed-out exchange (sticky device flag) stops training at the next step instead of
    running on partial BatchNorm statistics until the epoch ends."""
    from simclr_amd.comm.ipc import IpcExchangeError, StepGuard
    st = _FakeSt()
    g = StepGuard(st)
    g.check(0)
    g.check(1)  # flag clear
    st.ipc.err.fill_(1)
    g.check(2)  # copies the set flag (asynchronously on a GPU)
    with pytest.raises(IpcExchangeError):
        g.check(3)
    d = StepGuard(st, on_error="defer")
    d.check(0)
    d.check(1)  # deferred: the caller (bench.py) checks collectively


def _guard_worker(rank, world, port, out_dir, s_bad):
    import os
    import time
    import torch
    import torch.distributed as dist
    from simclr_amd.comm.ipc import IpcExchangeError, StepGuard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class St:
        comm = True
    st = St()
    st.rank, st.group, st.ipc = rank, dist.group.WORLD, _FakeIpc()
    g = StepGuard(st)
    raised_at = -1
    for step in range(s_bad + 4):
        def body():
            if step == s_bad:
                if rank == 1:
                    time.sleep(0.5)  # rank 1 arrives late at this step's exchanges ...
                elif st.ipc is not None:
                    st.ipc.err.fill_(1)  # ... so rank 0's spin times out (sticky device flag)
        try:
            g.run(body)
            g.check(step)
        except IpcExchangeError:
            raised_at = step
            break
    with open(os.path.join(out_dir, f"g{rank}"), "w") as f:
        f.write(str(raised_at))
    dist.destroy_process_group()


def test_step_guard_timeout_raises_on_every_rank_within_one_step(tmp_path, monkeypatch):
    """A peer's late arrival makes rank 0's exchange time out at step s: EVERY rank (the late
    one too, which saw no timeout itself) raises IpcExchangeError no later than step s + 1 —
    the flag is all-reduced on the device and its copy is awaited one step later."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    s_bad = 4  # after the RCCL-statistics tuning steps
    mp.spawn(_guard_worker, args=(2, port, str(tmp_path), s_bad), nprocs=2, join=True)
    for r in range(2):
        at = int((tmp_path / f"g{r}").read_text())
        assert s_bad <= at <= s_bad + 1, (r, at)


def test_site_table_exhaustion():
    t = SiteTable(8, region_words(8, 2, 64), 16)
    t.get("x", 2, 64)
    with pytest.raises(RuntimeError):
        t.get("y", 2, 64)


def test_no_exchange_on_cpu_or_single_rank():
    class St:
        comm, world_size, rank = False, 1, 0
    import torch
    st = St()
    assert setup_stats_exchange(st, torch.device("cpu")) is None and st.ipc is None


def _fallback_worker(rank, world, port, out_dir):
    import os
    import torch
    import torch.distributed as dist
    from simclr_amd.comm import fallback_if_failed
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class FakeExchange:  # stands in for IpcStatsExchange: only rank 1 saw a spin time out
        def failed(self):
            return rank == 1

    class St:
        pass
    st = St()
    st.rank, st.group, st.ipc = rank, dist.group.WORLD, FakeExchange()
    switched = fallback_if_failed(st, torch.device("cpu"))
    st2 = St()
    st2.rank, st2.group, st2.ipc = rank, dist.group.WORLD, None
    untouched = fallback_if_failed(st2, torch.device("cpu"))
    with open(os.path.join(out_dir, f"fb{rank}"), "w") as f:
        f.write(f"{int(switched)} {int(st.ipc is None)} {int(untouched)}")
    dist.destroy_process_group()


def test_timeout_fallback_is_collective(tmp_path):
    """One rank's timed-out exchange switches EVERY rank to RCCL (the decision is all-reduced,
    so no rank keeps waiting in an exchange its peers abandoned)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_fallback_worker, args=(3, port, str(tmp_path)), nprocs=3, join=True)
    for r in range(3):
        assert (tmp_path / f"fb{r}").read_text() == "1 1 0"


def _tuning_worker(rank, world, port, out_dir):
    import os
    import torch.distributed as dist
    from simclr_amd.ops import tuning
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tuning._CACHE.clear()
    # each rank timed the same shapes on its own GPU: near-ties resolved differently
    tuning._CACHE.update({("igemm", (1, 2, 3)): rank, ("wgrad", (4, 5)): 7,
                          ("igemm", (9,)): 3 + rank})
    changed = tuning.sync_from_rank0()
    with open(os.path.join(out_dir, f"t{rank}"), "w") as f:
        f.write(repr((sorted(tuning.table().items()), changed)))
    dist.destroy_process_group()


def test_tuning_tables_identical_across_ranks(tmp_path):
    """After the tuning steps every rank runs rank 0's tile choices (the reference pins one
    algorithm everywhere: cudnn.deterministic, /root/reference/main.py:150-151)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_tuning_worker, args=(3, port, str(tmp_path)), nprocs=3, join=True)
    got = [eval((tmp_path / f"t{r}").read_text()) for r in range(3)]
    assert got[0][0] == got[1][0] == got[2][0]
    assert dict(got[0][0])[("igemm", (1, 2, 3))] == 0
    assert [g[1] for g in got] == [0, 2, 2]
