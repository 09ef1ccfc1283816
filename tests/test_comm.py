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
    with pytest.raises(ValueError):
        a.get(("bn1", "fwd"), 2, 128)  # peers hold the old layout


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
