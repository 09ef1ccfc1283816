"""Gathered NT-Xent over the one-shot IPC collectives (comm/ipc.py ``all_gather`` /
``reduce_scatter``, csrc/comm.hip) against the process-group collectives: 2 ranks share cuda:0
over gloo (RCCL refuses two ranks on one device) — the same kernels and arena protocol as the
driver's one-rank-per-GPU runs.  Loss and the embedding gradient are bitwise equal (the
reduce-scatter sums in rank order; with 2 ranks a + b is the process group's sum too).
Reference: the columns of /root/reference/loss.py:42-52 extended to the global batch
(SURVEY §5.7, §5.8)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from simclr_amd.comm import setup_stats_exchange
    from simclr_amd.loss.ntxent import NTXent
    from simclr_amd.parallel import state as pstate
    st = pstate.set_state(rank=rank, world_size=world, local_rank=0, group=dist.group.WORLD,
                          backend="gloo", force_comm=True)
    st.device = dev
    ex = setup_stats_exchange(st, dev, mode="ipc")
    assert ex is not None
    R, D = 256, 128
    g = torch.Generator(device="cpu").manual_seed(100 + rank)
    z0 = torch.randn(R, D, generator=g).to(dev, torch.bfloat16)
    loss_fn = NTXent(0.5, gather=True)
    res = {}
    for mode in ("ipc", "pg", "ipc2"):  # ipc twice: both arena parities, epochs advance
        st.ipc = ex if mode.startswith("ipc") else None
        z = z0.clone().requires_grad_(True)
        loss = loss_fn(z)
        loss.backward()
        torch.cuda.synchronize()
        res[mode] = (loss.detach().cpu(), z.grad.detach().float().cpu())
    st.ipc = ex
    ok_loss = torch.equal(res["ipc"][0], res["pg"][0]) and torch.equal(res["ipc2"][0], res["pg"][0])
    ok_grad = torch.equal(res["ipc"][1], res["pg"][1]) and torch.equal(res["ipc2"][1], res["pg"][1])
    failed = ex.failed()
    dist.barrier()
    ex.close()
    with open(os.path.join(out_dir, f"r{rank}"), "w") as f:
        f.write(f"{int(ok_loss)} {int(ok_grad)} {int(failed)} {float(res['pg'][0]):.6f} "
                f"{float((res['ipc'][1] - res['pg'][1]).abs().max()):.3e}")
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gathered_ntxent_ipc_matches_process_group(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        got = (tmp_path / f"r{r}").read_text().split()
        assert got[:3] == ["1", "1", "0"], (r, got)
