"""Multi-process correctness without a cluster: gloo, world_size 2, CPU.

* flat-store bucketed DDP + segmented SyncBN + global-negative NT-Xent (``loss.gather``) on 2
  ranks with n images each gives the same parameter gradients as 1 process with 2n images;
* SyncBN running statistics agree with the single-process batch statistics;
* the fail-fast launcher terminates surviving ranks when one rank dies.
"""
import os
import socket
import subprocess
import sys
import tempfile
import textwrap
import time
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n_total, size=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    v0 = torch.rand(n_total, 3, size, size, generator=g, dtype=torch.float64)
    v1 = torch.rand(n_total, 3, size, size, generator=g, dtype=torch.float64)
    return v0, v1


def _model(seed=0):
    """fp64 ResNet-18: the equivalence is checked to ~1e-12, far below the fp32 noise that
    per-rank partial sums vs one full-batch sum amplify through a dozen tiny-batch BN
    backwards (≈1e-2 relative at W=4 in fp32 — conditioning, not semantics)."""
    from simclr_amd.models import ContrastiveModel
    torch.manual_seed(seed)
    return ContrastiveModel("resnet18", d=32).double()


def _worker(rank, world, port, n, out_dir, gather=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from simclr_amd.loss.ntxent import NTXent
    from simclr_amd.parallel import state as pstate
    from simclr_amd.parallel.flat import FlatParamStore
    pstate.set_state(rank=rank, world_size=world, local_rank=rank, group=dist.group.WORLD)
    torch.set_num_threads(1)
    m = _model()
    store = FlatParamStore(m, "cpu", shadow_dtype=None, bucket_mb=1.0, first_bucket_mb=0.25,
                           dtype=torch.float64)
    store.broadcast_from(0)
    v0, v1 = _data(n * world)
    x = torch.cat([v0[rank * n:(rank + 1) * n], v1[rank * n:(rank + 1) * n]])
    z = m(x, segments=2)
    loss = NTXent(0.5, gather=gather)(z)
    store.zero_grad()
    loss.backward()
    store.finish()
    if rank == 0:
        torch.save({"grad": store.grad.clone() / world, "names": store.names,
                    "rm": m.f.layer1[0].bn1.running_mean.clone(), "loss": loss.detach()},
                   os.path.join(out_dir, "r0.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,gather", [(2, True), (4, True), (2, False), (4, False)])
def test_ddp_syncbn_gather_equivalence(tmp_path, world, gather):
    """W ranks × n images vs one process with W·n images (per-view BN over the whole batch).
    gather=True: global negatives, the loss equals the single-process loss on the full batch.
    gather=False (reference semantics): each rank's loss uses its own 2n rows as negatives and
    DDP averages the gradients, i.e. the single-process gradient of the mean of the W shard
    losses computed from the full-batch (SyncBN) embeddings."""
    from simclr_amd.loss.ntxent import NTXent
    from simclr_amd.parallel import state as pstate
    from simclr_amd.parallel.flat import FlatParamStore
    n = 4
    mp.spawn(_worker, args=(world, _free_port(), n, str(tmp_path), gather), nprocs=world,
             join=True)
    got = torch.load(tmp_path / "r0.pt", weights_only=True)
    pstate.reset()
    m = _model()
    store = FlatParamStore(m, "cpu", shadow_dtype=None, dtype=torch.float64)
    v0, v1 = _data(n * world)
    z = m(torch.cat([v0, v1]), segments=2)
    if gather:
        loss = NTXent(0.5)(z)
    else:
        z0, z1 = z[:n * world], z[n * world:]
        loss = sum(NTXent(0.5)(torch.cat([z0[r * n:(r + 1) * n], z1[r * n:(r + 1) * n]]))
                   for r in range(world)) / world
    store.zero_grad()
    loss.backward()
    assert got["names"] == store.names
    rel = (got["grad"] - store.grad).abs().max() / store.grad.abs().max()
    assert rel < 1e-10, float(rel)
    assert torch.allclose(got["rm"], m.f.layer1[0].bn1.running_mean, rtol=1e-10, atol=1e-12)


def _ring_worker(rank, world, port, n, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from simclr_amd.loss.ntxent import nt_xent_torch
    from simclr_amd.loss.ring import nt_xent_ring
    torch.set_num_threads(1)
    g = torch.Generator().manual_seed(3)
    zall = torch.randn(world, 2 * n, 16, generator=g, dtype=torch.float64).float()
    out = {}
    for name, fn in (("ring", lambda z: nt_xent_ring(z, n, 0.5, dist.group.WORLD, world, rank)),
                     ("gather", lambda z: nt_xent_torch(z, n, 0.5, "mean", True,
                                                        dist.group.WORLD, world, rank))):
        z = zall[rank].clone().requires_grad_(True)
        loss = fn(z)
        loss.backward()
        out[name] = (loss.detach(), z.grad.clone())
    torch.save(out, os.path.join(out_dir, f"ring{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_ring_ntxent_matches_gathered(tmp_path, world):
    """loss.gather=ring (blocks circulated point-to-point, online log-sum-exp) gives the same
    per-rank loss and embedding gradient as the all-gather implementation."""
    n = 6
    mp.spawn(_ring_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        got = torch.load(tmp_path / f"ring{r}.pt", weights_only=True)
        (lr, gr), (lg, gg) = got["ring"], got["gather"]
        assert torch.allclose(lr, lg, rtol=1e-5, atol=1e-6), (r, float(lr), float(lg))
        assert torch.allclose(gr, gg, rtol=1e-4, atol=1e-6), (r, float((gr - gg).abs().max()))


def test_launcher_fail_fast(tmp_path):
    script = tmp_path / "job.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)
    """))
    t0 = time.time()
    r = subprocess.run([sys.executable, str(ROOT / "launch.py"), "--nproc_per_node=2", "--use_env",
                        "--kill_grace=2", str(script)], cwd=str(tmp_path), timeout=90)
    assert r.returncode == 3
    assert time.time() - t0 < 60


def test_launcher_env_and_overrides():
    from simclr_amd.runtime.launcher import build_commands, parse_args
    cmds = build_commands(parse_args(["--nproc_per_node=2", "--nnodes=2", "--node_rank=1", "-m",
                                      "main", "parameter.epochs=1"]))
    (c0, e0), (c1, e1) = cmds
    assert e0["RANK"] == "2" and e1["RANK"] == "3" and e1["LOCAL_RANK"] == "1"
    assert e0["WORLD_SIZE"] == "4"
    assert c1[-3:] == ["distributed.local_rank=1", "distributed.world_size=4",
                       "parameter.epochs=1"]
    assert c0[1:4] == ["-u", "-m", "main"]


@pytest.mark.parametrize("base,stem", [("resnet50", True), ("resnet18", None)])
def test_bucket_layout(base, stem):
    """Buckets tile the flat gradient contiguously in backward order; the first holds the head,
    the last (stem + layer1: the only all-reduce left exposed after the backward) is small."""
    from simclr_amd.models import ContrastiveModel
    from simclr_amd.parallel import state as pstate
    from simclr_amd.parallel.flat import FlatParamStore
    pstate.reset()
    m = ContrastiveModel(base, cifar_stem=stem)
    st = FlatParamStore(m, "cpu", shadow_dtype=None, bucket_mb=32.0, first_bucket_mb=4.0,
                        last_bucket_mb=2.0)
    assert st.buckets[0][0] == 0 and st.buckets[-1][1] == st.total
    for (b0, e0, _), (b1, _, _) in zip(st.buckets, st.buckets[1:]):
        assert e0 == b1
    assert sum(c for _, _, c in st.buckets) == len(st.params)
    assert st.bucket_of == sorted(st.bucket_of)
    mib = [(e - b) * 4 / 2 ** 20 for b, e, _ in st.buckets]
    assert mib[-1] <= 2.0 and mib[0] <= 4.0 and max(mib) <= 32.0, mib
    assert st.names[-1] == "f.conv1.weight" and st.bucket_of[-1] == len(st.buckets) - 1
    assert st.names[0].startswith("g.")
