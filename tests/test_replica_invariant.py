"""Data-parallel replica invariant (parallel/invariant.py) on 2 gloo ranks: identical replicas
pass, and a one-ulp change of one rank's master weight, momentum or BatchNorm buffer is caught
on EVERY rank (the field is named); ``resync`` restores rank 0's state; the training loop's
epoch-end check raises ``ReplicaDivergence``.  Reference: the DDP invariant of
/root/reference/main.py:176-178 (never checked there)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from simclr_amd.models import ContrastiveModel
    from simclr_amd.optim.lars import FusedLARS, weight_decay_per_param
    from simclr_amd.parallel import invariant as inv
    from simclr_amd.parallel import state as pstate
    from simclr_amd.parallel.flat import FlatParamStore
    pstate.set_state(rank=rank, world_size=world, local_rank=rank, group=dist.group.WORLD)
    torch.manual_seed(rank)  # different init per rank: broadcast_from(0) must equalise them
    m = ContrastiveModel("resnet18", d=16)
    store = FlatParamStore(m, "cpu", shadow_dtype=None, bucket_mb=1.0, first_bucket_mb=0.25)
    store.broadcast_from(0)
    opt = FusedLARS(store, weight_decay_per_param(store, 1e-4), lr0=0.1, momentum=0.9)
    res = {}
    res["init"] = inv.check_replicas(store, opt)
    # one real data-parallel step on rank-specific data keeps the replicas identical
    torch.manual_seed(100 + rank)
    x = torch.rand(8, 3, 16, 16)
    from simclr_amd.loss.ntxent import NTXent
    store.zero_grad()
    NTXent(0.5)(m(x, segments=2)).backward()
    store.finish()
    opt.step()
    res["after_step"] = inv.check_replicas(store, opt)

    def corrupt(t, i=5):
        if rank == 1:
            with torch.no_grad():
                v = t.view(-1)
                v[i] = torch.nextafter(v[i], v[i] + 1.0)

    corrupt(store.master)
    res["master"] = inv.check_replicas(store, opt)
    inv.resync(store, opt)
    res["resynced"] = inv.check_replicas(store, opt)
    corrupt(opt.mom)
    res["momentum"] = inv.check_replicas(store, opt)
    inv.resync(store, opt)
    corrupt(m.f.layer1[0].bn1.running_var, 3)
    res["buffers"] = inv.check_replicas(store, opt)
    try:
        inv.require_replicas(store, opt, where="at epoch 1")
        res["raised"] = None
    except inv.ReplicaDivergence as e:
        res["raised"] = str(e)
    inv.resync(store, opt)
    # a swap of two master values keeps the 32-bit word sum but not the 64-bit one
    if rank == 1:
        with torch.no_grad():
            a, b = float(store.master[0]), float(store.master[3])
            store.master[0], store.master[3] = b, a
    res["swap"] = inv.check_replicas(store, opt)
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_replica_check_catches_divergence(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert res["init"]["ok"] and res["after_step"]["ok"], res
        assert not res["master"]["ok"] and res["master"]["fields"][:1] == ["master"], res
        assert res["resynced"]["ok"], res
        assert res["momentum"]["fields"] == ["momentum"], res
        assert res["buffers"]["fields"] == ["buffers"], res
        assert res["raised"] and "diverged at epoch 1" in res["raised"], res
        assert not res["swap"]["ok"] and "master64" in res["swap"]["fields"], res


def test_single_process_is_trivially_consistent():
    from simclr_amd.models import ContrastiveModel
    from simclr_amd.parallel import invariant as inv
    from simclr_amd.parallel import state as pstate
    from simclr_amd.parallel.flat import FlatParamStore
    pstate.reset()
    m = ContrastiveModel("resnet18", d=16)
    store = FlatParamStore(m, "cpu", shadow_dtype=None)
    fp = inv.fingerprint(store)
    assert fp.dtype == torch.int64 and fp.numel() == len(inv.FIELDS)
    assert inv.check_replicas(store)["ok"]
    with torch.no_grad():
        store.master[7] += 1.0
    assert not torch.equal(inv.fingerprint(store), fp)
