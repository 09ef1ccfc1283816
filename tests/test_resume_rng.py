"""Resume restores the random generators (torch host / device, NumPy) saved with the optimizer
state, so the draws after a resume continue the interrupted run's sequence (an extension: the
reference saves weights only, /root/reference/main.py:129-131).  Also: the attribution knobs
that drop gradients are refused by the training entry points."""
import numpy as np
import pytest
import torch

from simclr_amd.models.contrastive import ContrastiveModel
from simclr_amd.utils.checkpoint import load_resume, save_resume


def test_resume_restores_rng(tmp_path):
    m = ContrastiveModel("resnet18")
    torch.manual_seed(5)
    np.random.seed(5)
    torch.rand(3)
    np.random.rand(2)
    path = str(tmp_path / "resume-1.pt")
    save_resume(path, m, None, epoch=1, step=10)
    want_t, want_n = torch.rand(4), np.random.rand(4)
    torch.manual_seed(123)
    np.random.seed(123)
    blob = load_resume(path, m)
    assert blob["epoch"] == 1 and blob["step"] == 10
    assert torch.equal(torch.rand(4), want_t)
    assert np.array_equal(np.random.rand(4), want_n)


def _rank_rng_worker(rank, world, port, path):
    import os
    import torch.distributed as dist
    from simclr_amd.utils.checkpoint import gather_rng_states, restore_rng
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)  # every rank's generators differ
    np.random.seed(100 + rank)
    if rank == 0:
        save_resume(path, ContrastiveModel("resnet18"), None, epoch=1, step=3,
                    group=dist.group.WORLD)
    else:
        gather_rng_states(0, dist.group.WORLD)
    want_t, want_n = torch.rand(4), np.random.rand(4)
    dist.barrier()
    torch.manual_seed(7)
    np.random.seed(7)
    restore_rng(torch.load(path, weights_only=True))
    ok = torch.equal(torch.rand(4), want_t) and np.array_equal(np.random.rand(4), want_n)
    with open(f"{path}.{rank}", "w") as f:
        f.write("ok" if ok else "mismatch")
    dist.destroy_process_group()


def test_resume_restores_each_ranks_own_rng(tmp_path):
    """Rank 0 writes the resume file, but every rank gets ITS OWN generators back (gathered at
    save time, indexed by rank), not rank 0's copy."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    path = str(tmp_path / "resume-1.pt")
    mp.spawn(_rank_rng_worker, args=(2, port, path), nprocs=2, join=True)
    assert [open(f"{path}.{r}").read() for r in range(2)] == ["ok", "ok"]


@pytest.mark.parametrize("knob", ["SIMCLR_SKIP_WGRAD"])
def test_training_refuses_attribution_knobs(monkeypatch, knob):
    from simclr_amd.train.pretrain import pretrain
    from simclr_amd.train.supervised import supervised
    monkeypatch.setenv(knob, "1")
    for fn in (pretrain, supervised):
        with pytest.raises(RuntimeError, match=knob):
            fn({})


def test_restore_rng_legacy_device_state(monkeypatch, caplog):
    """Resume files written before the per-rank entries keep the device generators as a
    top-level ``cuda_rng`` list: the current device's entry is restored from it; a file with no
    device state at all logs a warning instead of silently skipping the restore."""
    from simclr_amd.utils import checkpoint as ck
    seen = []
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 1)
    monkeypatch.setattr(torch.cuda, "set_rng_state", lambda s: seen.append(s))
    st = [torch.zeros(4, dtype=torch.uint8), torch.ones(4, dtype=torch.uint8)]
    ck.restore_rng({"torch_rng": torch.get_rng_state(), "cuda_rng": st}, rank=0)
    assert len(seen) == 1 and torch.equal(seen[0], st[1])
    with caplog.at_level("WARNING"):
        ck.restore_rng({"torch_rng": torch.get_rng_state()}, rank=0)
    assert len(seen) == 1 and "NOT restored" in caplog.text
