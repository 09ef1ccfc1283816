"""NT-Xent oracle vs the reference formulation; data sharding and augmentation properties."""
import numpy as np
import pytest
import torch
from torch.utils.data.distributed import DistributedSampler

from bench.torch_reference import nt_xent_reference
from simclr_amd.data import augment_ref
from simclr_amd.data.datasets import synthetic_dataset, load_dataset
from simclr_amd.data.loader import ContrastiveLoader, shard_indices
from simclr_amd.loss.ntxent import NTXent, nt_xent_torch


@pytest.mark.parametrize("n,tau", [(8, 0.5), (33, 0.1), (5, 1.0)])
def test_ntxent_equals_reference(n, tau):
    torch.manual_seed(n)
    v0 = torch.randn(n, 16, dtype=torch.float64, requires_grad=True)
    v1 = torch.randn(n, 16, dtype=torch.float64, requires_grad=True)
    a = NTXent(tau)(v0, v1)
    b = nt_xent_reference(v0, v1, tau)
    assert torch.allclose(a.double(), b, rtol=1e-6)
    ga = torch.autograd.grad(a, [v0, v1])
    gb = torch.autograd.grad(b, [v0, v1])
    for x, y in zip(ga, gb):
        assert torch.allclose(x.double(), y, rtol=1e-5, atol=1e-8)


def test_ntxent_reductions():
    torch.manual_seed(0)
    v0, v1 = torch.randn(6, 8), torch.randn(6, 8)
    none = NTXent(0.5, reduction="none")(v0, v1)
    assert none.shape == (2, 6)
    assert torch.allclose(NTXent(0.5, reduction="sum")(v0, v1), none.sum())
    assert torch.allclose(NTXent(0.5)(v0, v1), none.mean())


def test_shard_indices_match_distributed_sampler():
    class DS:
        def __len__(self):
            return 103
    for world in (1, 2, 4):
        for rank in range(world):
            s = DistributedSampler(DS(), num_replicas=world, rank=rank, shuffle=True, seed=0)
            s.set_epoch(5)
            assert list(s) == shard_indices(103, 5, rank, world).tolist()


def test_augment_params_distribution():
    rng_flips = rng_gray = rng_jit = 0
    N = 2000
    for i in range(N):
        P = augment_ref.sample_params(augment_ref.Rng(augment_ref.image_key(7, 1, 0, i)), 32, 32,
                                      0.5)
        assert 1 <= P["ch"] <= 32 and 1 <= P["cw"] <= 32
        assert 0 <= P["ci"] <= 32 - P["ch"] and 0 <= P["cj"] <= 32 - P["cw"]
        assert 0.6 <= P["fb"] <= 1.4 and -0.1 <= P["fh"] <= 0.1
        assert sorted(P["order"]) == [0, 1, 2, 3]
        rng_flips += P["flip"]
        rng_gray += P["gray"]
        rng_jit += P["jitter"]
    assert abs(rng_flips / N - 0.5) < 0.05
    assert abs(rng_gray / N - 0.2) < 0.04
    assert abs(rng_jit / N - 0.8) < 0.04


def test_augment_output_and_views_differ():
    ds = synthetic_dataset(16, 10, seed=3)
    ld = ContrastiveLoader(ds, 8, torch.device("cpu"), seed=7, views=2)
    x, y = next(iter(ld))
    assert x.shape == (16, 3, 32, 32) and y.shape == (8,)
    assert float(x.min()) >= 0.0 and float(x.max()) <= 1.0
    assert not torch.allclose(x[:8], x[8:])
    plain = augment_ref.augment_batch(ds.images, np.arange(2), 1, 32, 32, 0.5, 0, 0, augment=False)
    assert np.allclose(plain[0].transpose(1, 2, 0) * 255, ds.images[0])


def test_cifar_binary_reader(tmp_path):
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    rng = np.random.default_rng(0)
    for name in [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]:
        rec = np.concatenate([rng.integers(0, 10, (4, 1)), rng.integers(0, 256, (4, 3072))], 1)
        rec.astype(np.uint8).tofile(d / name)
    tr = load_dataset("cifar10", train=True, root=str(tmp_path))
    assert tr.images.shape == (20, 32, 32, 3) and tr.labels.shape == (20,)
    te = load_dataset("cifar10", train=False, root=str(tmp_path))
    assert len(te) == 4
    with pytest.raises(FileNotFoundError):
        load_dataset("cifar100", root=str(tmp_path))


def test_ce_rank_fallback_nan_matches_topk():
    from simclr_amd.ops.classify import ce_rank
    torch.manual_seed(3)
    B, C = 128, 10
    z = torch.randn(B, C)
    y = torch.randint(0, C, (B,))
    z[:32] = float("nan")
    z[32:64, 3] = float("nan")
    z[64:80].scatter_(1, y[64:80, None], float("nan"))
    _, rank = ce_rank(z, y)
    nan_t = torch.isnan(z.gather(1, y[:, None])).view(-1)
    assert bool((rank[nan_t] == C).all())  # topk may pick a NaN target: we never count it
    for k in (1, 5):
        ref = (torch.topk(z, k, dim=1)[1] == y[:, None]).any(1)
        assert torch.equal((rank < k)[~nan_t], ref[~nan_t]), k
