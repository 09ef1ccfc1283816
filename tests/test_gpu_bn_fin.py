"""In-launch forward BatchNorm finalize (``csrc/conv.hip`` fin_publish / fin_tail, epilogue mode 6).

Every tile variant that admits it, on shapes that exercise one and several level-1 chunks per
XCD range, XCD ranges of unequal length (grid not a multiple of 8, fewer tiles than XCDs), a
partial last channel column and the BN-apply prologue: the conv output must be bitwise the plain
mode-0 output, and mean / invstd, scale / shift, running statistics and num_batches_tracked must
match a plain PyTorch fp32 reference computed from that output (the reference's BatchNorm2d
forward, /root/reference/model.py:76-114 via torchvision).  Two back-to-back launches per
variant check that the tagged-word arenas and tickets are left clean for the next launch."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from simclr_amd.ops import _ext
    _ext.require()
    o = torch.ops.simclr_amd
    o.bn_tickets_init(torch.empty(1, device=DEV))
    return o


def _bf(t):
    return t.to(torch.bfloat16)


# (images, H, Ci, Co, k, stride, pad, BN-apply prologue)
SHAPES = [
    (16, 16, 64, 256, 1, 1, 0, False),
    (16, 16, 64, 256, 1, 1, 0, True),
    (16, 16, 64, 64, 3, 1, 1, False),
    (16, 32, 64, 128, 3, 2, 1, False),
    (6, 16, 64, 64, 1, 1, 0, False),     # 6 tiles of 256 rows: fewer tiles than XCDs
    (18, 16, 64, 192, 1, 1, 0, False),   # uneven XCD ranges, partial last column
    (512, 32, 64, 64, 1, 1, 0, False),   # several level-1 chunks per (XCD, segment)
]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(str(v) for v in s))
def test_fin_matches_fp32_every_variant(ops, shape):
    from simclr_amd.ops.conv_hip import fwd_geom, igemm_launch
    Nb, H, Ci, Co, k, s, p, use_pro = shape
    S = 2
    torch.manual_seed(11)
    OH = (H + 2 * p - k) // s + 1
    M = Nb * OH * OH
    x = _bf(torch.randn(Nb, H, H, Ci, device=DEV))
    w = _bf(torch.randn(Co, k, k, Ci, device=DEV) / math.sqrt(Ci * k * k))
    g = fwd_geom(Nb, H, H, Ci, OH, OH, k, k, s, p, Co)
    pro = None
    if use_pro:
        sc = (torch.rand(S, Ci, device=DEV) + 0.5).contiguous()
        sh = (torch.randn(S, Ci, device=DEV) * 0.3).contiguous()
        pro = (sc.view(-1), sh.view(-1), M // S, True)
    gamma = torch.rand(Co, device=DEV) + 0.5
    beta = torch.randn(Co, device=DEV) * 0.1
    eps, mom = 1e-5, 0.1
    tested = 0
    for v in range(ops.igemm_nvariants()):
        if not ops.igemm_variant_ok(v, g, use_pro, False) or not ops.igemm_fin_ok(v, g, S):
            continue
        ref = torch.empty(Nb, OH, OH, Co, device=DEV, dtype=torch.bfloat16)
        igemm_launch(ops, x, w, ref, g, v, pro=pro)
        rm = torch.full((Co,), 0.1, device=DEV)
        rv = torch.ones(Co, device=DEV)
        nbt = torch.zeros((), device=DEV, dtype=torch.long)
        rm_ref, rv_ref = rm.clone(), rv.clone()
        for rep in range(2):
            out = torch.empty_like(ref)
            mi = torch.full((2 * S * Co,), float("nan"), device=DEV)
            ss = torch.full((2 * S * Co,), float("nan"), device=DEV)
            igemm_launch(ops, x, w, out, g, v, pro=pro,
                         fin={"mi": mi, "ss": ss, "rm": rm, "rv": rv, "nbt": nbt,
                              "gamma": gamma, "beta": beta, "count": float(M // S), "eps": eps,
                              "momentum": mom, "S": S, "slot": rep})
            torch.cuda.synchronize()
            assert ops.igemm_fin_err(out, rep) == 0, f"variant {v}: a poll timed out"
            assert torch.equal(out, ref), f"variant {v}: conv output differs from mode 0"
            a = out.float().view(S, -1, Co)
            mean = a.mean(1)
            var = a.var(1, unbiased=False)
            inv = torch.rsqrt(var + eps)
            got = mi.view(2, S, Co)
            tol = dict(rtol=2e-4, atol=2e-5)
            torch.testing.assert_close(got[0], mean, **tol, msg=f"variant {v} mean")
            torch.testing.assert_close(got[1], inv, rtol=1e-3, atol=1e-4, msg=f"variant {v} inv")
            sc_ref = gamma * inv
            sh_ref = beta - mean * sc_ref
            sg = ss.view(2, S, Co)
            torch.testing.assert_close(sg[0], sc_ref, rtol=1e-3, atol=1e-4)
            torch.testing.assert_close(sg[1], sh_ref, rtol=1e-3, atol=1e-3)
            n = float(M // S)
            for si in range(S):  # segment order, like the reference's two forward calls
                rm_ref = (1 - mom) * rm_ref + mom * mean[si]
                rv_ref = (1 - mom) * rv_ref + mom * var[si] * n / (n - 1)
            torch.testing.assert_close(rm, rm_ref, rtol=1e-4, atol=1e-5)
            torch.testing.assert_close(rv, rv_ref, rtol=1e-3, atol=1e-4)
            assert int(nbt) == S * (rep + 1)
        tested += 1
    assert tested > 0, "no variant admits the in-launch finalize on this shape"

