"""Fused projection head (models/head_fused.py) against a plain fp32 torch
``Linear → BatchNorm1d (train, per view) → ReLU → Linear`` — forward, every gradient and the
running statistics, two view segments — and its launch count against the per-op path."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _head(H, D, nonlinear=False):
    from simclr_amd.models.heads import NonLinearClassifier, ProjectionHead
    torch.manual_seed(3)
    m = (NonLinearClassifier(H, D) if nonlinear else ProjectionHead(H, D)).to(DEV)
    with torch.no_grad():  # bf16-representable weights: the fp32 reference sees the same values
        for p in m.parameters():
            p.copy_(p.to(torch.bfloat16).float())
        s = m._seq
        s.bn1.weight.uniform_(0.5, 1.5)
        s.bn1.bias.normal_(0.0, 0.3)
    m.train()
    return m


def _reference(m, x, R, S):
    """fp32 torch ops, SyncBN-per-view semantics (reference model.py:56-73, main.py:112-113)."""
    s = m._seq
    W1 = s.linear1.weight.detach().clone().requires_grad_()
    b1 = s.linear1.bias.detach().clone().requires_grad_()
    g = s.bn1.weight.detach().clone().requires_grad_()
    b = s.bn1.bias.detach().clone().requires_grad_()
    W2 = s.linear2.weight.detach().clone().requires_grad_()
    b2 = (s.linear2.bias.detach().clone().requires_grad_() if s.linear2.bias is not None
          else None)
    xf = x.detach().float().requires_grad_()
    y1 = xf @ W1.t() + b1
    n = x.shape[0] // S
    ys, means, vars_ = [], [], []
    for k in range(S):
        yk = y1[k * n:(k + 1) * n]
        mu = yk.mean(0)
        var = yk.var(0, unbiased=False)
        ys.append((yk - mu) / torch.sqrt(var + s.bn1.eps) * g + b)
        means.append(mu.detach())
        vars_.append(var.detach() * n / (n - 1))
    h = torch.relu(torch.cat(ys))
    z = h @ W2.t() + (b2 if b2 is not None else 0.0)
    (z * R).sum().backward()
    rm, rv = torch.zeros_like(means[0]), torch.ones_like(vars_[0])
    for mu, v in zip(means, vars_):
        rm = 0.9 * rm + 0.1 * mu
        rv = 0.9 * rv + 0.1 * v
    grads = {"linear1.weight": W1.grad, "linear1.bias": b1.grad, "bn1.weight": g.grad,
             "bn1.bias": b.grad, "linear2.weight": W2.grad}
    if b2 is not None:
        grads["linear2.bias"] = b2.grad
    return z.detach(), xf.grad, grads, rm, rv


@pytest.mark.parametrize("H,D,nonlinear", [(2048, 128, False), (512, 128, False),
                                            (128, 64, True)])
def test_fused_head_matches_fp32(H, D, nonlinear):
    from simclr_amd.models import head_fused
    from simclr_amd.parallel import state as pstate
    pstate.reset()
    S, n = 2, 256
    m = _head(H, D, nonlinear)
    torch.manual_seed(4)
    x = torch.randn(S * n, H, device=DEV).to(torch.bfloat16).requires_grad_()
    R = torch.randn(S * n, D, device=DEV) / math.sqrt(S * n)
    assert head_fused.eligible(m, x, S)
    z_ref, dx_ref, g_ref, rm_ref, rv_ref = _reference(m, x, R, S)
    z = m(x, segments=S)
    assert z.dtype == torch.bfloat16 and z.grad_fn is not None
    assert type(z.grad_fn).__name__.startswith("MLPHeadFn"), "fused head did not run"
    (z.float() * R).sum().backward()
    torch.cuda.synchronize()
    s = m._seq
    assert _rel(z, z_ref) < 1e-2
    assert _rel(x.grad, dx_ref) < 2e-2
    got = {"linear1.weight": s.linear1.weight.grad, "bn1.weight": s.bn1.weight.grad,
           "bn1.bias": s.bn1.bias.grad, "linear2.weight": s.linear2.weight.grad}
    if nonlinear:
        got["linear2.bias"] = s.linear2.bias.grad
    for k, v in got.items():
        assert v is not None, k
        assert _rel(v, g_ref[k]) < 2e-2, (k, _rel(v, g_ref[k]))
    # b1 in front of a BatchNorm: the exact gradient is 0 (the fp32 reference's is round-off)
    assert bool((s.linear1.bias.grad == 0).all())
    assert g_ref["linear1.bias"].abs().max().item() < 1e-3 * g_ref["linear1.weight"].abs().max().item()
    assert _rel(s.bn1.running_mean, rm_ref) < 3e-3 and _rel(s.bn1.running_var, rv_ref) < 3e-3
    assert int(s.bn1.num_batches_tracked) == S


def _head_kernels(m, x, R, S, fused):
    """Kernel launches of one head forward + backward (a captured graph's kernel nodes)."""
    from simclr_amd.runtime.graph_exec import StreamReplay
    m.use_fused = fused
    R16 = R.to(torch.bfloat16)
    for _ in range(2):  # eager: autotune, plans
        x.grad = None
        m(x, segments=S).backward(R16)
    torch.cuda.synchronize()
    x.grad = None
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        m(x, segments=S).backward(R16)
    g.instantiate()
    st = StreamReplay(g, max_streams=1).stats()
    g.replay()
    torch.cuda.synchronize()
    return st["kernels"] + st["subgraphs"] + st["memsets"]


def test_fused_head_cuts_launches():
    """The fused head (K6) issues at most 60 % of the kernels of the per-op head path for the
    same forward + backward (bound to a flat parameter store, as in training).  Measured on
    MI355X: 10 vs 17 (forward: GEMM, finalize, split-K GEMM + its ordered reduction, one
    batched weight transpose; backward: dgrad + mask/partials, one-split weight gradient,
    finalize, dgrad with the BN-backward prologue, one-split weight gradient)."""
    from simclr_amd.parallel import state as pstate
    from simclr_amd.parallel.flat import FlatParamStore
    pstate.reset()
    pstate.get().device = torch.device(DEV, 0)
    S, n, H, D = 2, 256, 2048, 128
    m = _head(H, D)
    FlatParamStore(m, torch.device(DEV, 0), shadow_dtype=torch.bfloat16)
    x = torch.randn(S * n, H, device=DEV).to(torch.bfloat16).requires_grad_()
    R = torch.randn(S * n, D, device=DEV)
    k_fused = _head_kernels(m, x, R, S, True)
    k_ops = _head_kernels(m, x, R, S, False)
    print("head kernels fused / per-op:", k_fused, k_ops)
    assert k_fused <= 10 and 10 * k_fused <= 6 * k_ops, (k_fused, k_ops)


def test_capture_without_warmup_skips_plan_build():
    """A graph capture that reaches the fused head before any eager step would have to build
    the weight-transpose plan inside the capture (a host-table upload recorded as a memcpy from
    a temporary host tensor).  The head then takes the per-op path for that capture; after an
    eager step has built the plan, a capture uses the fused head.  Both replays match an eager
    fused step on the same weights."""
    from simclr_amd.models import head_fused
    from simclr_amd.parallel import state as pstate
    from simclr_amd.parallel.flat import FlatParamStore
    pstate.reset()
    pstate.get().device = torch.device(DEV, 0)
    S, n, H, D = 2, 256, 2048, 128
    m = _head(H, D)
    store = FlatParamStore(m, torch.device(DEV, 0), shadow_dtype=torch.bfloat16)
    x = torch.randn(S * n, H, device=DEV).to(torch.bfloat16)
    assert head_fused.eligible(m, x, S) and not head_fused._plan_ready(m)
    names = []

    def run():
        z = m(x, segments=S)
        names.append(type(z.grad_fn).__name__)
        return z

    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        z_cap = run()
    g.instantiate()
    assert not names[-1].startswith("MLPHeadFn"), names
    assert "_head_wt" not in m.__dict__  # no plan was built inside the capture
    z_eager = run().detach().clone()  # eager: the fused head, builds the plan
    assert names[-1].startswith("MLPHeadFn") and head_fused._plan_ready(m)
    g.replay()
    torch.cuda.synchronize()
    assert _rel(z_cap, z_eager) < 1e-2
    g2 = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g2):
        z_cap2 = run()
    g2.instantiate()
    assert names[-1].startswith("MLPHeadFn")
    g2.replay()
    torch.cuda.synchronize()
    assert _rel(z_cap2, z_eager) < 1e-2
    del store


@pytest.mark.parametrize("M,K,N,ks,seg", [(1024, 2048, 128, 16, 512), (512, 1024, 64, 4, 256),
                                          (256, 512, 128, 2, 256)])
def test_gemm_splitk_matches_fp32(M, K, N, ks, seg):
    """The projection head's split-K GEMM 2 (misc.hip k_gemm_sk): relu(bn(y1)) · W2ᵀ + b2 with
    per-segment scale / shift, against fp32 torch on the same bf16 operands; and with no
    prologue; bitwise repeatable."""
    from simclr_amd.ops import _ext
    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    torch.manual_seed(M + K)
    S = M // seg
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
    sc = (0.5 + torch.rand(S, K, device=dev)).contiguous()
    sh = (torch.randn(S, K, device=dev) * 0.3).contiguous()
    bias = torch.randn(N, device=dev)
    part = torch.empty(ks * M * N, device=dev)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.gemm_sk(A, B, sc.view(-1), sh.view(-1), seg, ks, part, bias, out)
    sg = torch.arange(M, device=dev) // seg
    Ap = torch.relu(A.float() * sc[sg] + sh[sg]).to(torch.bfloat16).float()
    ref = Ap @ B.float().t() + bias
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 5e-3, err
    out2 = torch.empty_like(out)
    ops.gemm_sk(A, B, sc.view(-1), sh.view(-1), seg, ks, part, bias, out2)
    assert torch.equal(out, out2)
    ops.gemm_sk(A, B, None, None, seg, ks, part, None, out)
    ref = A.float() @ B.float().t()
    assert ((out.float() - ref).norm() / ref.norm()).item() < 5e-3

