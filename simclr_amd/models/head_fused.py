"""Fused projection head: ``Linear(H,H)+b → BN1d → ReLU → Linear(H,d)`` as one
short launch sequence on the MFMA implicit-GEMM kernels, instead of a chain of per-op autograd
nodes (tests/test_gpu_head.py counts both).

Reference: ``ProjectionHead`` (``/root/reference/model.py:56-73``) with its BatchNorm1d converted
to SyncBatchNorm (main.py:176) and the two views run as separate forwards (main.py:112-113, so
the statistics are per view: SURVEY Q17).  Same math; what changes is where the BatchNorm work
runs (S = 2 view segments, statistics per segment, all-reduced across ranks)::

    forward   y1 = x·W1ᵀ + b1            GEMM 1, epilogue: bias + Σ, Σ² partials of y1
              finalize                   one launch: mean / invstd, running stats, scale/shift
                                         (the cross-GPU statistics combine happens here)
              z = relu(bn(y1))·W2ᵀ       GEMM 2, the BN + ReLU applied to its A operand in the
                                         prologue: relu(bn(y1)) is never written to HBM
              (+ the transposed weights W1ᵀ, W2ᵀ for the backward: one batched launch)
    backward  g = (dz·W2)·[bn(y1) > 0]   dgrad 2, epilogue: ReLU mask + Σg, Σg·x̂ partials
              dW2 = dzᵀ·relu(bn(y1))     weight gradient, the BN + ReLU in the X prologue, one
                                         split written straight into the flat gradient
              finalize                   dγ, dβ (flat gradient buffer) and the input-gradient
                                         coefficients; cross-GPU combine here
              dx = (A·g + B·y1 + D)·W1   dgrad 1, the BN backward in the A-operand prologue:
                                         the BN's input gradient is never written to HBM
              dW1 = (A·g + B·y1 + D)ᵀ·x  weight gradient, the same prologue on its dY operand
                                         (per-row view segment), one split, no reduction

The gradient of b1 is exactly zero: a bias in front of a BatchNorm cancels in (y − mean(y)),
so dL/db1 = Σ_rows dL/dy1 = 0 for every view over the global batch (the reference's autograd
produces that zero up to fp32 round-off; the data-parallel average of per-rank values is the
same zero).  Its slot in the flat gradient buffer is zeroed once and left alone.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import _ext
from ..ops.conv_hip import igemm_choose, igemm_launch
from ..parallel import state as pstate


def _geom(M, K, N):
    return [M, 1, 1, K, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, N, 1, 1, 1, 1, 0, 0, N]


def _w16(weight: torch.Tensor) -> torch.Tensor:
    slot = getattr(weight, "_slot", None)
    if slot is not None and slot.shadow is not None:
        return slot.shadow
    return weight.detach().to(torch.bfloat16).contiguous()


def _bnops():
    from .fused import FusedStages
    return FusedStages.__new__(FusedStages)  # the stateless BatchNorm helpers of the executor


def _wgrad_direct(ops, dY, X, out, geom, creal, pro=None, dpro=None):
    """Weight gradient in ONE split written straight into ``out`` (no split-reduction launch):
    the head's GEMMs have 1,024 rows, so the 128 x 128 output tiles already give up to 256
    blocks.  ``pro = (sc, sh, seg_rows, relu, S)``: X-operand BN + ReLU; ``dpro = (dY2, coef,
    seg_rows, S)``: dY-operand BatchNorm backward (register-staged variants, which take the
    per-row view segment)."""
    from ..ops import tuning
    psc, psh, pseg, prelu, pS = pro if pro is not None else (None, None, 0, False, 1)
    dY2, dcoef, dseg, dS = dpro if dpro is not None else (None, None, 0, 1)
    key = ("wgrad1split", tuple(geom), creal, psc is not None, dpro is not None)

    def launch(v, o):
        ops.wgrad(dY, X, o, o, geom, 1, creal, 0.0, psc, psh, pseg, prelu, pS, v, dY2, dcoef,
                  dseg, dS)

    v = tuning.cached(key)
    if v is None:
        cands = [v for v in range(ops.wgrad_nvariants())
                 if ops.wgrad_variant_ok(v, geom, psc is not None, dpro is not None)
                 and (dpro is None or not ops.wgrad_variant_glds(v))]
        v = tuning.pick(key, cands, 0, lambda vv: launch(vv, torch.empty_like(out)))
    launch(v, out)


def _deliver(param: torch.Tensor, compute) -> Optional[torch.Tensor]:
    """``compute(out)`` writes the fp32 gradient of ``param`` into its flat-store slot (and
    notifies the reducer); returns the gradient tensor for autograd when unbound."""
    slot = getattr(param, "_slot", None)
    if slot is not None:
        compute(slot.grad)
        slot.store.mark_ready(slot.index)
        return None
    g = torch.empty(param.shape, device=param.device, dtype=torch.float32)
    compute(g)
    return g


def eligible(mod, x: torch.Tensor, segments: int) -> bool:
    """bf16 GPU rows, per-view row counts that tile evenly (256-row BN-backward prologue tiles),
    and feature sizes the LDS-DMA tiles take (multiples of 64)."""
    s = mod._seq
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and mod.training):
        return False
    if not getattr(s.bn1, "training", True):
        return False
    M, K = x.shape
    H, D = s.linear1.out_features, s.linear2.out_features
    return (M % segments == 0 and (M // segments) % 256 == 0 and K % 64 == 0 and H % 64 == 0
            and D % 64 == 0 and s.linear1.bias is not None and s.linear2.in_features == H)


def _splitk_ok(M: int, H: int, D: int) -> bool:
    """GEMM 2 as the split-K kernel: 64-row / 64-column tiles, K / 128 >= 2 splits
    (``SIMCLR_HEAD_SPLITK=0`` keeps the implicit-GEMM launch, A/B)."""
    import os
    return (M % 64 == 0 and D % 64 == 0 and H % 128 == 0 and H >= 256
            and os.environ.get("SIMCLR_HEAD_SPLITK", "1") != "0")


def _pregather_ok(mod, st, S: int, seg: int, D: int) -> bool:
    """The NT-Xent with global negatives follows (``mod._zgather``, set by the trainer), over
    RCCL (the IPC exchange keeps its own one-shot gather in the loss), with one view per
    segment, and ``SIMCLR_ZGATHER_OVERLAP=1``.  Off by default, measured: GEMM 2 has only
    16-32 blocks and is bound by its 2,048-deep K loop, so each per-view launch takes as long
    as the one-launch GEMM 2 (39.4 vs 40 us): the split adds ~40 us to the critical path,
    more than the 256 KiB z exchange it hides (profiles/r6_optimization_log.md)."""
    import os
    return (getattr(mod, "_zgather", False) and st.comm and getattr(st, "ipc", None) is None
            and S == 2 and D in (32, 64, 128, 256) and (2 * seg) % 16 == 0
            and os.environ.get("SIMCLR_ZGATHER_OVERLAP", "0") == "1")


PREGATHER_CALLS = [0]  # launches of the per-view gather path (tests)


def _gemm2_pregather(ops, st, y1, W2, z, v2, bias2, bs, S: int, seg: int, H: int, D: int):
    """GEMM 2 view by view, each view's z all-gathered over RCCL on the loss's side stream
    while the next view's GEMM 2 runs (the north star's gather under the projection head).
    Same tile variant and per-row math as the one-launch GEMM 2, so z is bitwise the same; the
    gathered rows are assembled rank-major ([rank][view][row]), the layout the loss's
    one-shot all-gather produces, so the loss is bitwise the same too."""
    import torch.distributed as dist
    from ..loss import ntxent as ntx
    dev = z.device
    W = st.world_size
    cur = torch.cuda.current_stream(dev)
    side = ntx._side_stream(dev)
    parts = []
    splitk = _splitk_ok(S * seg, H, D)
    for v in range(S):
        rows = slice(v * seg, (v + 1) * seg)
        zv = z[rows]
        sc, sh = bs.ss[0][v * H:(v + 1) * H], bs.ss[1][v * H:(v + 1) * H]
        if splitk:  # the one-launch path's split-K kernel, per view: the same bits per row
            ks = H // 128
            p2 = torch.empty((ks * seg * D,), device=dev, dtype=torch.float32)
            ops.gemm_sk(y1[rows], W2.view(D, H), sc, sh, seg, ks, p2, bias2, zv)
        else:
            igemm_launch(ops, y1[rows], W2, zv, _geom(seg, H, D), v2, bias=bias2,
                         pro=(sc, sh, seg, True))
        tmp = torch.empty((W * seg, D), device=dev, dtype=torch.bfloat16)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            dist.all_gather_into_tensor(tmp, zv, group=st.group)
        parts.append(tmp)
    zb_all = torch.empty((W * S * seg, D), device=dev, dtype=torch.bfloat16)
    with torch.cuda.stream(side):
        za = zb_all.view(W, S, seg, D)
        for v in range(S):
            za[:, v].copy_(parts[v].view(W, seg, D))
    # every buffer the side stream touches stays referenced until the loss joins it
    ntx.register_pregather(z, zb_all, (parts, z))
    PREGATHER_CALLS[0] += 1


class MLPHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, gamma, beta, w2, b2, mod, S):
        ops = _ext.ops()
        st = pstate.get()
        s = mod._seq
        lin1, bn, lin2 = s.linear1, s.bn1, s.linear2
        M, K = x.shape
        H, D = lin1.out_features, lin2.out_features
        seg = M // S
        dev = x.device
        xc = x.contiguous()
        W1, W2 = _w16(lin1.weight), _w16(lin2.weight)
        # GEMM 1: bias + BatchNorm statistics partials
        y1 = torch.empty((M, H), device=dev, dtype=torch.bfloat16)
        g1 = _geom(M, K, H)
        bias1 = b1.detach().float().contiguous()
        v = igemm_choose(ops, xc, W1, y1, g1, bias=bias1, want_stats=True, seg_rows=seg)
        bm = ops.igemm_variant_bm(v)
        part = torch.empty(((M // bm) * 2 * H,), device=dev, dtype=torch.float32)
        igemm_launch(ops, xc, W1, y1, g1, v, bias=bias1, stats=part)
        bs = _bnops()._bn_fwd(ops, bn, part, seg // bm, seg, S, st)
        # GEMM 2 on relu(bn(y1)) formed in the operand prologue
        z = torch.empty((M, D), device=dev, dtype=torch.bfloat16)
        g2 = _geom(M, H, D)
        pro = (bs.ss[0], bs.ss[1], seg, True)
        bias2 = b2.detach().float().contiguous() if b2 is not None else None
        v2 = igemm_choose(ops, y1, W2, z, g2, bias=bias2, pro=pro, seg_rows=seg)
        if _pregather_ok(mod, st, S, seg, D):
            _gemm2_pregather(ops, st, y1, W2, z, v2, bias2, bs, S, seg, H, D)
        elif _splitk_ok(M, H, D):
            # split-K GEMM 2 (misc.hip k_gemm_sk): K / 128 splits, fixed-order reduction
            ks = H // 128
            part2 = torch.empty((ks * M * D,), device=dev, dtype=torch.float32)
            ops.gemm_sk(y1, W2.view(D, H), bs.ss[0], bs.ss[1], seg, ks, part2, bias2, z)
        else:
            igemm_launch(ops, y1, W2, z, g2, v2, bias=bias2, pro=pro)
        # the backward's transposed weights, one batched launch (weights are final until the
        # optimizer step, which comes after the backward)
        wt1, wt2 = _transposed(ops, mod, W1, W2, K, H, D)
        ctx.save_for_backward(xc, y1)
        ctx.bs = bs
        ctx.mod = mod
        ctx.wts = (wt1, wt2)
        ctx.S = S
        ctx.has_b2 = b2 is not None
        return z

    @staticmethod
    def backward(ctx, dz):
        ops = _ext.ops()
        st = pstate.get()
        xc, y1 = ctx.saved_tensors
        bs, mod, S = ctx.bs, ctx.mod, ctx.S
        wt1, wt2 = ctx.wts
        s = mod._seq
        lin1, bn, lin2 = s.linear1, s.bn1, s.linear2
        M, K = xc.shape
        H, D = lin1.out_features, lin2.out_features
        seg = M // S
        dev = dz.device
        dzc = dz.contiguous()
        if dzc.dtype != torch.bfloat16:
            dzc = dzc.to(torch.bfloat16)
        bnx = _bnops()
        # dgrad 2: g = (dz·W2)·[bn(y1) > 0] with the BN-backward partials Σg, Σg·x̂
        gm = torch.empty((M, H), device=dev, dtype=torch.bfloat16)
        gd = _geom(M, D, H)
        epi = (3, None, y1)
        tables = (bs.ss.view(-1), bs.mi)
        v = igemm_choose(ops, dzc, wt2, gm, gd, want_stats=True, epi=epi, seg_rows=seg,
                         epi_tables=tables)
        nb = seg // ops.igemm_variant_bm(v)
        part = torch.empty((S * nb * 2 * H,), device=dev, dtype=torch.float32)
        igemm_launch(ops, dzc, wt2, gm, gd, v, stats=part, epi=epi, seg_rows=seg,
                     epi_tables=tables, remap=(nb, 0))
        h = bnx._bn_bwd_start(ops, bn, part, nb, bs, S, st)
        # dW2 = dzᵀ · relu(bn(y1)) (X prologue), independent of the BN backward
        pro = (bs.ss[0], bs.ss[1], seg, True, S)
        gw2 = _deliver(lin2.weight, lambda o: _wgrad_direct(ops, dzc, y1, o.view(D, 1, 1, H),
                                                            _geom(M, H, D), H, pro=pro))
        gb2 = None
        if ctx.has_b2:
            gb2 = _deliver(lin2.bias, lambda o: ops.colsum(dzc, o, 0.0))
        coef = bnx._bn_bwd_finish(ops, h, S)
        # dgrad 1 with the BN backward da = A·g + B·y1 + D in the A-operand prologue
        SC = S * H
        bpro = (coef[:SC], coef[SC:2 * SC], coef[2 * SC:], seg, y1)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((M, K), device=dev, dtype=torch.bfloat16)
            gx = _geom(M, H, K)
            v = igemm_choose(ops, gm, wt1, dx, gx, bnb=bpro)
            igemm_launch(ops, gm, wt1, dx, gx, v, bnb=bpro)
        # dW1 = daᵀ · x, the same prologue on the dY operand
        gw1 = _deliver(lin1.weight, lambda o: _wgrad_direct(ops, gm, xc, o.view(H, 1, 1, K),
                                                            _geom(M, K, H), K,
                                                            dpro=(y1, coef, seg, S)))
        gb1 = _zero_bias_grad(mod, lin1.bias)
        return dx, gw1, gb1, None, None, gw2, gb2, None, None


def _zero_bias_grad(mod, bias: torch.Tensor) -> Optional[torch.Tensor]:
    slot = getattr(bias, "_slot", None)
    if slot is None:
        return torch.zeros(bias.shape, device=bias.device, dtype=torch.float32)
    done = mod.__dict__.setdefault("_zeroed_slots", {})
    key = (id(slot.store), slot.index)
    if done.get(key) != slot.grad.data_ptr():
        slot.grad.zero_()  # once per buffer: nothing else ever writes this slot
        done[key] = slot.grad.data_ptr()
    slot.store.mark_ready(slot.index)
    return None


def _transposed(ops, mod, W1, W2, K, H, D):
    """W1ᵀ [K][H] and W2ᵀ [H][D] (the dgrads' B operands) in one batched launch; the plan is
    rebuilt when the bf16 weights move (never during a graph capture: the first eager step
    builds it)."""
    sig = (W1.data_ptr(), W2.data_ptr(), K, H, D)
    cache = mod.__dict__.get("_head_wt")
    if cache is None or cache[0] != sig:
        dev = W1.device
        wt1 = torch.empty((K, 1, 1, H), device=dev, dtype=torch.bfloat16)
        wt2 = torch.empty((H, 1, 1, D), device=dev, dtype=torch.bfloat16)
        params = [H, 1, 1, K, 1, 1, 0, 1, 0, 1, D, 1, 1, H, 1, 1, 0, 1, 0, 1]
        plan = ops.weight_transform_plan([W1, W2], [wt1, wt2], params)
        cache = (sig, plan[:-1].to(dev), int(plan[-1]), wt1, wt2, (W1, W2))
        mod.__dict__["_head_wt"] = cache
    ops.weight_transform_batch(cache[1], cache[2])
    return cache[3].view(K, H), cache[4].view(H, D)


def _plan_ready(mod) -> bool:
    """True when the cached transpose plan (``_transposed``) matches the current bf16 weights.
    Building a plan uploads a host table; inside a graph capture that upload would become a
    memcpy node reading a temporary host tensor freed when the capture ends."""
    s = mod._seq
    cache = mod.__dict__.get("_head_wt")
    if cache is None:
        return False
    slots = [getattr(w, "_slot", None) for w in (s.linear1.weight, s.linear2.weight)]
    if any(sl is None or sl.shadow is None for sl in slots):
        return False  # unbound weights get a fresh bf16 copy (a new pointer) per call
    return cache[0][:2] == (slots[0].shadow.data_ptr(), slots[1].shadow.data_ptr())


def fused_mlp(mod, x: torch.Tensor, segments: int) -> Optional[torch.Tensor]:
    """The fused head's output, or None when the shapes / mode are not eligible, or when a
    graph capture would have to build the weight-transpose plan (the per-op head then runs
    inside the capture; an eager step before the capture builds the plan)."""
    if not eligible(mod, x, segments):
        return None
    if torch.cuda.is_current_stream_capturing() and not _plan_ready(mod):
        return None
    _ext.require()
    s = mod._seq
    return MLPHeadFn.apply(x, s.linear1.weight, s.linear1.bias, s.bn1.weight, s.bn1.bias,
                           s.linear2.weight, s.linear2.bias, mod, segments)
