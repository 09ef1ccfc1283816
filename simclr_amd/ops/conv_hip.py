"""Autograd wrapper of the implicit-GEMM conv kernels (``csrc/conv.hip``).

Tensors: activations are logical NCHW / physical NHWC (``channels_last``) bf16; weights are
consumed as OHWI bf16 (the flat store's shadow) and their gradients are produced as OHWI fp32
directly into the flat gradient buffer.

Pass decomposition (all on ``igemm_nt`` / ``wgrad_tn``):

* forward   : gather x with (stride s, pad p); epilogue also emits per-channel Σy, Σy² block
              partials that the following BatchNorm consumes instead of re-reading y.
* dgrad s=1 : dx = conv(dy, flip(W)ᵀ) — gather dy with offset −(K−1−p), B = weight_transform
              (W[co][K−1−kh][K−1−kw][ci] → [ci][kh][kw][co]).
* dgrad s=2 : per output parity class (r, c) ∈ {0,1}²: the taps kh ≡ r+p (mod 2) form a
              stride-1 sub-convolution with negative tap step (dh = −1) whose outputs land on
              rows 2i+r, cols 2j+c (strided epilogue).  No zero-inserted MACs.
* wgrad     : dW[co][kh][kw][ci] = Σ_m dy[m][co] · im2col(x)[m][(kh,kw,ci)], split over m.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from . import _ext, tuning


def igemm_choose(ops, A, B, out, geom, bias=None, want_stats=False, pro=None, epi=None,
                 seg_rows: int = 0, epi_tables=None, bnb=None, dual=None,
                 patch_only: bool = False) -> int:
    """Autotuned tile variant for this problem (admissible: BM divides the segment rows /
    M whenever per-segment prologue, statistics or the mode-3 epilogue need block-uniform
    segments).  ``dual = (res, rss, out, mask)``: block-output prologue (see igemm_launch)."""
    M = geom[0] * geom[4] * geom[5]
    N = geom[14]
    psc, psh, pseg, prelu = pro if pro is not None else (None, None, 0, False)
    pd, A2 = None, None
    if bnb is not None:  # BN-backward prologue: a = coefA·A + coefB·A2 + coefD
        psc, psh, pd, pseg, A2 = bnb
    rss, pout, pmask = None, None, None
    if dual is not None:
        A2, rss, pout, pmask = dual
    emode, ea, eb = epi[:3] if epi is not None else (0, None, None)
    ess, emi = epi_tables if epi_tables is not None else (None, None)
    key = ("igemm", tuple(geom), want_stats, psc is not None, emode, bias is not None, seg_rows,
           bnb is not None, dual is not None, patch_only)
    hit = tuning.cached(key)
    if hit is not None:  # steady state: no per-launch walk over the variant table
        return hit
    cands = []
    for v in range(ops.igemm_nvariants()):
        bm = ops.igemm_variant_bm(v)
        if dual is not None:
            if not ops.igemm_dual_ok(v, geom):
                continue
        elif not ops.igemm_variant_ok(v, geom, psc is not None, bnb is not None):
            continue  # e.g. LDS-DMA variants: C % 64 == 0, BN-apply prologue only on 1x1
        if (bnb is not None and emode & 255 == 4 and ops.igemm_variant_glds(v)
                and bm * ops.igemm_variant_bn(v) > 256 * 128):
            continue  # BN-backward prologue + mode-4 epilogue: not instantiated at 256 x 256
        if want_stats and M % bm:
            continue
        if psc is not None and pseg % bm:
            continue
        if seg_rows and seg_rows % bm:
            continue
        if patch_only and not ops.igemm_variant_patch(v):
            continue  # (the materialised BN-backward operand exists only in the patch kernel)
        cands.append(v)
    if not cands:
        raise ValueError(f"no igemm tile variant admissible for M={M} segment rows "
                         f"{seg_rows or pseg}")
    default = 1 if N <= 64 else 0
    if default not in cands:
        default = cands[0]
    ec = epi[3] if epi is not None and len(epi) > 3 else None
    em = epi[4] if epi is not None and len(epi) > 4 else None

    def trial(v):
        bm = ops.igemm_variant_bm(v)
        st = (torch.empty(((M + bm - 1) // bm) * 2 * N, device=out.device, dtype=torch.float32)
              if want_stats else None)
        # every output of a trial is scratch (tuning.py: trials touch no live tensor), the
        # block-output prologue's out / mask included
        tout = torch.empty_like(pout) if pout is not None else None
        tmask = torch.empty_like(pmask) if pmask is not None else None
        ops.igemm(A, B, torch.empty_like(out), bias, st, geom, psc, psh, pseg, prelu, emode, ea,
                  eb, v, ess, emi, seg_rows, 0, 0, ec, em, None, None, None, pd, A2, rss, tout,
                  tmask)

    return tuning.pick(key, cands, default, trial)


def igemm_launch(ops, A, B, out, geom, v, bias=None, stats=None, pro=None, epi=None,
                 seg_rows: int = 0, epi_tables=None, remap=(0, 0), second=None,
                 bnb=None, dual=None, bnb_out=None) -> None:
    """``second = (c2, mi2, stats2)``: mode-4 second BatchNorm stream (see conv.hip);
    ``bnb = (coefA, coefB, coefD, seg_rows, A2)``: BatchNorm-backward A-operand prologue;
    ``dual = (res, rss, out, mask)``: block-output prologue — A is a block's pre-BN conv3
    activation, ``pro`` its BN scale/shift, ``res`` the residual (``rss`` its BN [2][S][C] table
    or None for identity); the conv consumes relu(bn(A) + res') and also writes it to ``out``
    with its ReLU bitmask ``mask``.  ``bnb_out``: with ``bnb`` on a patch variant, the
    BatchNorm-backward operand is also written there (the weight gradient's dY)."""
    psc, psh, pseg, prelu = pro if pro is not None else (None, None, 0, False)
    pd, A2 = None, None
    if bnb is not None:
        psc, psh, pd, pseg, A2 = bnb
    rss, pout, pmask = None, None, None
    if dual is not None:
        A2, rss, pout, pmask = dual
    if bnb_out is not None:  # patch kernels: the BN-backward operand also stored (wgrad's dY)
        pout = bnb_out
    emode, ea, eb = epi[:3] if epi is not None else (0, None, None)
    ec = epi[3] if epi is not None and len(epi) > 3 else None
    em = epi[4] if epi is not None and len(epi) > 4 else None
    ess, emi = epi_tables if epi_tables is not None else (None, None)
    c2, mi2, st2 = second if second is not None else (None, None, None)
    ops.igemm(A, B, out, bias, stats, geom, psc, psh, pseg, prelu, emode, ea, eb, v, ess, emi,
              seg_rows, remap[0], remap[1], ec, em, c2, mi2, st2, pd, A2, rss, pout, pmask)


def run_igemm(ops, A, B, out, geom, bias=None, want_stats=False, pro=None, epi=None):
    """Launch the implicit GEMM with the autotuned tile variant for this problem.

    pro = (scale[S][C], shift[S][C], rows_per_segment, relu) applies the previous BatchNorm on the
    A operand; epi = (mode, a, b) accumulates into the output.  Returns (stats, nblk) or None."""
    M = geom[0] * geom[4] * geom[5]
    N = geom[14]
    try:
        v = igemm_choose(ops, A, B, out, geom, bias, want_stats, pro, epi)
    except ValueError:
        if pro is not None:
            raise ValueError("BN prologue fusion impossible for this shape")
        want_stats = False
        v = igemm_choose(ops, A, B, out, geom, bias, False, pro, epi)
    bm = ops.igemm_variant_bm(v)
    stats = None
    if want_stats:
        stats = torch.empty(((M // bm) * 2 * N,), device=out.device, dtype=torch.float32)
    igemm_launch(ops, A, B, out, geom, v, bias, stats, pro, epi)
    return (stats, M // bm) if stats is not None else None




# weight gradients issued beside the dgrad / BatchNorm chain (the fused executor's side stream)
# skip the 256 x 256 output tiles: the autotuner times candidates alone, where those tiles win,
# but their 128 KB of LDS per block keeps every chain block off the CU; under the concurrent
# step the best <= 256 x 128 tile is 0.17 ms/step faster (4 of 4 interleaved A/B rounds,
# profiles/r5_optimization_log.md)
CONCURRENT_MAX_TILE = 256 * 128


def run_wgrad(ops, dY, X, out, geom, creal, pro=None, dpro=None, concurrent: bool = False):
    """Split-M weight gradient (fp32, written to ``out`` = OHWI) with the autotuned variant.

    ``dpro = (dY2, coef[3][S][N], seg_rows, S)``: the dY operand is the BatchNorm backward
    A·dY + B·dY2 + D computed on the fly (splits are aligned to the segments).
    ``concurrent``: the kernel runs beside the critical chain (``CONCURRENT_MAX_TILE``)."""
    psc, psh, seg_rows, prelu, pS = pro if pro is not None else (None, None, 0, False, 1)
    dY2, dcoef, dseg, dS = dpro if dpro is not None else (None, None, 0, 1)
    N = geom[14]
    K = geom[6] * geom[7] * geom[3]
    M = geom[0] * geom[4] * geom[5]
    key = ("wgrad", tuple(geom), creal, psc is not None, dpro is not None, concurrent)

    def nsplit(v):
        splits = ops.wgrad_splits(geom, v)
        if dpro is None:
            return splits
        seg_iters = dseg // 64
        sps = max(1, splits // dS)
        while seg_iters % sps:
            sps -= 1
        return dS * sps

    def launch(v, o, trial=False):
        splits = nsplit(v)
        partial = torch.empty((splits * N * K,), device=dY.device, dtype=torch.float32)
        ops.wgrad(dY, X, partial, o, geom, splits, creal, 0.0, psc, psh, seg_rows, prelu, pS, v,
                  dY2, dcoef, dseg, dS)

    v = tuning.cached(key)
    if v is None:
        cands = [v for v in range(ops.wgrad_nvariants())
                 if ops.wgrad_variant_ok(v, geom, psc is not None, dpro is not None)]
        if concurrent:
            cands = [c for c in cands
                     if ops.wgrad_variant_area(c) <= CONCURRENT_MAX_TILE] or cands
        v = tuning.pick(key, cands, 1 if N <= 64 else 0,
                        lambda vv: launch(vv, torch.empty_like(out), trial=True))
    launch(v, out)


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    """Contiguous NHWC view of a channels_last 4-D tensor (copies only if needed)."""
    if t.dim() == 4:
        if not t.is_contiguous(memory_format=torch.channels_last):
            t = t.contiguous(memory_format=torch.channels_last)
        return t.permute(0, 2, 3, 1)
    return t.contiguous()


def _empty_cl(n, c, h, w, device, dtype=torch.bfloat16):
    return torch.empty((n, c, h, w), device=device, dtype=dtype,
                       memory_format=torch.channels_last)


def fwd_geom(N, H, W, C, OH, OW, KH, KW, stride, pad, Co):
    return [N, H, W, C, OH, OW, KH, KW, stride, stride, 1, 1, -pad, -pad, Co,
            OH, OW, 1, 1, 0, 0, Co]


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def shadow_ohwi(weight: torch.Tensor, cpad: int) -> torch.Tensor:
    """bf16 OHWI weight for the kernels (flat-store shadow when bound; cast otherwise)."""
    slot = getattr(weight, "_slot", None)
    if slot is not None and slot.shadow is not None:
        w = slot.shadow  # [Co, KH, KW, Ci] bf16 contiguous
    else:
        w = weight.detach().permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()
    ci = w.shape[-1]
    if cpad != ci:
        w = torch.nn.functional.pad(w, (0, cpad - ci)).contiguous()
    return w


class ConvHipFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, weight: torch.Tensor, stride: int, pad: int,
                emit_stats: bool):
        ops = _ext.ops()
        N, Cx, H, W = x.shape
        Co, Ci, KH, KW = weight.shape
        assert Cx >= Ci and Cx % 8 == 0, f"input channels {Cx} vs weight {Ci}"
        OH = (H + 2 * pad - KH) // stride + 1
        OW = (W + 2 * pad - KW) // stride + 1
        xn = _nhwc(x)
        w = shadow_ohwi(weight, Cx)
        y = _empty_cl(N, Co, OH, OW, x.device)
        g = fwd_geom(N, H, W, Cx, OH, OW, KH, KW, stride, pad, Co)
        res = run_igemm(ops, xn, w, y.permute(0, 2, 3, 1), g, want_stats=emit_stats)
        if res is not None:
            y._simclr_stats = res  # (partials, nblk): consumed by the next BatchNorm
        ctx.save_for_backward(x, weight)
        ctx.geom = (N, H, W, Cx, Ci, OH, OW, KH, KW, stride, pad, Co)
        return y

    @staticmethod
    def backward(ctx, dy: torch.Tensor):
        ops = _ext.ops()
        x, weight = ctx.saved_tensors
        N, H, W, Cx, Ci, OH, OW, KH, KW, stride, pad, Co = ctx.geom
        dyn = _nhwc(dy)
        if dyn.dtype != torch.bfloat16:
            dyn = dyn.to(torch.bfloat16)
        dx = None
        if ctx.needs_input_grad[0]:
            assert Cx == Ci, "dgrad through a channel-padded stem is not supported"
            w = shadow_ohwi(weight, Ci)
            dx = conv_dgrad(ops, dyn, w, N, H, W, Ci, OH, OW, KH, KW, stride, pad, Co)
        dw = None
        if ctx.needs_input_grad[1]:
            g = fwd_geom(N, H, W, Cx, OH, OW, KH, KW, stride, pad, Co)
            slot = getattr(weight, "_slot", None)
            if slot is not None:
                out = slot.grad  # [Co, KH, KW, Ci] fp32 contiguous view into the flat buffer
            else:
                out = torch.empty((Co, KH, KW, Ci), device=dy.device, dtype=torch.float32)
            run_wgrad(ops, dyn, _nhwc(x), out, g, Ci)
            if slot is not None:
                slot.store.mark_ready(slot.index)
            else:
                dw = out.permute(0, 3, 1, 2)
        return dx, dw, None, None, None


_WT_CACHE: dict = {}


def conv_dgrad(ops, dyn, w_ohwi, N, H, W, Ci, OH, OW, KH, KW, stride, pad, Co):
    """dx [N, Ci, H, W] (channels_last) from dy (NHWC view) and the OHWI bf16 weight."""
    dev = dyn.device
    dx = _empty_cl(N, Ci, H, W, dev)
    dxn = dx.permute(0, 2, 3, 1)
    if stride == 1:
        wt = torch.empty((Ci, KH, KW, Co), device=dev, dtype=torch.bfloat16)
        ops.weight_transform(w_ohwi, wt, [Co, KH, KW, Ci, KH, KW, KH - 1, -1, KW - 1, -1])
        g = [N, OH, OW, Co, H, W, KH, KW, 1, 1, 1, 1, -(KH - 1 - pad), -(KW - 1 - pad), Ci,
             H, W, 1, 1, 0, 0, Ci]
        run_igemm(ops, dyn, wt, dxn, g)
        return dx
    assert stride == 2, "only stride 1/2 convolutions are supported"
    classes = []
    for r in (0, 1):
        for c in (0, 1):
            kh0 = (r + pad) % 2
            kw0 = (c + pad) % 2
            nkh = (KH - kh0 + 1) // 2 if kh0 < KH else 0
            nkw = (KW - kw0 + 1) // 2 if kw0 < KW else 0
            ohc = (H - r + 1) // 2
            owc = (W - c + 1) // 2
            classes.append((r, c, kh0, kw0, nkh, nkw, ohc, owc))
    if any(cl[4] == 0 or cl[5] == 0 for cl in classes if cl[6] > 0 and cl[7] > 0):
        dx.zero_()
    for (r, c, kh0, kw0, nkh, nkw, ohc, owc) in classes:
        if nkh == 0 or nkw == 0 or ohc == 0 or owc == 0:
            continue
        wt = torch.empty((Ci, nkh, nkw, Co), device=dev, dtype=torch.bfloat16)
        ops.weight_transform(w_ohwi, wt, [Co, KH, KW, Ci, nkh, nkw, kh0, 2, kw0, 2])
        ih0 = (r + pad - kh0) // 2
        iw0 = (c + pad - kw0) // 2
        g = [N, OH, OW, Co, ohc, owc, nkh, nkw, 1, 1, -1, -1, ih0, iw0, Ci,
             H, W, 2, 2, r, c, Ci]
        run_igemm(ops, dyn, wt, dxn, g)
    return dx


def conv2d(x: torch.Tensor, w: torch.Tensor, stride, padding, weight_param=None,
           emit_stats: bool = True) -> Optional[torch.Tensor]:
    """HIP conv forward; returns None if this configuration is not supported by the kernels."""
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    if sh != sw or ph != pw or sh not in (1, 2) or x.dtype != torch.bfloat16 or x.dim() != 4:
        return None
    if x.shape[1] % 8 != 0:
        return None
    param = weight_param if weight_param is not None else w
    return ConvHipFn.apply(x, param, sh, ph, emit_stats)
