"""Fused residual-stage executor: the ResNet body (layer1..layer4) as ONE hand-scheduled
forward/backward on the HIP kernels, instead of a chain of per-op autograd nodes.

Reference semantics: torchvision BasicBlock / Bottleneck (v1.5) inside the reference's
``ContrastiveModel.f`` (``/root/reference/model.py:76-114``) with every BatchNorm converted to
SyncBatchNorm (main.py:176) and the two views run as separate forwards (main.py:112-113, so BN
statistics are per view: SURVEY Q17).  The math is unchanged; what changes is where the
BatchNorm work happens:

forward, per block (S = 2 view segments, stats per segment, all-reduced across ranks)::

    a1 = conv1(x)                      epilogue: Σ, Σ² partials of a1        (BN1 stats)
    a2 = conv2(relu(bn1(a1)))          prologue applies BN1+ReLU on the gathered operand, so
                                       the BN1 output is never written to HBM; epilogue: BN2 stats
    a3 = conv3(relu(bn2(a2)))          (bottleneck only) same
    ad = convd(x)                      (downsample) epilogue: BNd stats
    out = relu(bn3(a3) + [bnd(ad) | x])  one elementwise pass (two affines + add + ReLU)

backward, per block, given g = dL/d out::

    BN3 (and BNd) backward reduce/apply with the ReLU mask of ``out`` → da3 (, dad, or the
    identity-path gradient g3 = g·[out > 0])
    db2 = dgrad3(da3): the epilogue applies the BN2-ReLU mask (recomputed from a2) and emits the
          BN2 backward partials Σg, Σg·x̂ (no separate reduce pass) → finalize → da2 (one pass)
    dW3 = wgrad(da3, relu(bn2(a2)))   prologue recomputes the BN2 output on the fly
    ... same for conv2 / BN1 ...
    dx  = dgrad1(da1) + [dgrad_d(dad) | g3]  accumulated in the dgrad epilogue (no extra add)

Compared with the module path this removes the BN1/BN2 apply passes, both backward reduce
passes of BN1/BN2, every autograd gradient-accumulation add at the residual branches, and the
materialised BN outputs (less HBM traffic and memory).  Weight / BN-parameter gradients go
straight into the flat fp32 gradient buffer and notify the bucketed all-reducer as soon as
they are final (overlap with the rest of the backward).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import _ext
from ..ops.conv_hip import (fwd_geom, igemm_choose, igemm_launch, run_wgrad, shadow_ohwi)
from ..parallel import state as pstate
from ..parallel.state import site_key


# attribution experiment (never for training): SIMCLR_SKIP_WGRAD=1 drops the backbone's weight-
# gradient kernels, exposing how much of the step the dgrad / BatchNorm chain alone takes
_SKIP_WGRAD = os.environ.get("SIMCLR_SKIP_WGRAD", "0") == "1"
# attribution experiment: SIMCLR_EXPERIMENT_SKIP_BNREDUCE=fwd|bwd|all drops the BatchNorm
# reduce/finalize launches (garbage statistics): the upper bound of folding them into the convs
_SKIP_BNRED = os.environ.get("SIMCLR_EXPERIMENT_SKIP_BNREDUCE", "")


def _empty_nhwc(n, h, w, c, dev, dtype=torch.bfloat16):
    return torch.empty((n, h, w, c), device=dev, dtype=dtype)


def _allreduce(t: torch.Tensor, st, branch: bool = False) -> None:
    if st.comm:
        g = st.branch_stat_group if branch and st.branch_stat_group is not None else st.stats_group
        dist.all_reduce(t, group=g)


def _stage_of(b: "_BlockSpec") -> int:
    """ResNet stage (1-4) of a block named ``layer<s>.<i>``."""
    return int(b.name[5]) if b.name.startswith("layer") else 0


def _deliver_grad(param: torch.Tensor, compute) -> None:
    """Run ``compute(out)`` writing the fp32 gradient of ``param`` into its flat-store slot
    (and notify the reducer); unbound parameters accumulate into ``param.grad``."""
    slot = getattr(param, "_slot", None)
    if slot is not None:
        compute(slot.grad)
        slot.store.mark_ready(slot.index)
        return
    g = torch.empty(param.shape if param.dim() != 4 else
                    (param.shape[0], param.shape[2], param.shape[3], param.shape[1]),
                    device=param.device, dtype=torch.float32)
    compute(g)
    if param.dim() == 4:
        g = g.permute(0, 3, 1, 2)
    if param.grad is None:
        param.grad = g.contiguous() if param.dim() != 4 else g
    else:
        param.grad.add_(g)


@dataclass
class _ConvSpec:
    conv: torch.nn.Module
    bn: torch.nn.Module
    stride: int
    k: int
    pad: int


@dataclass
class _BlockSpec:
    convs: List[_ConvSpec]
    down: Optional[_ConvSpec]
    name: str = ""


@dataclass
class _BNState:
    mi: torch.Tensor        # [2][S][C] mean / invstd
    ss: torch.Tensor        # [2][S][C] scale / shift
    count: float


@dataclass
class _BlockTape:
    x: torch.Tensor                     # block input, NHWC bf16
    acts: List[torch.Tensor] = field(default_factory=list)   # pre-BN conv outputs (NHWC)
    bns: List[_BNState] = field(default_factory=list)
    # what conv i actually consumed: (tensor, prologue scale/shift or None)
    ins: List[Tuple[torch.Tensor, Optional[torch.Tensor]]] = field(default_factory=list)
    ad: Optional[torch.Tensor] = None
    bnd: Optional[_BNState] = None
    out: Optional[torch.Tensor] = None
    mask: Optional[torch.Tensor] = None  # uint8 ReLU bitmask of ``out`` (bit per channel)
    # pooled stem only: (window argmax bytes, pre-BN value at the argmax) of the max-pool
    pool: Optional[Tuple[torch.Tensor, torch.Tensor]] = None


# persistent blocks per view segment of the fused 1x1 backward (2 segments: 2x this many blocks)
_BWD1X1_BPS = 128

# bit 8 of the igemm epilogue mode: the residual operand is stride-2 subsampled (conv.hip)
_EPI_SUB = 256


class FusedStages:
    """Executor over ``resnet.layer1..layer4`` (modules stay the parameter / state owners).

    The fusion switches below are instance attributes (tests and A/B tools flip them on a built
    executor); the class attribute ``BLOCK_OUT_PROLOGUE`` is the default of new executors."""

    BLOCK_OUT_PROLOGUE = True
    # SIMCLR_FUSED_STEM=0: the stem stays on the per-module path (A/B attribution)
    STEM_FUSED = os.environ.get("SIMCLR_FUSED_STEM", "1") != "0"

    def __init__(self, resnet: torch.nn.Module, segments: int = 2):
        from .resnet import BasicBlock, Bottleneck
        self.resnet = resnet
        self.S = segments
        self.calls = 0
        # launch accounting (tests): block outputs formed in a conv1 prologue / as their own pass
        self.dual_launches = 0
        self.out_apply_calls = 0
        # BN backward of a bottleneck's conv3 inside conv3's dgrad/wgrad operand prologues
        # (only up to 128 input channels: measured net loss or break-even above, r2 log)
        self.bnb_prologue = True
        self._bnb_max_cin = 128
        # BN1's backward in conv1's operand prologues as well: measured +0.85 ms/step (r4 log)
        self.lazy_bn1 = False
        # expansion convs from this many input channels on read a materialised BN2+ReLU input
        # (_mat_expand)
        self.mat_expand_min_cin = 128
        # a downsample block's output gradient: BN3's backward in conv3's operand prologues and
        # only the downsample BN's gradient materialised (one-output apply instead of the
        # two-output bn_bwd_apply2) where conv3's backward is the fused 1x1 kernel (layer1.0):
        # -0.12 ms/step (3 of 3 A/B rounds); also on the other prologue-eligible conv3s
        # (layer2.0, register-staged weight gradient) neutral to worse (r4 optimisation log)
        self.lazy_bn3_ds = True
        self._lazy_bn3_ds_dual_only = True
        # a 3x3 stride-1 conv2's output-gradient BatchNorm backward (BN2) in its patch-kernel
        # dgrad prologue, which also stores it for the weight gradient: one pass instead of a
        # bn_bwd_apply pass plus the dgrad's re-read (layer1 / layer2; _patch_bnb_ok)
        self.patch_bnb = os.environ.get("SIMCLR_PATCH_BNB", "1") != "0"
        # weight gradients on a second stream (forked after each conv's dY is final, joined at
        # the end of the backward): they only feed the flat gradient buffer, so they overlap the
        # dgrad / BatchNorm chain that the next layer's gradient depends on
        self.wgrad_stream = os.environ.get("SIMCLR_WGRAD_STREAM", "1") != "0"
        self._side = None
        # the downsample branch of a stage's first block (forward conv + BN, backward dgrad) on
        # its own stream, concurrent with the main branch until the block output / conv1 dgrad
        self.branch_stream = os.environ.get("SIMCLR_BRANCH_STREAM", "1") != "0"
        # a stride-2 1x1 downsample's dgrad is kept compact ([N, H/2, W/2, C]: it only reaches
        # the even positions) and added by conv1's dgrad epilogue through the subsampled-residual
        # mode — instead of zero-filling a full-resolution tensor (0.9 GB/step of fills at
        # ResNet-50 CIFAR) and re-reading it whole
        self.compact_ds = True
        self._branch = None
        # a block's output (BN3 + shortcut + ReLU) formed inside the next block's conv1 prologue
        # instead of a separate pass that conv1 re-reads, at every stage (the prologue kernels
        # keep their DMA pipelined: 24.06 -> 23.80 ms/step A/B, r2 optimisation log)
        self.block_out_min_hw = 1
        self.block_out_prologue = type(self).BLOCK_OUT_PROLOGUE
        # a bottleneck's conv3 backward at Ci = 64 / Co = 256 (ResNet-50 layer1) as ONE fused
        # pass (conv.hip conv1x1_bwd_dual): dgrad + BN2 mask / partials + weight gradient, so the
        # 0.5-1 GB output gradient is read once instead of once per pass
        self.fused_bwd1x1 = True
        # ... and the wide form at Ci = 128 / Co = 512 (ResNet-50 layer2 conv3; conv.hip
        # conv1x1_bwd_dual_w: the Ci slices of a row range share each dY tile through L2), which
        # also takes the forward's materialised BN2+ReLU input (_mat_expand) as its X operand
        self.fused_bwd1x1_wide = True
        # a stride-1 1x1 downsample of that shape (layer1.0, Co 256 / Ci 64) whose BatchNorm
        # backward is lazy: its dgrad and weight gradient from one pass over g and its pre-BN
        # activation (the plain form of conv1x1_bwd_dual) instead of a BN-apply pass writing
        # its input gradient, a dgrad and a weight gradient each reading it; on the main stream
        # ("main") or the downsample branch stream ("branch")
        # the narrow fused 1x1 backward (Co 256 / Ci 64) as the 8-wave kernel
        # (conv1x1_bwd_dual_w, 64-row tiles) instead of the 4-wave one: -0.03..-0.08 ms/step,
        # 3 of 3 rounds (r6 log)
        self.dual8 = True
        # the fused 1x1 backward kernels' weight-gradient slab reduction on the main stream
        # (serial, ~10 µs at the full chip) instead of the weight-gradient stream
        self.dual_reduce_main = False
        self.fused_ds_dual = True
        # persistent blocks per view segment of the fused 1x1 backward kernels (A/B knobs):
        # narrow form / layer1.0 downsample, and the wide form (x 2 Ci slices)
        self.bwd1x1_bps = _BWD1X1_BPS
        self.bwd1x1_bps_wide = 64
        # the ImageNet stem (7x7 / stride 2 / pad 3 over the 3 image channels) as a 4x4 / stride-1
        # conv over the 2x2 space-to-depth of the padded image (csrc/eval.hip k_stem_s2d):
        # K 256 instead of 392 gathered columns, 32-byte instead of 16-byte gathers
        self.stem_s2d = True
        # ... and layer2.0's stride-2 downsample (Co 512 / Ci 256, dY materialised): measured
        # neutral to +0.06 ms (r6 log), so off by default
        self.fused_ds_dual_s2 = False
        self.ds_dual_stream = "main"
        self._side_keep: List[torch.Tensor] = []
        # dgrad weight transforms of the whole backbone: one batched launch per backward
        self._wt_sig = None
        self._wt_cache = {}
        self._wt_table = None
        self._wt_ready = False
        # the stem (conv1 + bn1 + ReLU, when no max-pool follows) inside the executor: its BatchNorm
        # backward partials come from layer1.0's conv1 dgrad epilogue (mode 4, like every block
        # boundary) and its weight gradient applies the BN backward in the dY prologue — no
        # separate reduce pass over the 1024 x 32 x 32 x 64 stem activation, no materialised
        # input gradient (stem_forward / backward)
        # A/B of the fusion switches above without code edits (tools/envab.sh):
        # SIMCLR_FUSED_ATTRS="attr=value,..." (ints / true / false / strings), applied at
        # construction
        for kv in filter(None, os.environ.get("SIMCLR_FUSED_ATTRS", "").split(",")):
            k, v = kv.split("=", 1)
            if not hasattr(self, k):
                raise ValueError(f"SIMCLR_FUSED_ATTRS: FusedStages has no switch {k!r}")
            if v.lower() in ("true", "false"):
                setattr(self, k, v.lower() == "true")
            else:
                try:
                    setattr(self, k, int(v))
                except ValueError:
                    setattr(self, k, v)
        self.stem_fused = type(self).STEM_FUSED
        self.stem = None
        self._stem_block = None
        # the ImageNet stem's max-pool (k, stride, pad), fused around (stem_forward / backward):
        # BN + ReLU + max-pool in one pass, the max-pool / ReLU / BN backward in one pass
        self.stem_pool = None
        from .resnet import _Identity
        from ..ops.pooling import MaxPool2d
        mp = getattr(resnet, "maxpool", None)
        if isinstance(mp, (_Identity, MaxPool2d)):
            c1 = resnet.conv1
            k = c1.kernel_size[0] if isinstance(c1.kernel_size, tuple) else c1.kernel_size
            st_ = c1.stride[0] if isinstance(c1.stride, tuple) else c1.stride
            pd = c1.padding[0] if isinstance(c1.padding, tuple) else c1.padding
            self.stem = _ConvSpec(c1, resnet.bn1, st_, k, pd)
            self._stem_block = _BlockSpec([self.stem], None, "stem")
            if isinstance(mp, MaxPool2d):
                self.stem_pool = (int(mp.kernel_size), int(mp.stride), int(mp.padding))
        self.blocks: List[_BlockSpec] = []
        for li, layer in enumerate((resnet.layer1, resnet.layer2, resnet.layer3, resnet.layer4)):
            for bi, blk in enumerate(layer):
                if isinstance(blk, Bottleneck):
                    convs = [_ConvSpec(blk.conv1, blk.bn1, 1, 1, 0),
                             _ConvSpec(blk.conv2, blk.bn2, blk.stride, 3, 1),
                             _ConvSpec(blk.conv3, blk.bn3, 1, 1, 0)]
                elif isinstance(blk, BasicBlock):
                    convs = [_ConvSpec(blk.conv1, blk.bn1, blk.stride, 3, 1),
                             _ConvSpec(blk.conv2, blk.bn2, 1, 3, 1)]
                else:
                    raise TypeError(f"unsupported block {type(blk).__name__}")
                down = None
                if blk.downsample is not None:
                    down = _ConvSpec(blk.downsample[0], blk.downsample[1], blk.stride, 1, 0)
                self.blocks.append(_BlockSpec(convs, down, f"layer{li + 1}.{bi}"))

    # ------------------------------------------------------------------ feasibility
    def supported(self, x: torch.Tensor) -> bool:
        """Every fused launch needs view segments aligned to the smallest tile (64 rows)."""
        if x.dtype != torch.bfloat16 or not x.is_cuda or x.dim() != 4:
            return False
        Nb, C, H, W = x.shape
        return self._shape_ok(Nb, H, W)

    def stem_supported(self, img: torch.Tensor) -> bool:
        """The image batch can enter at the stem: a stem conv without max-pool, an input that
        needs no gradient, and stem-output rows per view that tile (256-row BatchNorm-backward
        prologue splits of the stem weight gradient)."""
        if not (getattr(self, "stem_fused", False) and self.stem is not None):
            return False
        if (img.requires_grad or img.dtype != torch.bfloat16 or not img.is_cuda
                or img.dim() != 4 or img.shape[1] % 8 or img.shape[1] < self.stem.conv.in_channels):
            return False
        Nb, _, H, W = img.shape
        cs = self.stem
        OH = (H + 2 * cs.pad - cs.k) // cs.stride + 1
        OW = (W + 2 * cs.pad - cs.k) // cs.stride + 1
        if self.stem_pool is not None:
            # the stem weight gradient reads a materialised BN input gradient (no 256-row
            # BN-backward prologue splits); the blocks see the pooled map
            K, Sd, P = self.stem_pool
            if Nb % self.S or ((Nb // self.S) * OH * OW) % 64 or self.stem.conv.out_channels % 8:
                return False
            PH, PW = (OH + 2 * P - K) // Sd + 1, (OW + 2 * P - K) // Sd + 1
            return self._shape_ok(Nb, PH, PW)
        if Nb % self.S or ((Nb // self.S) * OH * OW) % 256:
            return False
        return self._shape_ok(Nb, OH, OW)

    def _shape_ok(self, Nb: int, H: int, W: int) -> bool:
        if Nb % self.S or H != W:
            return False
        n = Nb // self.S
        for b in self.blocks:
            hin = H
            for i, cs in enumerate(b.convs):
                oh = (hin + 2 * cs.pad - cs.k) // cs.stride + 1
                if (n * oh * oh) % 64:
                    return False
                if cs.stride == 2:  # BN-epilogue dgrad: per parity-class segments
                    for r in (0, 1):
                        if (n * ((hin - r + 1) // 2) ** 2) % 64:
                            return False
                hin = oh
            H = hin
        return True

    # ------------------------------------------------------------------ building blocks
    def _conv_bn_fwd(self, ops, xn, cs: _ConvSpec, pro_ss: Optional[torch.Tensor], S: int, st,
                     dual=None, slot: int = 0):
        """a = conv(pro(x)) and the BatchNorm state of ``cs.bn`` over it (statistics partials
        from the conv epilogue, one reduce / finalize launch)."""
        a, partial, nblk = self._conv_fwd(ops, xn, cs, pro_ss, S, dual=dual)
        rows_seg = a.shape[0] * a.shape[1] * a.shape[2] // S
        return a, self._bn_fwd(ops, cs.bn, partial, nblk, rows_seg, S, st, slot=slot)

    def _s2d_ok(self, cs: _ConvSpec, xn: torch.Tensor) -> bool:
        """The stem conv runs in its space-to-depth form (``stem_s2d``)."""
        if not (getattr(self, "stem_s2d", False) and cs is self.stem and xn.is_cuda):
            return False
        Nb, H, W, C = xn.shape
        return (cs.k == 7 and cs.stride == 2 and cs.pad == 3 and cs.conv.in_channels <= 4
                and C % 4 == 0 and (H + 6) % 2 == 0 and (W + 6) % 2 == 0)

    def _s2d_input(self, ops, xn: torch.Tensor) -> torch.Tensor:
        """[Nb, (H+6)/2, (W+6)/2, 16]: the padded image, 2x2 space-to-depth (kept for the
        weight gradient of the same step)."""
        c = getattr(self, "_s2d_cache", None)
        if c is not None and c[0] is xn:
            return c[1]
        Nb, H, W, _ = xn.shape
        xs = _empty_nhwc(Nb, (H + 6) // 2, (W + 6) // 2, 16, xn.device)
        ops.stem_s2d(xn, self.stem.conv.in_channels, 3, xs)
        self._s2d_cache = (xn, xs)
        return xs

    @staticmethod
    def _s2d_weight(weight: torch.Tensor) -> torch.Tensor:
        """7x7 kernel [Co][Ci<=4][7][7] -> the 4x4 kernel over the space-to-depth input,
        OHWI [Co][4][4][16]: w'[co][bh][bw][(dy * 2 + dx) * 4 + c] = w[co][c][2bh + dy][2bw + dx]
        (zero at 2bh + dy = 7 or 2bw + dx = 7 and for c >= Ci)."""
        w = shadow_ohwi(weight, weight.shape[1])  # [Co][7][7][Ci] bf16
        Co, Ci = w.shape[0], w.shape[-1]
        w8 = torch.nn.functional.pad(w, (0, 4 - Ci, 0, 1, 0, 1))  # [Co][8][8][4]
        return w8.view(Co, 4, 2, 4, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(Co, 4, 4, 16)

    @staticmethod
    def _s2d_unfold_grad(gs: torch.Tensor, out: torch.Tensor) -> None:
        """Weight gradient of the 4x4 form [Co][4][4][16] -> the 7x7 kernel's, OHWI
        [Co][7][7][Ci] (``out``, fp32)."""
        Co, Ci = out.shape[0], out.numel() // (out.shape[0] * 49)
        g8 = gs.view(Co, 4, 4, 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(Co, 8, 8, 4)
        out.view(Co, 7, 7, Ci).copy_(g8[:, :7, :7, :Ci])

    def _conv_fwd(self, ops, xn, cs: _ConvSpec, pro_ss: Optional[torch.Tensor], S: int,
                  dual=None):
        """a = conv(pro(x)) with BN statistics partials in the epilogue.

        ``dual = (aL, ss, res, rss, out, mask)``: the input is the previous block's output,
        formed in this conv's prologue from that block's conv3 activation ``aL`` and residual
        ``res`` and written to ``out`` / ``mask`` by the same kernel (``xn`` is ``out``).
        Returns (a, partials, blocks per segment); the caller reduces the partials
        (``_bn_fwd``)."""
        Nb, H, W, C = xn.shape
        Co = cs.conv.out_channels
        OH = (H + 2 * cs.pad - cs.k) // cs.stride + 1
        OW = (W + 2 * cs.pad - cs.k) // cs.stride + 1
        a = _empty_nhwc(Nb, OH, OW, Co, xn.device)
        if dual is None and pro_ss is None and self._s2d_ok(cs, xn):
            xn = self._s2d_input(ops, xn)
            w = self._s2d_weight(cs.conv.weight)
            g = fwd_geom(Nb, xn.shape[1], xn.shape[2], 16, OH, OW, 4, 4, 1, 0, Co)
        else:
            w = shadow_ohwi(cs.conv.weight, C)
            g = fwd_geom(Nb, H, W, C, OH, OW, cs.k, cs.k, cs.stride, cs.pad, Co)
        M = Nb * OH * OW
        pro, dl, A = None, None, xn
        if dual is not None:
            aL, ss, res, rss, out, mask = dual
            pro = (ss[0], ss[1], M // S, True)
            dl, A = (res, None if rss is None else rss.view(-1), out, mask), aL
        elif pro_ss is not None:
            pro = (pro_ss[0], pro_ss[1], M // S, True)
        v = igemm_choose(ops, A, w, a, g, want_stats=True, pro=pro, seg_rows=M // S, dual=dl)
        bm = ops.igemm_variant_bm(v)
        stats = torch.empty(((M // bm) * 2 * Co,), device=xn.device, dtype=torch.float32)
        igemm_launch(ops, A, w, a, g, v, stats=stats, pro=pro, dual=dl)
        return a, stats, M // bm // S

    def _dual_ok(self, ops, xn, cs: _ConvSpec, S: int) -> bool:
        """Can ``cs`` (a block's conv1) form its input — the previous block's output — in its
        prologue (1x1 / stride 1 / unpadded, an LDS-DMA tile that fits the doubled staging)?"""
        if not (getattr(self, "block_out_prologue", False) and xn.is_cuda and cs.k == 1
                and cs.stride == 1 and cs.pad == 0):
            return False
        Nb, H, W, C = xn.shape
        if H < getattr(self, "block_out_min_hw", 1):
            return False
        key = (Nb, H, W, C, cs.conv.out_channels, S)
        cache = self.__dict__.setdefault("_dual_cache", {})
        if key not in cache:  # host-side admissibility, once per shape
            g = fwd_geom(Nb, H, W, C, H, W, 1, 1, 1, 0, cs.conv.out_channels)
            M = Nb * H * W
            cache[key] = any(ops.igemm_dual_ok(v, g) and (M // S) % ops.igemm_variant_bm(v) == 0
                             for v in range(ops.igemm_nvariants()))
        return cache[key]

    def _bn_fwd(self, ops, bn, partial, nblk_seg: int, rows_seg: int, S: int, st,
                slot: int = 0) -> _BNState:
        """``slot``: ticket array of the last-arriver reduce (1 on the downsample stream, so a
        concurrent reduce on the main stream never shares its counters)."""
        C = bn.num_features
        dev = partial.device
        count = float(rows_seg * st.world_size)
        mi = torch.empty((2 * S * C,), device=dev, dtype=torch.float32)
        ss = torch.empty((2 * S * C,), device=dev, dtype=torch.float32)
        ipc = st.ipc
        if _SKIP_BNRED in ("fwd", "all"):
            return _BNState(mi, ss.view(2, S * C), count)
        if not st.comm or ipc is not None:
            # one launch: reduce + finalize (last-arriver); at world > 1 the IPC statistics
            # exchange runs inside it (comm/ipc.py)
            ops.bn_reduce_fused(partial, nblk_seg, S, C, 1, None, count, bn.eps, bn.momentum,
                                bn.running_mean, bn.running_var, mi, bn.num_batches_tracked,
                                bn.weight.detach(), bn.bias.detach(), ss, None, None, None, slot,
                                **(ipc.kwargs(site_key(bn, "fwd"), S, C) if ipc is not None else {}))
        else:
            stats = torch.empty((2 * S * C,), device=dev, dtype=torch.float32)
            ops.bn_reduce_fused(partial, nblk_seg, S, C, 0, stats, ticket_slot=slot)
            _allreduce(stats, st, branch=slot == 1)
            ops.bn_finalize(stats, S, C, count, bn.eps, bn.momentum, bn.running_mean,
                            bn.running_var, mi, bn.num_batches_tracked, bn.weight.detach(),
                            bn.bias.detach(), ss)
        return _BNState(mi, ss.view(2, S * C), count)

    def _deliver_bn_grads(self, bn, run) -> None:
        """``run(dgamma_out, dbeta_out)`` writes dγ, dβ; route them into the flat store."""
        gslot = getattr(bn.weight, "_slot", None)
        bslot = getattr(bn.bias, "_slot", None)
        if gslot is not None and bslot is not None:
            run(gslot.grad, bslot.grad)
            gslot.store.mark_ready(gslot.index)
            bslot.store.mark_ready(bslot.index)
            return
        C = bn.num_features
        dg = torch.empty((C,), device=bn.weight.device, dtype=torch.float32)
        db = torch.empty((C,), device=bn.weight.device, dtype=torch.float32)
        run(dg, db)
        _deliver_grad(bn.weight, lambda o: o.copy_(dg))
        _deliver_grad(bn.bias, lambda o: o.copy_(db))

    def _bn_bwd_start(self, ops, bn, partial, nblk_seg: int, bs: _BNState, S: int, st):
        """Phase 1 of a BN backward from Σg, Σg·x̂ partials.

        Distributed: reduce to the LOCAL [2][S][C] sums, write dγ, dβ from them (SyncBN
        semantics: parameter gradients are per-rank and summed by the data-parallel reducer
        like every other gradient — using the all-reduced sums here would count them W
        times), then start the all-reduce of the sums asynchronously; the caller schedules
        independent work (a weight gradient) before ``_bn_bwd_finish``.  Single GPU: nothing
        to wait for (one fused launch in the finish)."""
        C = bn.num_features
        if not st.comm or st.ipc is not None:
            return ("local", bn, partial, nblk_seg, bs, st.ipc)
        dev = partial.device
        sums = torch.empty((2 * S * C,), device=dev, dtype=torch.float32)
        # one launch: the local sums (all-reduced below) and dγ, dβ from them
        self._deliver_bn_grads(bn, lambda dg, db: ops.bn_reduce_fused(
            partial, nblk_seg, S, C, 0, sums, dgamma=dg, dbeta=db))
        work = dist.all_reduce(sums, group=st.stats_group, async_op=True)
        return ("dist", bn, sums, work, bs)

    def _bn_bwd_finish(self, ops, h, S: int) -> torch.Tensor:
        """Phase 2: coef [3][S][C] for the input gradient (from the global sums)."""
        bn, bs = h[1], h[4]
        C = bn.num_features
        dev = bs.mi.device
        coef = torch.empty((3 * S * C,), device=dev, dtype=torch.float32)
        if _SKIP_BNRED in ("bwd", "all"):
            return coef
        if h[0] == "local":
            # single launch; with the IPC exchange dγ, dβ come from the local sums and coef
            # from the global ones (SyncBN semantics, see _bn_bwd_start)
            partial, nblk_seg, ipc = h[2], h[3], h[5]
            kw = ipc.kwargs(site_key(bn, "bwd"), S, C) if ipc is not None else {}
            self._deliver_bn_grads(bn, lambda dg, db: ops.bn_reduce_fused(
                partial, nblk_seg, S, C, 2, None, bs.count, 0.0, 0.0, None, None, bs.mi,
                None, bn.weight.detach(), None, None, dg, db, coef, **kw))
        else:
            sums, work = h[2], h[3]
            work.wait()
            ops.bn_bwd_finalize(sums, bs.mi, bn.weight.detach(), S, C, bs.count, None, None,
                                coef)
        return coef

    def _bn_bwd(self, ops, bn, partial, nblk_seg: int, bs: _BNState, S: int, st) -> torch.Tensor:
        return self._bn_bwd_finish(ops, self._bn_bwd_start(ops, bn, partial, nblk_seg, bs, S, st),
                                   S)

    def _wgrad(self, ops, dyn, xn, cs: _ConvSpec, pro_ss: Optional[torch.Tensor], S: int,
               bnb: Optional[Tuple] = None, main: bool = False):
        """``bnb = (a, coef)``: dy = coef.A·dyn + coef.B·a + coef.D, the BatchNorm backward of
        the conv's own BN, computed in the dY operand's prologue (never written to HBM)."""
        Nb, H, W, C = xn.shape
        Co = cs.conv.out_channels
        OH, OW = dyn.shape[1], dyn.shape[2]
        s2d = pro_ss is None and self._s2d_ok(cs, xn)
        if s2d:
            xn = self._s2d_input(ops, xn)
            g = fwd_geom(Nb, xn.shape[1], xn.shape[2], 16, OH, OW, 4, 4, 1, 0, Co)
        else:
            g = fwd_geom(Nb, H, W, C, OH, OW, cs.k, cs.k, cs.stride, cs.pad, Co)
        M = Nb * OH * OW
        pro = None
        if pro_ss is not None:
            pro = (pro_ss[0], pro_ss[1], M // S, True, S)
        dpro = (bnb[0], bnb[1], M // S, S) if bnb is not None else None

        side = getattr(self, "_side", None) if getattr(self, "wgrad_stream", False) else None
        concurrent = side is not None and not main

        def run():
            if _SKIP_WGRAD:  # attribution experiment only: the step without weight gradients
                _deliver_grad(cs.conv.weight, lambda out: None)
                return
            if s2d:  # the 4x4 form's gradient, folded back onto the 7x7 kernel
                def s2d_grad(out):
                    gs = torch.empty((Co, 4, 4, 16), device=dyn.device, dtype=torch.float32)
                    run_wgrad(ops, dyn, xn, gs, g, 16, pro=pro, dpro=dpro, concurrent=concurrent)
                    self._s2d_unfold_grad(gs, out)
                _deliver_grad(cs.conv.weight, s2d_grad)
                return
            # creal: the stem's 3 image channels are gathered as 8 (zero-padded)
            _deliver_grad(cs.conv.weight,
                          lambda out: run_wgrad(ops, dyn, xn, out, g, cs.conv.in_channels,
                                                pro=pro, dpro=dpro, concurrent=concurrent))

        if side is None or main:
            run()
            return
        # operands stay referenced until the join (the caching allocator must not hand their
        # memory to a main-stream allocation while the side stream still reads them)
        self._side_keep.extend(t for t in (dyn, xn, pro_ss, *(bnb or ())) if t is not None)
        side.wait_stream(torch.cuda.current_stream(dyn.device))
        with torch.cuda.stream(side):
            run()

    @staticmethod
    def _bwd1x1_bps(rows_seg: int, cap: int = _BWD1X1_BPS) -> int:
        """Persistent blocks per view segment of conv1x1_bwd_dual (64-row tiles, equal shares)."""
        tiles = rows_seg // 64
        b = min(cap, tiles)
        while b > 1 and tiles % b:
            b -= 1
        return b

    def _bwd1x1_ok(self, cs: _ConvSpec, dyn: torch.Tensor, xin: torch.Tensor, pro_ss, a_prev,
                   S: int) -> bool:
        M = dyn.numel() // dyn.shape[-1]
        if not (getattr(self, "fused_bwd1x1", False) and cs.k == 1 and cs.stride == 1
                and M % S == 0 and (M // S) % 64 == 0):
            return False
        co, ci = cs.conv.out_channels, cs.conv.in_channels
        if (co, ci) == (256, 64):
            return xin is a_prev and pro_ss is not None and M * 256 * 2 < (1 << 31)
        if (co, ci) == (512, 128) and getattr(self, "fused_bwd1x1_wide", False):
            # X: a2 with the BN2 prologue, or the forward's materialised relu(bn2(a2))
            return ((xin is a_prev and pro_ss is not None)
                    or (pro_ss is None and xin.shape == a_prev.shape)) and M * 512 * 2 < (1 << 31)
        return False

    def _bwd1x1_fused(self, ops, dyn, bnb, cs: _ConvSpec, a_prev, bs_prev: _BNState, S: int,
                      xin: Optional[torch.Tensor] = None):
        """conv3 dgrad (mode-3 epilogue of BN2) + weight gradient in one launch; the weight
        gradient's split reduction runs on the side stream.  Returns (gm, partials, blocks per
        segment) like ``_dgrad`` with ``bn_epi=("mask", ...)``.  ``xin``: the conv's forward
        input when it was materialised (relu(bn2(a2)); wide form only)."""
        Nb, H, W, Ci = a_prev.shape
        Co = cs.conv.out_channels
        M = Nb * H * W
        wide = (Co, Ci) == (512, 128)
        # the wide kernel launches 2 blocks (Ci slices) per row block: 64 row blocks per view
        # segment fill the chip's 256 CUs once at S = 2
        bps = self._bwd1x1_bps(M // S, self.bwd1x1_bps_wide if wide else self.bwd1x1_bps)
        xraw = xin if (wide and xin is not None and xin is not a_prev) else None
        w = shadow_ohwi(cs.conv.weight, Ci)
        wt = self._dgrad_weight(ops, cs, w, (0, 0), [Co, 1, 1, Ci, 1, 1, 0, -1, 0, -1])
        dev = dyn.device
        gm = _empty_nhwc(Nb, H, W, Ci, dev)
        stats = torch.empty((S * bps * 2 * Ci,), device=dev, dtype=torch.float32)
        wpart = torch.empty((S * bps * Co * Ci,), device=dev, dtype=torch.float32)
        a3, coef = (bnb[0], bnb[1]) if bnb is not None else (None, None)
        if xraw is not None:  # X = the materialised relu(bn2(a2)); a2 for the epilogue
            ops.conv1x1_bwd_dual(dyn, a3, coef, xraw, bs_prev.ss.view(-1), bs_prev.mi.view(-1),
                                 wt, gm, stats, wpart, S, bps, a_prev)
        else:
            ops.conv1x1_bwd_dual(dyn, a3, coef, a_prev, bs_prev.ss.view(-1),
                                 bs_prev.mi.view(-1), wt, gm, stats, wpart, S, bps,
                                 dual8=bool(getattr(self, "dual8", False)))

        def run():
            if _SKIP_WGRAD:
                _deliver_grad(cs.conv.weight, lambda out: None)
                return
            _deliver_grad(cs.conv.weight,
                          lambda out: ops.wgrad_reduce_slabs(wpart, S * bps, out))

        side = getattr(self, "_side", None) if getattr(self, "wgrad_stream", False) else None
        if getattr(self, "dual_reduce_main", False):
            side = None
        if side is None:
            run()
        else:
            self._side_keep.append(wpart)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                run()
        return gm, stats, bps

    def _ds_dual_ok(self, b: _BlockSpec, tp: _BlockTape, S: int) -> bool:
        """A 1x1 downsample whose input needs no transform (the block input): stride 1 at the
        narrow dual shape (Co 256 / Ci 64, lazy BN backward), or stride 2 at Co 512 / Ci 256
        (layer2.0; dY materialised: ``_ds_dual_s2``)."""
        cs = b.down
        if not (getattr(self, "fused_ds_dual", False) and getattr(self, "fused_bwd1x1", False)
                and tp.x.is_cuda and cs.k == 1 and cs.pad == 0 and b.convs[0].stride == 1):
            return False
        Nb, H, W, Ci = tp.x.shape
        shape = (cs.conv.out_channels, cs.conv.in_channels)
        if cs.stride == 1:
            M = Nb * H * W
            return (shape == (256, 64) and Ci == 64 and M % S == 0 and (M // S) % 64 == 0
                    and M * 256 * 2 < (1 << 31))
        if cs.stride == 2 and getattr(self, "fused_ds_dual_s2", False):
            Mo = Nb * ((H + 1) // 2) * ((W + 1) // 2)
            return (shape == (512, 256) and Ci == 256 and Nb % S == 0 and (Mo // S) % 64 == 0
                    and Mo * 512 * 2 < (1 << 31) and tp.x.numel() * 2 < (1 << 31))
        return False

    def _ds_dual(self, ops, b: _BlockSpec, tp: _BlockTape, lazy_d, S: int) -> torch.Tensor:
        """The downsample's input gradient (the residual of conv1's dgrad) and weight gradient
        from one pass over g3 and the pre-BN activation ad, the downsample BN's backward applied
        in registers (conv1x1_bwd_dual, plain form).  The weight gradient's split reduction runs
        on the weight-gradient stream."""
        cs = b.down
        g3, coefd = lazy_d
        Nb, H, W, Ci = tp.x.shape
        Co = cs.conv.out_channels
        dev = g3.device
        _ext.TAG = f"{b.name} ds dgrad+wgrad"
        if cs.stride == 2:
            # layer2.0: dY materialised (the lazy form of the wide kernel spills), then ONE pass
            # for the compact input gradient and the weight gradient (strided X)
            OH, OW = (H + 1) // 2, (W + 1) // 2
            dad = torch.empty_like(tp.ad)
            ops.bn_bwd_apply(g3, None, tp.ad, coefd, S, False, dad, None)
            bps = self._bwd1x1_bps(Nb * OH * OW // S, 32)
            w = shadow_ohwi(cs.conv.weight, Ci)
            wt = self._dgrad_weight(ops, cs, w, (0, 0), [Co, 1, 1, Ci, 1, 1, 0, 2, 0, 2])
            resid = _empty_nhwc(Nb, OH, OW, Ci, dev)
            wpart = torch.empty((S * bps * Co * Ci,), device=dev, dtype=torch.float32)
            ops.conv1x1_bwd_dual_s2(dad, None, None, tp.x, wt, resid, wpart, S, bps)
        else:
            M = Nb * H * W
            bps = self._bwd1x1_bps(M // S, self.bwd1x1_bps)
            w = shadow_ohwi(cs.conv.weight, Ci)
            wt = self._dgrad_weight(ops, cs, w, (0, 0), [Co, 1, 1, Ci, 1, 1, 0, -1, 0, -1])
            resid = _empty_nhwc(Nb, H, W, Ci, dev)
            wpart = torch.empty((S * bps * Co * Ci,), device=dev, dtype=torch.float32)
            nostats = torch.empty((1,), device=dev, dtype=torch.float32)
            ops.conv1x1_bwd_dual(g3, tp.ad, coefd, tp.x, None, None, wt, resid, nostats, wpart,
                                 S, bps, dual8=bool(getattr(self, "dual8", False)))

        def run():
            if _SKIP_WGRAD:
                _deliver_grad(cs.conv.weight, lambda out: None)
                return
            _deliver_grad(cs.conv.weight, lambda out: ops.wgrad_reduce_slabs(wpart, S * bps, out))

        side = getattr(self, "_side", None) if getattr(self, "wgrad_stream", False) else None
        if getattr(self, "dual_reduce_main", False):
            side = None
        if side is None:
            run()
        else:
            self._side_keep.append(wpart)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                run()
        return resid

    def _bnb_ok(self, cs: _ConvSpec, a: torch.Tensor, S: int) -> bool:
        """The BN-backward operand prologue applies to a 1x1 stride-1 conv whose per-segment
        rows tile evenly (64-row wgrad splits, 64..256-row dgrad tiles), and pays off only
        while each dy element is loaded about once: the dgrad re-reads its A operand per
        output-channel tile and the wgrad its dY operand per input-channel tile, so with
        ≥ 256 input channels the repeated prologue work outweighs the saved HBM pass
        (measured on layer3/layer4 of ResNet-50: net loss or break-even)."""
        M = a.numel() // a.shape[-1]
        return (self.bnb_prologue and cs.k == 1 and cs.stride == 1 and M % S == 0
                and (M // S) % 256 == 0 and cs.conv.in_channels <= getattr(self, "_bnb_max_cin", 128))

    def _mat_expand(self, cs: _ConvSpec) -> bool:
        """A bottleneck's expansion 1x1 conv (conv3, Co = 4 Ci) takes its input BN2+ReLU as a
        materialised tensor instead of in its operand prologue from ``mat_expand_min_cin`` input
        channels on: the short-K GEMM re-reads and re-transforms its A tile once per output
        column tile (34-46 % of its roofline, r4 per-op table), and the backward's weight gradient
        then reads the stored input with the LDS-DMA tiles instead of an X-operand prologue.
        Below that (layer1, Ci = 64) conv3's backward is the fused 1x1 kernel, which applies
        BN2 itself.  -0.3 ms/step (r4 optimisation log)."""
        cin, cout = cs.conv.in_channels, cs.conv.out_channels
        return cs.k == 1 and cout >= 4 * cin and cin >= self.mat_expand_min_cin

    def _lazy_bn3_ds_ok(self, b: _BlockSpec, tp: _BlockTape, aL: torch.Tensor, S: int) -> bool:
        L = len(b.convs) - 1
        if not (getattr(self, "lazy_bn3_ds", False) and L > 0 and self._bnb_ok(b.convs[L], aL, S)):
            return False
        if not getattr(self, "_lazy_bn3_ds_dual_only", True):
            return True
        xin, pro_ss = tp.ins[L]
        return self._bwd1x1_ok(b.convs[L], aL, xin, pro_ss, tp.acts[L - 1], S)

    def _patch_bnb_ok(self, ops, cs: _ConvSpec, a: torch.Tensor, S: int) -> bool:
        """Can conv ``cs`` (output ``a``) take its output gradient's BatchNorm backward in the
        dgrad prologue of the LDS-resident-patch kernel (3x3 / stride 1 / pad 1, the second
        operand fits the kernel's register stage) and store it for the weight gradient?"""
        if not (self.patch_bnb and a.is_cuda and cs.k == 3 and cs.stride == 1 and cs.pad == 1):
            return False
        Nb, H, W, C = a.shape
        M = Nb * H * W
        if M % S or (M // S) % 256:
            return False
        Ci = cs.conv.in_channels
        key = (Nb, H, W, C, Ci)
        cache = self.__dict__.setdefault("_patch_bnb_cache", {})
        if key not in cache:
            g = [Nb, H, W, C, H, W, 3, 3, 1, 1, 1, 1, -1, -1, Ci, H, W, 1, 1, 0, 0, Ci]
            cache[key] = any(ops.igemm_variant_patch(v) and ops.igemm_variant_ok(v, g, True, True)
                             for v in range(ops.igemm_nvariants()))
        return cache[key]

    def _lazy_bn1_ok(self, b: _BlockSpec, a1: torch.Tensor, S: int) -> bool:
        """BN1's backward applied in conv1's dgrad / weight-gradient operand prologues instead
        of a materialising pass (a bottleneck's 1x1 stride-1 conv1)."""
        cs0 = b.convs[0]
        M = a1.numel() // a1.shape[-1]
        return (getattr(self, "lazy_bn1", False) and cs0.k == 1 and cs0.stride == 1
                and M % S == 0 and (M // S) % 256 == 0)

    def _dgrad(self, ops, dyn, cs: _ConvSpec, in_shape, S: int, accumulate: bool = False,
               dx: Optional[torch.Tensor] = None, bn_epi: Optional[Tuple] = None,
               bnb: Optional[Tuple] = None, compact: bool = False,
               sub_resid: bool = False, bnb_out: Optional[torch.Tensor] = None):
        """dx (NHWC) = conv-transpose(dy).  ``accumulate``: dx += result (dx must be given).

        ``bn_epi`` selects a BatchNorm-backward epilogue that also returns Σg, Σg·x̂ partials
        (segment-major across stride-2 parity classes) → (dx, partial, blocks_per_segment):
          ("mask", a_prev, bn_state)      mode 3: g = dx·[bn(a_prev) > 0] (BN+ReLU producer)
          ("res", resid, mask, a_prev, mi, ad, mid)
                                          mode 4: g = (dx + resid)·[y > 0] (residual-block
                                          producer: mask = its output's ReLU bitmask, a_prev =
                                          its last pre-BN activation; resid may alias dx); with
                                          ``ad`` (the producer's downsample pre-BN activation)
                                          the partials of its downsample BN too → (p3, pd)
        ``bnb = (a, coef)`` (1x1 stride-1; 3x3 stride-1 on the patch kernel with ``bnb_out``):
        the A operand is the BatchNorm backward coef.A·dyn + coef.B·a + coef.D computed in the
        prologue; ``bnb_out`` receives that operand (the weight gradient's dY).
        ``compact`` (stride-2 1x1, pad 0): return the dgrad only at the even input positions, as
        a dense [N, ceil(H/2), ceil(W/2), Ci] tensor (one stride-1 GEMM, no zero fill).
        ``sub_resid``: the residual (``dx`` with ``accumulate``, or bn_epi's resid) is such a
        compact tensor; the epilogue adds it at the even positions and dx is a new tensor.
        """
        Nb, H, W, Ci = in_shape
        _, OH, OW, Co = dyn.shape
        KH = KW = cs.k
        dev = dyn.device
        w = shadow_ohwi(cs.conv.weight, Ci)
        if compact:
            assert cs.stride == 2 and KH == 1 and cs.pad == 0 and bn_epi is None
            assert not accumulate and (OH, OW) == ((H + 1) // 2, (W + 1) // 2)
            dc = _empty_nhwc(Nb, OH, OW, Ci, dev)
            wt = self._dgrad_weight(ops, cs, w, (0, 0), [Co, 1, 1, Ci, 1, 1, 0, 2, 0, 2])
            g = [Nb, OH, OW, Co, OH, OW, 1, 1, 1, 1, 1, 1, 0, 0, Ci, OH, OW, 1, 1, 0, 0, Ci]
            v = igemm_choose(ops, dyn, wt, dc, g)
            igemm_launch(ops, dyn, wt, dc, g, v)
            return dc, None, 0
        resid_c = None
        if sub_resid:
            assert cs.stride == 1 and (accumulate or bn_epi is not None)
            resid_c = dx if bn_epi is None else bn_epi[1]
            dx = None  # the full-resolution result is a new tensor
        if dx is None:
            dx = _empty_nhwc(Nb, H, W, Ci, dev)
        launches = []
        if cs.stride == 1:
            wt = self._dgrad_weight(ops, cs, w, (0, 0),
                                    [Co, KH, KW, Ci, KH, KW, KH - 1, -1, KW - 1, -1])
            g = [Nb, OH, OW, Co, H, W, KH, KW, 1, 1, 1, 1, -(KH - 1 - cs.pad),
                 -(KW - 1 - cs.pad), Ci, H, W, 1, 1, 0, 0, Ci]
            launches.append((wt, g, Nb * H * W))
        else:
            assert cs.stride == 2
            zero_needed = False
            for r in (0, 1):
                for c in (0, 1):
                    kh0, kw0 = (r + cs.pad) % 2, (c + cs.pad) % 2
                    nkh = (KH - kh0 + 1) // 2 if kh0 < KH else 0
                    nkw = (KW - kw0 + 1) // 2 if kw0 < KW else 0
                    ohc, owc = (H - r + 1) // 2, (W - c + 1) // 2
                    if ohc == 0 or owc == 0:
                        continue
                    if nkh == 0 or nkw == 0:
                        zero_needed = True
                        continue
                    wt = self._dgrad_weight(ops, cs, w, (r, c),
                                            [Co, KH, KW, Ci, nkh, nkw, kh0, 2, kw0, 2])
                    ih0 = (r + cs.pad - kh0) // 2
                    iw0 = (c + cs.pad - kw0) // 2
                    g = [Nb, OH, OW, Co, ohc, owc, nkh, nkw, 1, 1, -1, -1, ih0, iw0, Ci,
                         H, W, 2, 2, r, c, Ci]
                    launches.append((wt, g, Nb * ohc * owc))
            if zero_needed:
                assert bn_epi is None, "BN-epilogue dgrad needs every output position covered"
                if not accumulate:
                    dx.zero_()
        if bn_epi is None:
            epi = (1, dx, None) if accumulate else None
            if resid_c is not None:
                epi = (1 | _EPI_SUB, resid_c, None)
            for wt, g, M in launches:
                v = igemm_choose(ops, dyn, wt, dx, g, epi=epi)
                igemm_launch(ops, dyn, wt, dx, g, v, epi=epi)
            return dx, None, 0
        assert not accumulate
        if bn_epi[0] == "mask":
            _, a_prev, bs = bn_epi
            epi = (3, None, a_prev)
            tables = (bs.ss.view(-1), bs.mi)
        else:
            _, resid, mask, a_prev, mi, ad_prev, mid_prev = bn_epi
            epi = (4 | (_EPI_SUB if resid_c is not None else 0), resid, None, a_prev, mask)
            tables = (None, mi)
        chosen = []
        bpro = None
        if bnb is not None:
            assert cs.stride == 1 and len(launches) == 1 and (cs.k == 1 or bnb_out is not None)
            SC = S * dyn.shape[-1]
            c = bnb[1]
            bpro = (c[:SC], c[SC:2 * SC], c[2 * SC:], launches[0][2] // S, bnb[0])
        for wt, g, M in launches:
            seg = M // S
            v = igemm_choose(ops, dyn, wt, dx, g, want_stats=True, epi=epi, seg_rows=seg,
                             epi_tables=tables, bnb=bpro, patch_only=bnb_out is not None)
            chosen.append((wt, g, M, seg, ops.igemm_variant_bm(v), v))
        seg_blocks = sum(seg // bm for (_, _, _, seg, bm, _) in chosen)
        partial = torch.empty((S * seg_blocks * 2 * Ci,), device=dev, dtype=torch.float32)
        second, partial2 = None, None
        if bn_epi[0] == "res" and bn_epi[5] is not None:
            partial2 = torch.empty_like(partial)
            second = (bn_epi[5], bn_epi[6], partial2)
        base = 0
        for wt, g, M, seg, bm, v in chosen:
            igemm_launch(ops, dyn, wt, dx, g, v, stats=partial, epi=epi, seg_rows=seg,
                         epi_tables=tables, remap=(seg_blocks, base), second=second, bnb=bpro,
                         bnb_out=bnb_out)
            base += seg // bm
        if partial2 is not None:
            return dx, (partial, partial2), seg_blocks
        return dx, partial, seg_blocks

    # ------------------------------------------------------------------ dgrad weights
    @staticmethod
    def _wt_params(cs: _ConvSpec):
        """[(parity class, weight_transform params)] of a conv's dgrad: stride 1 → the flipped,
        transposed kernel; stride 2 → one sub-kernel per (row, col) parity class."""
        conv = cs.conv
        Co, Ci, KH, KW = conv.out_channels, conv.in_channels, cs.k, cs.k
        if cs.stride == 1:
            return [((0, 0), [Co, KH, KW, Ci, KH, KW, KH - 1, -1, KW - 1, -1])]
        out = []
        for r in (0, 1):
            for c in (0, 1):
                kh0, kw0 = (r + cs.pad) % 2, (c + cs.pad) % 2
                nkh = (KH - kh0 + 1) // 2 if kh0 < KH else 0
                nkw = (KW - kw0 + 1) // 2 if kw0 < KW else 0
                if nkh and nkw:
                    out.append(((r, c), [Co, KH, KW, Ci, nkh, nkw, kh0, 2, kw0, 2]))
        return out

    def prepare_backward(self, ops) -> None:
        """Transform every conv's dgrad weights in ONE launch (weights change only at the
        optimizer step).  Needs flat-store-bound bf16 shadows (stable addresses); the plan is
        built eagerly once and rebuilt if the shadows move — never during graph capture."""
        convs = [cs for b in self.blocks for cs in (b.convs + ([b.down] if b.down else []))]
        shadows = []
        for cs in convs:
            slot = getattr(cs.conv.weight, "_slot", None)
            if slot is None or slot.shadow is None:
                self._wt_ready = False
                return
            shadows.append(slot.shadow)
        sig = tuple(t.data_ptr() for t in shadows)
        if sig != self._wt_sig:
            if torch.cuda.is_current_stream_capturing():
                self._wt_ready = False
                return
            Ws, Wts, params, cache = [], [], [], {}
            for cs, w in zip(convs, shadows):
                for key, p in self._wt_params(cs):
                    wt = torch.empty((p[3], p[4], p[5], p[0]), device=w.device,
                                     dtype=torch.bfloat16)
                    Ws.append(w)
                    Wts.append(wt)
                    params.extend(p)
                    cache[(id(cs.conv), key)] = wt
            plan = ops.weight_transform_plan(Ws, Wts, params)
            self._wt_table = (plan[:-1].to(shadows[0].device), int(plan[-1]), Ws)
            self._wt_cache = cache
            self._wt_sig = sig
        ops.weight_transform_batch(self._wt_table[0], self._wt_table[1])
        self._wt_ready = True

    def _prefetch_dgrad_weights(self, ops, xn: torch.Tensor) -> None:
        """The batched dgrad-weight transform (prepare_backward) depends only on the weights, which
        are final once the previous optimizer step ran: issue it on the (idle during the forward)
        weight-gradient stream at the start of the forward, so it is off the critical path of
        the backward, which waits on its event."""
        self._wt_event = None
        if not (self.wgrad_stream and xn.is_cuda):
            return
        dev = xn.device
        if self._side is None or self._side.device != dev:
            self._side = torch.cuda.Stream(device=dev)
        self._side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self._side):
            self.prepare_backward(ops)
        if self._wt_ready:
            ev = torch.cuda.Event()
            ev.record(self._side)
            self._wt_event = ev

    def _dgrad_weight(self, ops, cs: _ConvSpec, w, key, p):
        if getattr(self, "_wt_ready", False):
            wt = self._wt_cache.get((id(cs.conv), key))
            if wt is not None and wt.shape[0] == p[3]:
                return wt
        wt = torch.empty((p[3], p[4], p[5], p[0]), device=w.device, dtype=torch.bfloat16)
        ops.weight_transform(w, wt, p)
        return wt

    # ------------------------------------------------------------------ forward / backward
    def forward(self, xn: torch.Tensor) -> Tuple[torch.Tensor, List[_BlockTape]]:
        ops = _ext.ops()
        st = pstate.get()
        S = self.S
        self.calls += 1
        tapes: List[_BlockTape] = []
        x = xn
        self._prefetch_dgrad_weights(ops, xn)
        br = self._branch_stream(xn)
        pend = None  # the previous block's output, not yet formed: (aL, ss, res, rss, out, mask)
        for b in self.blocks:
            tp = _BlockTape(x=x)
            pro_ss = None
            cur = x
            dual = None
            if pend is not None:
                if self._dual_ok(ops, x, b.convs[0], S):
                    dual = pend  # formed (and written to x) by this block's conv1 prologue
                else:
                    self._out_apply(ops, pend, S)
                pend = None
            forked = False

            def fork_down():
                # the downsample conv + BN only meet the main branch at the block output; their
                # statistics all-reduce uses its own communicator (no ordering with the main's)
                br.wait_stream(torch.cuda.current_stream(x.device))
                with torch.cuda.stream(br):
                    self._down_fwd(ops, b, tp, x, S, st, slot=1)

            if b.down is not None and br is not None and dual is None:
                fork_down()
                forked = True
            for ci_, cs in enumerate(b.convs):
                _ext.TAG = f"{b.name} conv{ci_ + 1} fwd"
                if pro_ss is not None and (cs.k > 1 or self._mat_expand(cs)):
                    # a k x k conv re-gathers every input pixel k² times: applying BN+ReLU in
                    # its prologue costs more VALU work than one materialising pass (measured,
                    # also for the LDS-resident patch kernels: r3 optimisation log); likewise
                    # the short-K expansion convs (_mat_expand)
                    bmat = torch.empty_like(cur)
                    ops.bn_apply_ss(cur, pro_ss, None, None, bmat, S, True)
                    cur, pro_ss = bmat, None
                tp.ins.append((cur, pro_ss))
                if ci_ == 0 and dual is not None:
                    a, bs = self._conv_bn_fwd(ops, cur, cs, None, S, st, dual=dual)
                    self.dual_launches += 1
                    if b.down is not None and br is not None:
                        fork_down()  # after the launch that writes its input x
                        forked = True
                else:
                    a, bs = self._conv_bn_fwd(ops, cur, cs, pro_ss, S, st)
                tp.acts.append(a)
                tp.bns.append(bs)
                cur, pro_ss = a, bs.ss
            aL, bsL = tp.acts[-1], tp.bns[-1]
            out = torch.empty_like(aL)
            # the next block's input-gradient epilogue only needs [out > 0]: 1 bit per element
            mask = torch.empty((aL.numel() // 8,), device=aL.device, dtype=torch.uint8)
            _ext.TAG = f"{b.name} ds fwd"
            if b.down is not None:
                if forked:
                    torch.cuda.current_stream(x.device).wait_stream(br)  # join
                else:
                    self._down_fwd(ops, b, tp, x, S, st)
                pend = (aL, bsL.ss, tp.ad, tp.bnd.ss, out, mask)
            else:
                pend = (aL, bsL.ss, x, None, out, mask)
            tp.out = out
            tp.mask = mask
            tapes.append(tp)
            x = out
        if pend is not None:
            self._out_apply(ops, pend, S)
        _ext.TAG = ""
        return x, tapes

    def stem_forward(self, img: torch.Tensor):
        """Stem conv (statistics epilogue) → BatchNorm finalize → BN + ReLU apply with the
        ReLU bitmask (the stem is the producer of layer1.0 like one block of another), then the
        blocks.  Returns (output, tapes, stem tape)."""
        ops = _ext.ops()
        st = pstate.get()
        S = self.S
        cs = self.stem
        _ext.TAG = "stem fwd"
        a, bs = self._conv_bn_fwd(ops, img, cs, None, S, st)
        if self.stem_pool is not None:
            # maxpool(relu(bn(a))) in one pass; the full-resolution BN output is never written
            K, Sd, P = self.stem_pool
            Nb, OH, OW, C = a.shape
            PH, PW = (OH + 2 * P - K) // Sd + 1, (OW + 2 * P - K) // Sd + 1
            x0 = _empty_nhwc(Nb, PH, PW, C, a.device)
            arg = torch.empty(x0.shape, device=a.device, dtype=torch.uint8)
            asel = torch.empty_like(x0)
            _ext.TAG = "stem bn+relu+maxpool"
            ops.bn_relu_maxpool(a, bs.ss.view(-1), S, x0, arg, asel, K, Sd, P)
            tp = _BlockTape(x=img, acts=[a], bns=[bs], out=x0, pool=(arg, asel))
        else:
            x0 = torch.empty_like(a)
            mask = torch.empty((a.numel() // 8,), device=a.device, dtype=torch.uint8)
            ops.bn_apply_ss(a, bs.ss, None, None, x0, S, True, mask)
            tp = _BlockTape(x=img, acts=[a], bns=[bs], out=x0, mask=mask)
        out, tapes = self.forward(x0)
        return out, tapes, tp

    def _out_apply(self, ops, pend, S: int) -> None:
        """Block output = relu(bn3(aL) + shortcut) and its ReLU bitmask, as its own pass."""
        aL, ss, res, rss, out, mask = pend
        self.out_apply_calls += 1
        ops.bn_apply_ss(aL, ss, res, rss, out, S, True, mask)

    def _branch_stream(self, t: torch.Tensor):
        if not (getattr(self, "branch_stream", False) and t.is_cuda):
            return None
        if self._branch is None or self._branch.device != t.device:
            self._branch = torch.cuda.Stream(device=t.device)
        return self._branch

    def _down_fwd(self, ops, b: _BlockSpec, tp: _BlockTape, x, S: int, st, slot: int = 0):
        tp.ad, tp.bnd = self._conv_bn_fwd(ops, x, b.down, None, S, st, slot=slot)

    def backward(self, gout: torch.Tensor, tapes: List[_BlockTape],
                 stem_tape: Optional[_BlockTape] = None) -> Optional[torch.Tensor]:
        """Gradient w.r.t. the executor input, or None with ``stem_tape`` (the stem's
        parameter gradients are delivered and the image needs none)."""
        ops = _ext.ops()
        st = pstate.get()
        S = self.S
        ev = getattr(self, "_wt_event", None)
        if ev is not None and self._wt_ready:
            torch.cuda.current_stream(gout.device).wait_event(ev)  # transposed during the forward
        else:
            self.prepare_backward(ops)
        self._wt_event = None
        main = None
        if self.wgrad_stream and gout.is_cuda:
            main = torch.cuda.current_stream(gout.device)
            if self._side is None or self._side.device != gout.device:
                self._side = torch.cuda.Stream(device=gout.device)
            store = self._flat_store()
            if store is not None:
                store.producer_streams = [main, self._side]
        g, pre = gout, None
        pooled = stem_tape is not None and stem_tape.pool is not None
        # a pooled stem is not a block-boundary producer (the max-pool sits between its BN and
        # layer1.0): layer1.0 returns the raw gradient of the pooled map
        stem_prev = (self._stem_block, stem_tape) if (stem_tape is not None and not pooled) \
            else None
        hook = getattr(self.resnet, "stage_grads_ready", None) if main is not None else None
        for idx in range(len(self.blocks) - 1, -1, -1):
            prev = (self.blocks[idx - 1], tapes[idx - 1]) if idx > 0 else stem_prev
            g, pre = self._block_backward(ops, st, S, self.blocks[idx], tapes[idx], g, pre, prev)
            stage = _stage_of(self.blocks[idx])
            if hook is not None and stage >= 2 and _stage_of(self.blocks[idx - 1]) != stage:
                # the stage's first block is done: every weight gradient of the stage is queued
                # on the side stream and every BN parameter gradient written on this one (its
                # last BN backward finished at the start of this block): its optimizer update
                # can run beside the rest of the backward instead of in the step's tail
                self._side.wait_stream(main)
                with torch.cuda.stream(self._side):
                    hook(stage)
        if pooled:
            # g = dL/d(pooled map).  BatchNorm partials from pooled-size tensors (g is zero off
            # the window argmaxes; relu'(y[argmax]) = [pooled > 0]), then ONE full-resolution
            # pass: max-pool backward + ReLU mask + BN input gradient (k_maxpool_bwd_bn)
            _ext.TAG = "stem bwd"
            arg, asel = stem_tape.pool
            a0, bs0, x0 = stem_tape.acts[0], stem_tape.bns[0], stem_tape.out
            C = a0.shape[-1]
            nblk = ops.bn_blocks(x0.numel() // C, C, S)
            partial = torch.empty((S * nblk * 2 * C,), device=a0.device, dtype=torch.float32)
            ops.bn_bwd_reduce(g, x0, asel, bs0.mi, S, True, partial)
            coef = self._bn_bwd(ops, self.stem.bn, partial, nblk, bs0, S, st)
            da = torch.empty_like(a0)
            K, Sd, P = self.stem_pool
            ops.maxpool_bwd_bn(g, arg, x0, a0, coef, S, da, K, Sd, P)
            _ext.TAG = "stem wgrad"
            self._wgrad(ops, da, stem_tape.x, self.stem, None, S, main=True)
            _ext.TAG = ""
            g = None
        elif stem_tape is not None:
            # g = dL/d(stem output)·[y > 0] with the stem BatchNorm's partials from layer1.0's
            # conv1 dgrad epilogue: finish its backward, weight gradient with the BN backward in
            # the dY prologue (da never materialised)
            _ext.TAG = "stem bwd"
            coef = self._bn_bwd_finish(ops, pre[0], S)
            _ext.TAG = "stem wgrad"
            # on the main stream: nothing else is left for it, while the weight-gradient stream
            # still works through layer1.0's (the tail of the step runs both side by side)
            self._wgrad(ops, g, stem_tape.x, self.stem, None, S, bnb=(stem_tape.acts[0], coef),
                        main=True)
            _ext.TAG = ""
            g = None
        if main is not None:
            if store is not None and getattr(store, "defer_side_join", False):
                # joined in store.finish(), after the stem's backward
                keep, self._side_keep = self._side_keep, []
                store.defer_join(self._side, keep)
            else:
                main.wait_stream(self._side)  # join: every weight gradient is in the flat buffer
                self._side_keep.clear()
        self._wt_ready = False  # the optimizer step changes the weights
        return g

    def _flat_store(self):
        for b in self.blocks:
            slot = getattr(b.convs[0].conv.weight, "_slot", None)
            if slot is not None:
                return slot.store
        return None

    def _block_backward(self, ops, st, S, b: _BlockSpec, tp: _BlockTape, g: torch.Tensor,
                        pre, prev):
        """``g`` = dL/d(block output).  ``pre = None``: g is the raw gradient; otherwise g is
        already ReLU-masked and ``pre`` is the started BN backward (``_bn_bwd_start``) of this
        block's last BN, whose Σg, Σg·x̂ partials the following block's dgrad epilogue
        produced.  Returns the same pair for the block input: masked + started when the
        producer is another block of this executor (``prev``), raw otherwise.

        Every BN all-reduce (distributed) is started before an independent weight-gradient
        kernel and finished after it, so its latency hides behind the wgrad."""
        out = tp.out
        L = len(b.convs) - 1
        _ext.TAG = f"{b.name} bn{L + 1} bwd"
        aL, bsL = tp.acts[L], tp.bns[L]
        C = aL.shape[-1]
        R = aL.numel() // C
        dev = aL.device
        da = torch.empty_like(aL)
        lazy = None
        if pre is None:
            nblk = ops.bn_blocks(R, C, S)
            partial = torch.empty((S * nblk * 2 * C,), device=dev, dtype=torch.float32)
            ops.bn_bwd_reduce(g, out, aL, bsL.mi, S, True, partial)
            coefL = self._bn_bwd(ops, b.convs[L].bn, partial, nblk, bsL, S, st)
            g3 = torch.empty_like(out)
            ops.bn_bwd_apply(g, out, aL, coefL, S, True, da, g3)  # g3 = g·[out > 0]
        else:
            g3 = g
            h3, hd = pre
            coefL = self._bn_bwd_finish(ops, h3, S)
            if hd is None:
                if L > 0 and self._bnb_ok(b.convs[L], aL, S):
                    lazy = (aL, coefL)  # da never materialised: conv L's operand prologues
                else:
                    ops.bn_bwd_apply(g3, None, aL, coefL, S, False, da, None)
        dad = None
        ds_dual = None  # (g3, coefd): the downsample's backward as one fused pass (_ds_dual)
        if b.down is not None:
            _ext.TAG = f"{b.name} bnds bwd"
            if pre is not None and hd is not None:
                # both BNs of the block output from one pass over g3 (their partials came
                # from the following block's dgrad epilogue) — or only the downsample BN's,
                # with BN3's backward left to conv3's operand prologues
                coefd = self._bn_bwd_finish(ops, hd, S)
                if self._lazy_bn3_ds_ok(b, tp, aL, S):
                    lazy = (aL, coefL)
                    if self._ds_dual_ok(b, tp, S):
                        ds_dual = (g3, coefd)  # dad never materialised
                    else:
                        dad = torch.empty_like(tp.ad)
                        ops.bn_bwd_apply(g3, None, tp.ad, coefd, S, False, dad, None)
                else:
                    dad = torch.empty_like(tp.ad)
                    ops.bn_bwd_apply2(g3, aL, coefL, da, tp.ad, coefd, dad, S)
            else:
                dad = torch.empty_like(tp.ad)
                nblk_d = ops.bn_blocks(R, C, S)
                partial_d = torch.empty((S * nblk_d * 2 * C,), device=dev, dtype=torch.float32)
                ops.bn_bwd_reduce(g3, None, tp.ad, tp.bnd.mi, S, False, partial_d)
                coefd = self._bn_bwd(ops, b.down.bn, partial_d, nblk_d, tp.bnd, S, st)
                if pre is not None:
                    ops.bn_bwd_apply2(g3, aL, coefL, da, tp.ad, coefd, dad, S)
                else:
                    ops.bn_bwd_apply(g3, None, tp.ad, coefd, S, False, dad, None)
        resid_f = None
        # (bottleneck blocks: conv1 is 1x1 stride 1, so its dgrad epilogue covers every input
        # position; a BasicBlock's conv1 carries the stride itself)
        compact = (b.down is not None and self.compact_ds and b.down.stride == 2 and b.down.k == 1
                   and b.down.pad == 0 and b.convs[0].stride == 1)
        br = self._branch_stream(tp.ad) if b.down is not None else None
        if ds_dual is not None:
            if br is not None and getattr(self, "ds_dual_stream", "main") == "branch":
                br.wait_stream(torch.cuda.current_stream(tp.ad.device))
                with torch.cuda.stream(br):
                    resid_f = self._ds_dual(ops, b, tp, ds_dual, S)
            else:
                resid = self._ds_dual(ops, b, tp, ds_dual, S)
        elif br is not None:
            # the downsample dgrad only meets the conv chain at conv1's dgrad epilogue
            br.wait_stream(torch.cuda.current_stream(dad.device))
            with torch.cuda.stream(br):
                _ext.TAG = f"{b.name} ds dgrad"
                resid_f, _, _ = self._dgrad(ops, dad, b.down, tp.x.shape, S, compact=compact)
        # conv chain, last to first: dgrad (+ BN-bwd partials) → start BN all-reduce → wgrad →
        # finish BN → apply
        lazy0 = None
        pend = None  # (g, a, coef): the BN backward feeding conv i, left to its patch dgrad
        for i in range(L, 0, -1):
            cs = b.convs[i]
            xin, pro_ss = tp.ins[i]
            a_prev, bs_prev = tp.acts[i - 1], tp.bns[i - 1]
            _ext.TAG = f"{b.name} conv{i + 1} dgrad"
            dyn, bnb = (g3, lazy) if (i == L and lazy is not None) else (da, None)
            if pend is not None:
                # dgrad with the BN backward in its patch prologue; that operand is stored as
                # the weight gradient's dY on the way (no separate bn_bwd_apply pass)
                gsrc, a_b, coef_b = pend
                pend = None
                dy_m = torch.empty_like(a_b)
                gm, part, nb = self._dgrad(ops, gsrc, cs, a_prev.shape, S,
                                           bn_epi=("mask", a_prev, bs_prev), bnb=(a_b, coef_b),
                                           bnb_out=dy_m)
                h = self._bn_bwd_start(ops, b.convs[i - 1].bn, part, nb, bs_prev, S, st)
                _ext.TAG = f"{b.name} conv{i + 1} wgrad"
                self._wgrad(ops, dy_m, xin, cs, pro_ss, S)
            elif self._bwd1x1_ok(cs, dyn, xin, pro_ss, a_prev, S):
                _ext.TAG = f"{b.name} conv{i + 1} dgrad+wgrad"
                gm, part, nb = self._bwd1x1_fused(ops, dyn, bnb, cs, a_prev, bs_prev, S, xin)
                h = self._bn_bwd_start(ops, b.convs[i - 1].bn, part, nb, bs_prev, S, st)
            else:
                gm, part, nb = self._dgrad(ops, dyn, cs, a_prev.shape, S,
                                           bn_epi=("mask", a_prev, bs_prev), bnb=bnb)
                h = self._bn_bwd_start(ops, b.convs[i - 1].bn, part, nb, bs_prev, S, st)
                _ext.TAG = f"{b.name} conv{i + 1} wgrad"
                self._wgrad(ops, dyn, xin, cs, pro_ss, S, bnb=bnb)
            _ext.TAG = f"{b.name} bn{i} bwd"
            coef = self._bn_bwd_finish(ops, h, S)
            if i == 1 and prev is not None and self._lazy_bn1_ok(b, a_prev, S):
                lazy0 = (a_prev, coef)  # da1 never materialised: conv1's operand prologues
                da = gm
                continue
            if i - 1 >= 1 and self._patch_bnb_ok(ops, b.convs[i - 1], a_prev, S):
                pend = (gm, a_prev, coef)
                continue
            da_next = torch.empty_like(a_prev)
            ops.bn_bwd_apply(gm, None, a_prev, coef, S, False, da_next, None)
            da = da_next
        cs0 = b.convs[0]
        if b.down is not None:
            if resid_f is not None:
                torch.cuda.current_stream(tp.ad.device).wait_stream(br)  # join
                resid = resid_f
            elif ds_dual is None:
                _ext.TAG = f"{b.name} ds dgrad"
                resid, _, _ = self._dgrad(ops, dad, b.down, tp.x.shape, S, compact=compact)
        else:
            resid = g3
        _ext.TAG = f"{b.name} conv1 dgrad"
        if prev is None:
            dx, _, _ = self._dgrad(ops, da, cs0, tp.x.shape, S, accumulate=True, dx=resid,
                                   sub_resid=compact)
            h = None
        else:
            pb, ptp = prev
            pds = pb.down is not None
            dx, part, nb = self._dgrad(ops, da, cs0, tp.x.shape, S, bnb=lazy0,
                                       dx=resid if b.down is not None and not compact else None,
                                       sub_resid=compact,
                                       bn_epi=("res", resid, ptp.mask, ptp.acts[-1],
                                               ptp.bns[-1].mi, ptp.ad if pds else None,
                                               ptp.bnd.mi if pds else None))
            if pds:
                p3, pd = part
                h = (self._bn_bwd_start(ops, pb.convs[-1].bn, p3, nb, ptp.bns[-1], S, st),
                     self._bn_bwd_start(ops, pb.down.bn, pd, nb, ptp.bnd, S, st))
            else:
                h = (self._bn_bwd_start(ops, pb.convs[-1].bn, part, nb, ptp.bns[-1], S, st), None)
        _ext.TAG = f"{b.name} conv1 wgrad"
        self._wgrad(ops, da, tp.x, cs0, None, S, bnb=lazy0)
        if b.down is not None and ds_dual is None:
            _ext.TAG = f"{b.name} ds wgrad"
            self._wgrad(ops, dad, tp.x, b.down, None, S)
        _ext.TAG = ""
        return dx, h


class FusedStemStagesFn(torch.autograd.Function):
    """Autograd boundary around stem + executor: input = the image batch (channels_last bf16,
    no gradient), output = last block output; every parameter gradient bypasses autograd (flat
    store).  ``anchor`` (the stem weight) makes autograd call the backward."""

    @staticmethod
    def forward(ctx, img, anchor, ex: FusedStages):
        xn = img.permute(0, 2, 3, 1)
        if not xn.is_contiguous():
            xn = img.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
        out, tapes, stem_tape = ex.stem_forward(xn)
        ctx.ex = ex
        ctx.tapes = tapes
        ctx.stem_tape = stem_tape
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gout):
        if gout.dtype != torch.bfloat16:
            gout = gout.to(torch.bfloat16)
        gn = gout.permute(0, 2, 3, 1)
        if not gn.is_contiguous():
            gn = gout.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
        ctx.ex.backward(gn, ctx.tapes, ctx.stem_tape)
        ctx.tapes = None
        ctx.stem_tape = None
        return None, None, None


class FusedStagesFn(torch.autograd.Function):
    """Autograd boundary around the executor: input = stem output (channels_last bf16),
    output = last block output; parameter gradients bypass autograd (flat store)."""

    @staticmethod
    def forward(ctx, x, anchor, ex: FusedStages):
        xn = x.permute(0, 2, 3, 1)
        if not xn.is_contiguous():
            xn = x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
        out, tapes = ex.forward(xn)
        ctx.ex = ex
        ctx.tapes = tapes
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gout):
        if gout.dtype != torch.bfloat16:
            gout = gout.to(torch.bfloat16)
        gn = gout.permute(0, 2, 3, 1)
        if not gn.is_contiguous():
            gn = gout.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
        dx = ctx.ex.backward(gn, ctx.tapes)
        ctx.tapes = None
        return dx.permute(0, 3, 1, 2), None, None
