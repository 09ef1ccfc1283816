"""One-shot cross-rank exchange of BatchNorm statistics through IPC-mapped device memory.

Reference behaviour replaced: SyncBatchNorm issues an ``all_gather`` of [mean‖invstd‖count]
per BN layer per forward and an ``all_reduce`` of [Σdy‖Σdy·x̂] per BN layer in backward
(/root/reference/main.py:176 → torch/nn/modules/_functions.py:74,159): ~2x53 latency-bound
collectives per ResNet-50 step, each a separate NCCL launch on the critical path.
The RCCL path of this framework already halves that (one all-reduce of both views' [Σ, Σ²]
per layer, csrc/bn.hip + models/fused.py); this module removes the collective launches
altogether on a single node: the fused BN reduce kernel that finalizes a layer's statistics
pushes its local sums straight into every peer's arena over xGMI and sums the W slots of its
own arena in rank order (csrc/bn.hip ``bn_ipc_exchange``) — one kernel per BatchNorm, no
RCCL, no host involvement, capturable in the step's hipGraph, bitwise-identical statistics on
every rank.

Arena layout: int64 words; every BatchNorm site (a (module name, direction, shape) key —
``site_key``: the module's qualified name inside its model, so a model rebuilt in the same
process reuses its sites instead of leaking arena space — allocated in first-call order, which
is identical on all ranks of an SPMD step) owns
``2 parities x world x [2][S][C]`` words at the same offset in every rank's arena, and
``ceil(C/64)`` epoch counters in a local int32 buffer.

``setup_stats_exchange`` builds the exchange only when every rank can (same node, GPU,
world <= 16) and keeps it only if a self-test — two exchanges against host-computed sums —
passes on every rank; otherwise the step falls back to the RCCL statistics all-reduce.
"""
from __future__ import annotations

import os
import sys
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import _ext
from ..parallel.state import site_key, tag_sites  # noqa: F401

# 128 MiB arena: ResNet-50 fwd + bwd BatchNorm sites at W = 8 need ~30 MiB, the gathered
# NT-Xent's embedding all-gather and column-gradient reduce-scatter ~24 MiB more
DEFAULT_WORDS = 1 << 24
MAX_WORLD = 16


def region_words(world: int, S: int, C: int) -> int:
    """Words of one site's region (mirrors kernels.h bn_ipc_region_words)."""
    return 2 * world * 2 * S * C


class SiteTable:
    """Deterministic sub-allocation of arena regions and epoch counters (host-only logic)."""

    def __init__(self, world: int, words: int, epochs: int):
        self.world = world
        self.words = words
        self.epochs = epochs
        self.sites: Dict[object, Tuple[int, int, int, int]] = {}
        self.next_word = 0
        self.next_epoch = 0

    def get(self, key, S: int, C: int) -> Tuple[int, int, int]:
        """(word offset, epoch offset, epoch count) of ``key``'s region at shape (S, C),
        allocated on first use (the same name at another shape — e.g. ResNet-18 then ResNet-50
        in one process — gets a region of its own)."""
        key = (key, S, C)
        if key in self.sites:
            off, eo, ne, _ = self.sites[key]
            return off, eo, ne
        n = region_words(self.world, S, C)
        ne = (C + 63) // 64
        if self.next_word + n > self.words or self.next_epoch + ne > self.epochs:
            raise RuntimeError("IPC statistics arena exhausted "
                               f"({self.next_word + n} > {self.words} words)")
        rec = (self.next_word, self.next_epoch, ne, S * 100000 + C)
        self.sites[key] = rec
        self.next_word += n
        self.next_epoch += ne
        return rec[:3]

    def get_raw(self, key, words: int, nepochs: int) -> Tuple[int, int, int]:
        """A region of ``words`` words and ``nepochs`` epoch counters (the IPC collectives)."""
        key = ("raw", key, words, nepochs)
        if key in self.sites:
            off, eo, ne, _ = self.sites[key]
            return off, eo, ne
        if self.next_word + words > self.words or self.next_epoch + nepochs > self.epochs:
            raise RuntimeError("IPC arena exhausted "
                               f"({self.next_word + words} > {self.words} words)")
        rec = (self.next_word, self.next_epoch, nepochs, words)
        self.sites[key] = rec
        self.next_word += words
        self.next_epoch += nepochs
        return rec[:3]


class IpcStatsExchange:
    def __init__(self, rank: int, world: int, device: torch.device, group=None,
                 words: int = DEFAULT_WORDS, epochs: int = 1 << 16):
        if world > MAX_WORLD:
            raise ValueError(f"IPC exchange supports at most {MAX_WORLD} ranks")
        ops = _ext.ops()
        self.rank, self.world, self.device = rank, world, device
        self.arena = ops.ipc_arena_alloc(words, device.index)
        handle = ops.ipc_handle(self.arena)
        handles: List[Optional[bytes]] = [None] * world
        dist.all_gather_object(handles, bytes(handle.numpy().tobytes()), group=group)
        self._opened: List[int] = []
        ptrs = []
        for r, hb in enumerate(handles):
            if r == rank:
                ptrs.append(self.arena.data_ptr())
                continue
            p = ops.ipc_open(torch.frombuffer(bytearray(hb), dtype=torch.uint8), device.index)
            self._opened.append(p)
            ptrs.append(p)
        self.peers = torch.tensor(ptrs, dtype=torch.int64, device=device)
        self.epoch = torch.zeros(epochs, dtype=torch.int32, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.table = SiteTable(world, words, epochs)

    def kwargs(self, key, S: int, C: int) -> dict:
        """Extra arguments of ``bn_reduce_fused`` (modes 1 / 2) for site ``key``."""
        off, eo, ne = self.table.get(key, S, C)
        return dict(ipc_peers=self.peers, ipc_arena=self.arena, ipc_site=off,
                    ipc_epoch=self.epoch[eo:eo + ne], ipc_err=self.err, world=self.world,
                    rank=self.rank)

    def _collective(self, op: int, key, src: torch.Tensor, dst: torch.Tensor, n: int) -> None:
        ops = _ext.ops()
        nb = int(ops.ipc_coll_blocks())
        off, eo, ne = self.table.get_raw(key, 2 * self.world * n, nb)
        ops.ipc_collective(op, src, dst, self.peers, self.arena, off, self.epoch[eo:eo + ne],
                           self.err, self.world, self.rank)

    def all_gather(self, key, src: torch.Tensor, dst: torch.Tensor) -> None:
        """``dst`` ([W * len(src)], rank-major) = every rank's ``src`` — one kernel on the current
        stream, one-shot stores into every peer's arena (csrc/comm.hip).  Same contract as
        ``dist.all_gather_into_tensor``; ``key`` names the arena site (identical on all ranks)."""
        self._collective(0, key, src, dst, src.numel() * src.element_size() // 4)

    def reduce_scatter(self, key, src: torch.Tensor, dst: torch.Tensor) -> None:
        """``dst`` = Σ_r (rank r's ``src``)[rank-th slice], fp32, summed in rank order (the same
        bits on every rank).  Same contract as ``dist.reduce_scatter_tensor``."""
        assert src.dtype == torch.float32 and dst.dtype == torch.float32
        self._collective(1, key, src, dst, dst.numel())

    def failed(self) -> bool:
        """A spin timed out (a peer never delivered): the statistics of that step are wrong."""
        return bool(self.err.item())

    def close(self) -> None:
        ops = _ext.ops()
        for p in self._opened:
            try:
                ops.ipc_close(p)
            except Exception:
                pass
        self._opened = []

    # ------------------------------------------------------------------ self-test
    def selftest(self, rounds: int = 3) -> bool:
        """Exchange rank-dependent sums through a dedicated site ``rounds`` times (both arena
        parities) and compare the finalized mean / invstd with the host-computed values."""
        ops = _ext.ops()
        S, C, nblk = 2, 192, 3
        dev = self.device
        ok = True
        for it in range(rounds):
            c = torch.arange(C, dtype=torch.float64)
            part = torch.zeros(S, nblk, 2, C, dtype=torch.float64)
            tot1 = torch.zeros(S, C, dtype=torch.float64)
            tot2 = torch.zeros(S, C, dtype=torch.float64)
            for r in range(self.world):
                for s in range(S):
                    for b in range(nblk):
                        v1 = (r + 1) * 0.25 + s + 0.01 * c + b + it
                        v2 = v1 * v1 + 1.0 + 0.1 * r
                        if r == self.rank:
                            part[s, b, 0] = v1
                            part[s, b, 1] = v2
                        tot1[s] += v1
                        tot2[s] += v2
            count = float(nblk * self.world)
            mean = tot1 / count
            var = (tot2 / count - mean * mean).clamp_min(0)
            inv = 1.0 / torch.sqrt(var + 1e-5)
            mi = torch.empty(2 * S * C, dtype=torch.float32, device=dev)
            ops.bn_reduce_fused(part.float().reshape(-1).to(dev), nblk, S, C, 1, None, count,
                                1e-5, 0.1, None, None, mi, None, None, None, None, None, None,
                                None, 0, **self.kwargs("__selftest__", S, C))
            got = mi.view(2, S, C).double().cpu()
            ok = ok and torch.allclose(got[0], mean, rtol=1e-4, atol=1e-4) and \
                torch.allclose(got[1], inv, rtol=1e-3, atol=1e-3)
        torch.cuda.synchronize(dev)
        return ok and not self.failed()


def setup_stats_exchange(st, device: torch.device, mode: Optional[str] = None):
    """Attach an IPC statistics exchange to the parallel state ``st`` when it applies.

    ``mode`` (or ``SIMCLR_BN_COMM``): ``rccl`` (the default: the exchange has not yet been
    validated across two physical GPUs, so training keeps the RCCL statistics all-reduce unless
    asked), ``ipc`` always (raise if impossible), ``auto`` at world > 1 over RCCL (one GPU per
    rank) when the self-test passes on every rank — bench.py uses ``auto`` as a candidate that
    its collective probe times against RCCL.  ``auto`` skips the gloo rehearsals that put several
    ranks on ONE GPU: their processes' queues are time-sliced, so every exchange waits for a
    context switch (correct — tests/test_gpu_distributed.py runs it explicitly — but ~50 ms per
    BatchNorm)."""
    mode = (mode or os.environ.get("SIMCLR_BN_COMM", "rccl")).lower()
    st.ipc = None
    if mode == "rccl" or not st.comm or st.world_size < 2 or device.type != "cuda":
        if mode == "ipc" and st.world_size > 1 and device.type != "cuda":
            raise RuntimeError("SIMCLR_BN_COMM=ipc needs GPUs")
        return None
    if mode == "auto" and dist.get_backend(st.group) != "nccl":
        return None
    ex, ok = None, 0
    try:
        if st.world_size <= MAX_WORLD and _ext.available():
            ex = IpcStatsExchange(st.rank, st.world_size, device, group=st.group)
            ok = int(ex.selftest())
    except Exception as e:  # every rank takes the same decision below
        print(f"[ipc] rank {st.rank}: exchange setup failed: {e!r}", file=sys.stderr, flush=True)
        ok = 0
    flag = torch.tensor([ok], dtype=torch.int32,
                        device=device if dist.get_backend(st.group) == "nccl" else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=st.group)
    if int(flag.item()) != 1:
        if ex is not None:
            ex.close()
        if mode == "ipc":
            raise RuntimeError("IPC statistics exchange failed its self-test")
        print(f"[ipc] rank {st.rank}: IPC statistics exchange unavailable, using RCCL",
              file=sys.stderr, flush=True)
        return None
    st.ipc = ex
    return ex


def fallback_if_failed(st, device: torch.device) -> bool:
    """Collective check (call it on every rank, outside any captured region): if a spin of the
    IPC exchange timed out on some rank — e.g. one rank still autotuning a conv seconds after
    its peers reached the next BatchNorm — that step's statistics were partial and the sticky
    error flag makes later exchanges skip waiting.  Every rank then drops to the RCCL path
    (``st.ipc = None``; the same decision everywhere).  Returns True when it switched; a
    captured HIP graph holding the exchange must then be discarded by the caller."""
    if st.ipc is None:
        return False
    f = torch.tensor([1 if st.ipc.failed() else 0], dtype=torch.int32, device=device)
    dist.all_reduce(f, op=dist.ReduceOp.MAX, group=st.group)
    if int(f.item()) == 0:
        return False
    print(f"[ipc] rank {st.rank}: statistics exchange timed out; continuing with RCCL",
          file=sys.stderr, flush=True)
    st.ipc = None
    return True


class IpcExchangeError(RuntimeError):
    """An IPC BatchNorm-statistics exchange timed out: that step ran on partial statistics."""


# eager steps that run with the BatchNorm statistics on RCCL (not the IPC exchange): every rank
# autotunes its conv tiles during its first step(s), seconds apart, which would exceed the IPC
# exchange's 2 s spin bound; afterwards the ranks adopt rank 0's tuning table
TUNING_STEPS = 2


class StepGuard:
    """Wraps the eager training step of a loop that may use the IPC exchange.

    * the first ``TUNING_STEPS`` steps run with ``st.ipc`` detached (statistics over RCCL) and
      end with ``tuning.sync_from_rank0`` — identical tiles on every rank;
    * after every step the exchange's sticky error flag is all-reduced (MAX) across the ranks
      on the device — a rank whose late arrival made a PEER time out learns of it too — and
      copied into pinned host memory behind an event; the next step's check waits for that
      event (the previous step has finished on the device by then; the host stays one step
      ahead) and reads the flag: ``on_error="raise"`` raises ``IpcExchangeError`` on every rank
      no later than the step after the timeout (the fail-fast launcher then stops the job —
      training never runs on from partial statistics), ``"defer"`` leaves the check to the
      caller (bench.py)."""

    def __init__(self, st, on_error: str = "raise"):
        self.st = st
        self.on_error = on_error
        self.eager_steps = 0
        self._pending = None  # (host flag, event or None, step) of the last issued check
        self._bufs: List[torch.Tensor] = []

    def run(self, body, *a):
        if self.eager_steps >= TUNING_STEPS or not self.st.comm:
            self.eager_steps += 1
            return body(*a)
        ipc, self.st.ipc = self.st.ipc, None
        try:
            out = body(*a)
        finally:
            self.st.ipc = ipc
        self.eager_steps += 1
        from ..ops import tuning
        tuning.sync_from_rank0(self.st.group)
        return out

    def _land(self) -> None:
        """Wait for the previously issued flag copy and raise if any rank timed out."""
        if self._pending is None:
            return
        host, ev, s = self._pending
        self._pending = None
        if ev is not None:
            ev.synchronize()
        if self.on_error == "raise" and int(host[0]) != 0:
            raise IpcExchangeError(
                f"rank {self.st.rank}: IPC BatchNorm-statistics exchange timed out on some rank "
                f"at or before step {s}; stopping (that step's statistics were partial)")

    def check(self, step: int = -1) -> None:
        ipc = self.st.ipc
        if ipc is None:
            return
        self._land()
        cuda = ipc.err.is_cuda
        if not self._bufs:  # two pinned flags: the one being written is never the one read
            self._bufs = [torch.zeros(1, dtype=torch.int32, pin_memory=cuda) for _ in range(2)]
        host = self._bufs[step % 2 if step >= 0 else 0]
        flag = ipc.err.clone()
        if self.st.comm and dist.is_initialized():
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.st.group)
        host.copy_(flag, non_blocking=cuda)
        ev = None
        if cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(flag.device))
        self._pending = (host, ev, step)

    def flush(self, step: int = -1) -> None:
        """Check the last issued flag now (epoch end, before saving or exiting)."""
        self.check(step)
        self._land()
