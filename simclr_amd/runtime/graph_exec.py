"""Replay modes of a captured training step.

``torch.cuda.CUDAGraph(keep_graph=True)`` keeps the captured ``hipGraph_t``; besides the HIP
graph executor (``graph.replay()``) the step can be issued by the native multi-stream executor in
``csrc/graphexec.cpp``: it walks the captured nodes in capture order and launches each one with
its own captured arguments on up to ``max_streams`` HIP streams, turning cross-stream edges into
events.  That keeps the eager schedule's side-stream concurrency (weight gradients beside the
dgrad / BatchNorm chain) at ~one ``hipLaunchKernel`` of host time per kernel instead of the ~30 µs
of Python + dispatcher work of eager issue.

Single GPU (``sched="list"``, the default there): the first replay is a planning step — the
nodes run serially with a timing event after each one, and the executor re-plans its issue order
and stream assignment by list scheduling on those durations (every stream ordered by simulated
start time, so no node waits behind a later-ready one on its stream).

With collectives in the step (N > 1, or a forced 1-rank group) ``Trainer.capture`` keeps the
capture-order plan (``sched="capture"``): the all-reduce chain stays on a stream of its own and
every rank issues the collectives in the captured order.  The list schedule is opt-in there
(``SIMCLR_REPLAY_SCHED=list``); every rank then plans from rank 0's durations (one
``dist.broadcast`` inside the first replay) so the collectives keep one issue order.

There is no reference counterpart (the reference issues every op eagerly through autograd:
``/root/reference/main.py:104-122``); this is the MI355X-native answer to its per-op launch cost.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import _ext

STAT_NAMES = ("kernels", "subgraphs", "memsets", "host", "empty", "event_records", "event_waits",
              "cross_stream_waits", "streams", "events")


class StreamReplay:
    """Native multi-stream issue of the nodes of ``graph`` (a ``CUDAGraph(keep_graph=True)``
    after ``capture_end``).  The CUDAGraph object must stay alive while this is used."""

    def __init__(self, graph: torch.cuda.CUDAGraph, max_streams: int = 3,
                 sched: Optional[str] = None):
        _ext.require()
        self._ops = torch.ops.simclr_amd
        self.graph = graph
        self.max_streams = int(max_streams)
        self.handle = int(self._ops.gexec_create(int(graph.raw_cuda_graph()), self.max_streams))
        # "list" (default): the first replay runs serially with a timing event per node and the
        # executor re-plans its issue order / streams from those durations (gexec_reschedule:
        # -0.05 ms/step in 6 of 6 interleaved rounds); "capture": gexec_create's capture-order plan
        self.sched = sched or os.environ.get("SIMCLR_REPLAY_SCHED", "list")
        self._pending = self.sched == "list"
        self.durations: Optional[List[float]] = None

    def _plan(self) -> None:
        """Timed serial replay (one step) → list schedule.  Every rank plans from rank 0's
        durations, so collectives keep one issue order across ranks."""
        d = torch.tensor(self._ops.gexec_timed_replay(self.handle), dtype=torch.float64)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dev = torch.device("cuda", torch.cuda.current_device())
            t = d.to(dev)
            dist.broadcast(t, 0)
            d = t.cpu()
        self.durations = d.tolist()
        # 4 µs per cross-stream event; 4 streams or 1 / 12 µs measured the same (r5 log)
        self._ops.gexec_reschedule(self.handle, self.durations, self.max_streams, 4.0)

    def stats(self) -> dict:
        d = dict(zip(STAT_NAMES, (int(v) for v in self._ops.gexec_stats(self.handle))))
        d["sched"] = self.sched if not self._pending else self.sched + "(pending)"
        return d

    def schedule(self):
        """[(stream, node kind)] per issued node, in issue order."""
        return [(int(v) // 16, int(v) % 16) for v in self._ops.gexec_streams(self.handle)]

    @property
    def pending(self) -> bool:
        """The next replay is the timed planning replay."""
        return self._pending

    def replay(self) -> None:
        if self._pending:
            self._pending = False
            self._plan()
            return
        self._ops.gexec_replay(self.handle)

    def close(self) -> None:
        if self.handle:
            self._ops.gexec_destroy(self.handle)
            self.handle = 0

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass
