"""Replay modes of a captured training step.

``torch.cuda.CUDAGraph(keep_graph=True)`` keeps the captured ``hipGraph_t``; besides the HIP
graph executor (``graph.replay()``) the step can be issued by the native multi-stream executor in
``csrc/graphexec.cpp``: it walks the captured nodes in capture order and launches each one with
its own captured arguments on up to ``max_streams`` HIP streams, turning cross-stream edges into
events.  That keeps the eager schedule's side-stream concurrency (weight gradients beside the
dgrad / BatchNorm chain) at ~one ``hipLaunchKernel`` of host time per kernel instead of the ~30 µs
of Python + dispatcher work of eager issue.

There is no reference counterpart (the reference issues every op eagerly through autograd:
``/root/reference/main.py:104-122``); this is the MI355X-native answer to its per-op launch cost.
"""
from __future__ import annotations

import torch

from ..ops import _ext

STAT_NAMES = ("kernels", "subgraphs", "memsets", "host", "empty", "event_records", "event_waits",
              "cross_stream_waits", "streams", "events")


class StreamReplay:
    """Native multi-stream issue of the nodes of ``graph`` (a ``CUDAGraph(keep_graph=True)``
    after ``capture_end``).  The CUDAGraph object must stay alive while this is used."""

    def __init__(self, graph: torch.cuda.CUDAGraph, max_streams: int = 3):
        _ext.require()
        self._ops = torch.ops.simclr_amd
        self.graph = graph
        self.handle = int(self._ops.gexec_create(int(graph.raw_cuda_graph()), int(max_streams)))

    def stats(self) -> dict:
        return dict(zip(STAT_NAMES, (int(v) for v in self._ops.gexec_stats(self.handle))))

    def schedule(self):
        """[(stream, node kind)] per issued node, in issue order."""
        return [(int(v) // 16, int(v) % 16) for v in self._ops.gexec_streams(self.handle)]

    def replay(self) -> None:
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
