"""The replay executor's list schedule (csrc/graphexec.cpp ``list_schedule``, host-only code
exposed as ``gexec_list_schedule``) on synthetic DAGs: a valid topological issue order, at most
``max_streams`` streams, the critical chain kept on one stream, and no node queued behind a
later-ready node on its stream when another stream is free (the head-of-line blocking the
capture-order heuristic of ``gexec_create`` can produce)."""
import random
from pathlib import Path

import pytest
import torch

SO = Path(__file__).resolve().parents[1] / "simclr_amd" / "_C.so"
pytestmark = pytest.mark.skipif(not SO.exists(), reason="extension not built")


def _sched(parents, dur, k=3, lat=4.0):
    torch.ops.load_library(str(SO))
    off, flat = [0], []
    for ps in parents:
        flat += ps
        off.append(len(flat))
    out = torch.ops.simclr_amd.gexec_list_schedule(off, flat, [float(d) for d in dur], k, lat)
    n = len(dur)
    return list(out[:n]), list(out[n:])


def _simulate(parents, dur, order, streams, lat):
    """Start / finish times of the issued schedule on in-order streams."""
    fin, start, free = {}, {}, {}
    for v in order:
        s = streams[v]
        t = free.get(s, 0.0)
        for u in parents[v]:
            t = max(t, fin[u] + (0.0 if streams[u] == s else lat))
        start[v], fin[v] = t, t + dur[v]
        free[s] = fin[v]
    return start, fin


def test_random_dags_valid_schedule():
    rng = random.Random(3)
    for trial in range(40):
        n = rng.randint(1, 80)
        parents = [sorted(rng.sample(range(p), min(p, rng.randint(0, 3)))) for p in range(n)]
        dur = [rng.uniform(0.0, 50.0) for _ in range(n)]
        k = rng.randint(1, 4)
        order, streams = _sched(parents, dur, k)
        assert sorted(order) == list(range(n))
        pos = {v: i for i, v in enumerate(order)}
        for v in range(n):
            assert 0 <= streams[v] < k
            assert all(pos[u] < pos[v] for u in parents[v]), (trial, v)
        if n:  # the busiest stream is stream 0
            cnt = [streams.count(s) for s in range(k)]
            assert cnt[0] == max(cnt)


def test_chain_stays_on_one_stream_and_side_work_does_not_block():
    # a 20-node chain (10 µs each) with a weight-gradient-like leaf (30 µs) hanging off every
    # chain node, captured right after its parent: the chain never leaves stream 0 and each
    # leaf starts as soon as its parent is done (2 side streams absorb them)
    parents, dur, chain, leaves = [], [], [], []
    prev = None
    for i in range(20):
        parents.append([] if prev is None else [prev])
        dur.append(10.0)
        c = len(parents) - 1
        chain.append(c)
        parents.append([c])
        dur.append(15.0)
        leaves.append(len(parents) - 1)
        prev = c
    order, streams = _sched(parents, dur, k=3, lat=4.0)
    assert {streams[c] for c in chain} == {0}
    assert all(streams[x] != 0 for x in leaves[:-1])  # (the last one may follow the chain)
    start, fin = _simulate(parents, dur, order, streams, 4.0)
    for c in chain[1:]:  # back to back: no chain node waits on side work
        assert start[c] == pytest.approx(fin[parents[c][0]])
    for x in leaves[:-1]:
        assert start[x] == pytest.approx(fin[parents[x][0]] + 4.0)


def test_late_ready_node_does_not_block_an_earlier_ready_one():
    # node 0 runs 100 µs; node 1 depends on it; node 2 is independent but captured after node 1.
    # In capture order a stream holding node 1 would keep node 2 queued until t = 100; the list
    # schedule issues node 2 first, at t = 0 beside node 0
    parents = [[], [0], []]
    dur = [100.0, 5.0, 5.0]
    order, streams = _sched(parents, dur, k=2, lat=4.0)
    start, _ = _simulate(parents, dur, order, streams, 4.0)
    assert start[2] == 0.0
    assert order.index(2) < order.index(1)
