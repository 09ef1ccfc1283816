"""Collective latency histogram for the message sizes the SimCLR step issues.

* BN-statistics all-reduce: [Σ, Σ²] x 2 views per layer = 4C floats, C in {64 .. 2048}
  (ResNet-50: 54 per forward, 54 per backward, on the latency-critical path)
* gradient buckets: 4 MiB first bucket, 32 MiB buckets (fp32), on the comm stream
* NT-Xent global negatives: all-gather of the normalised z (1024 x 128 fp32 per rank)

Each size is timed ITERS times with device events around the single collective (after a
barrier), and p50 / p90 / p99 / max in microseconds are printed per size, rank 0 only.  GPU: one
rank per GPU over RCCL (``torch.distributed.run --nproc-per-node N tools/coll_latency.py``);
``--world1`` times a 1-rank RCCL group on one GPU (the launch floor); CPU: gloo.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def _pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--world1", action="store_true", help="1-rank group without a launcher")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    if a.world1:
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29641")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    if cuda:
        torch.cuda.set_device(local % torch.cuda.device_count())
        dev = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dev = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    cases = [("bn_stats C=%d" % c, "all_reduce", 4 * c) for c in (64, 128, 256, 512, 1024, 2048)]
    cases += [("grad bucket 4MiB", "all_reduce", 1 << 20), ("grad bucket 32MiB", "all_reduce", 8 << 20),
              ("z all_gather 1024x128", "all_gather", 1024 * 128)]
    rows = []
    for name, kind, n in cases:
        x = torch.ones(n, device=dev)
        out = torch.empty(n * world, device=dev) if kind == "all_gather" else None
        iters = a.iters if n < (1 << 20) else max(10, a.iters // 10)
        lat = []
        for i in range(iters + 5):
            dist.barrier()
            if cuda:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
            t0 = time.perf_counter()
            if kind == "all_reduce":
                dist.all_reduce(x)
            else:
                dist.all_gather_into_tensor(out, x)
            if cuda:
                e.record()
                e.synchronize()
                us = s.elapsed_time(e) * 1e3
            else:
                us = (time.perf_counter() - t0) * 1e6
            if i >= 5:
                lat.append(us)
        t = torch.tensor([_pct(lat, 0.5), _pct(lat, 0.9), _pct(lat, 0.99), max(lat)],
                         dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rows.append(dict(name=name, bytes=4 * n, p50_us=t[0].item(), p90_us=t[1].item(),
                         p99_us=t[2].item(), max_us=t[3].item()))
    if rank == 0:
        be = dist.get_backend()
        print(f"# collective latency, world={world}, backend={be} (max over ranks)\n")
        print("| collective | bytes/rank | p50 us | p90 us | p99 us | max us |\n|---|---:|---:|---:|---:|---:|")
        for r in rows:
            print(f"| {r['name']} | {r['bytes']} | {r['p50_us']:.1f} | {r['p90_us']:.1f} | "
                  f"{r['p99_us']:.1f} | {r['max_us']:.1f} |")
        if a.json:
            with open(a.json, "w") as f:
                json.dump({"world": world, "backend": be, "rows": rows}, f, indent=1)
        sys.stdout.flush()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
