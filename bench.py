"""Headline benchmark: SimCLR pre-training images/sec (whole node), ResNet-50, CIFAR-10 shape.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 either launched
by ``torch.distributed.run`` (one rank per GPU, RCCL) or, when started directly (no
``WORLD_SIZE`` in the environment), it spawns the N ranks itself through the fail-fast launcher
(simclr_amd/runtime/launcher.py, the analogue of /root/reference/launch.py:202-259) before the
parent touches the GPU.  Every rank asserts ``WORLD_SIZE == --gpus``.  W untimed steps, then
exactly K timed steps bracketed by barrier + device synchronise, max over ranks, rank 0 prints
ONE JSON line.

Config (BASELINE.json "ResNet-50 SimCLR CIFAR-10 bf16, batch=512 on 1 MI355X"): ResNet-50 with
the CIFAR stem (3x3/s1, no maxpool — the north star's CIFAR-ResNet-50), 512 images per GPU (two
augmented views each → 1024 forward rows), 32x32 synthetic uint8 data augmented on device,
projection head 2048-2048-128, NT-Xent τ=0.5, LARS + warmup/cosine, full optimizer step inside
the timed region.  Weak scaling (512 images per GPU at every N).

``--impl reference`` times the reference-semantics step built from stock torch ops (fp32 NCHW,
two forwards, torch BN/SyncBN, DDP, LARC loop — bench/torch_reference.py) on the same hardware;
BASELINE publishes no throughput, so that measurement is the ``vs_baseline`` denominator
(``profiles/reference_baseline.json``).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "pretrain images/sec (whole node) + CIFAR-10 linear-probe top-1, ResNet-50"
PG_TIMEOUT_S = float(os.environ.get("SIMCLR_BENCH_PG_TIMEOUT", "300"))
PROBE_ROUNDS = 3  # execution-mode probe: 3 x (2 eager + 2 graph) interleaved steps


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args, argv) -> int:
    """``--gpus N`` without a launcher: spawn N ranks of this script (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment) and return the first non-zero exit code (the
    survivors are terminated) or 0.  Runs before any GPU call in this process; rank 0's JSON
    line reaches stdout directly."""
    from simclr_amd.runtime.launcher import launch, parse_args, visible_gpu_count
    # visibility variables / KFD topology only: this parent forks every rank and must never
    # initialise HIP itself (torch.cuda.device_count() can fall back to hipGetDeviceCount)
    ndev = visible_gpu_count()
    if ndev == 0:
        # every GPU hidden by a visibility variable: the ranks run on the CPU over gloo (the CPU
        # rehearsal of the driver contract), never silently on fewer GPUs
        print(f"[bench] no GPU visible: the {args.gpus} ranks run on the CPU (gloo)",
              file=sys.stderr, flush=True)
    elif ndev is not None and ndev < args.gpus and os.environ.get("SIMCLR_DIST_BACKEND") != "gloo":
        raise SystemExit(f"bench: --gpus {args.gpus} but only {ndev} GPU(s) visible")
    la = parse_args(["--nproc_per_node", str(args.gpus), "--master_addr", "127.0.0.1",
                     "--master_port", str(_free_port()), "--use_env", str(Path(__file__).resolve()),
                     *argv])
    return launch(la)


def _init():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        idx = local % torch.cuda.device_count()
        torch.cuda.set_device(idx)
        dev = torch.device("cuda", idx)
    else:
        dev = torch.device("cpu")
    force = os.environ.get("SIMCLR_FORCE_COMM", "0") == "1"
    if force and world == 1:
        # 1-rank process group: every collective of the multi-GPU step is still issued
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
    if (world > 1 or force) and not dist.is_initialized():
        # SIMCLR_DIST_BACKEND=gloo rehearses the multi-rank HIP path on one GPU (RCCL refuses
        # two ranks on the same device); the driver's runs use nccl (= RCCL over xGMI).
        be = os.environ.get("SIMCLR_DIST_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
        kw = {"device_id": dev} if be == "nccl" else {}
        # short process-group timeout: a dead or hung rank fails the bench in minutes instead of
        # holding the node for the default 30 min
        dist.init_process_group(be, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=PG_TIMEOUT_S), **kw)
    return rank, world, local, dev


def _sync(dev, world):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _set_mode(tr, graph, mode: str) -> None:
    """eager | graph (hipGraphLaunch) | streams (native multi-stream replay of the graph)."""
    tr.graph = None if mode == "eager" else graph
    tr.replay_mode = "streams" if mode == "streams" else "graph"


def _exec_mode(tr) -> str:
    if tr.graph is None:
        return "eager"
    return "streams" if (tr.replay_mode == "streams" and tr.sreplay is not None) else "graph"


def run_ours(args, rank, world, dev):
    from simclr_amd.config import compose, task_config, CONF_DIR
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    from simclr_amd.parallel import state as pstate
    from simclr_amd.train.pretrain import Trainer
    from simclr_amd.utils.misc import seed_everything

    st = pstate.set_state(rank=rank, world_size=world, local_rank=int(os.environ.get(
        "LOCAL_RANK", "0")), group=dist.group.WORLD if dist.is_initialized() else None,
        backend=dist.get_backend() if dist.is_initialized() else "none",
        force_comm=dist.is_initialized())
    st.device = dev
    pstate.make_stat_group(st)
    if st.comm and dev.type == "cuda":
        from simclr_amd.comm import setup_stats_exchange
        # IPC BatchNorm statistics as a CANDIDATE (self-tested, else RCCL): the probe below
        # times it against RCCL and keeps the faster; training defaults to RCCL
        setup_stats_exchange(st, dev, mode=os.environ.get("SIMCLR_BN_COMM", "auto"))
    ov = [f"experiment.base_cnn={args.model}", f"experiment.batches={args.batch}",
          f"model.cifar_stem={'true' if args.cifar_stem else 'null'}",
          "data.synthetic=true", f"runtime.precision={args.precision}",
          f"loss.gather={'true' if args.gather else 'false'}", "parameter.epochs=100",
          f"runtime.bucket_mb={args.bucket_mb}"]
    cfg = task_config(compose(str(CONF_DIR), "config", ov, job_name="bench"))
    seed_everything(cfg["parameter"]["seed"])
    # CIFAR-10's training-set length at every N: at N = 8 an epoch is 12 steps, as
    # in the reference; each rank's shard order is uploaded without a stream sync at rollover
    # (ImageNet-shape runs keep a smaller set: 50,000 224² images would be 7.5 GB of host RAM)
    n_img = 50000 if args.size <= 64 else max(8192, 4 * args.batch * world)
    ds = synthetic_dataset(n_img, 10, size=args.size, seed=rank)
    loader = ContrastiveLoader(ds, args.batch, dev, rank=rank, world=world,
                               strength=cfg["experiment"]["strength"], seed=7, views=2)
    loader.with_labels = False
    tr = Trainer(cfg, st, 50000)
    args.dtype = tr.precision  # fp32 on a CPU rehearsal
    tr.guard.on_error = "defer"  # an IPC timeout is checked collectively below (ipc_guard)
    it = iter(loader)
    args.bn_comm = ("ipc" if st.ipc is not None else "rccl") if st.comm else "none"

    def next_batch():
        nonlocal it
        try:
            return next(it)[0]
        except StopIteration:
            loader.set_epoch(loader.epoch + 1)
            it = iter(loader)
            return next(it)[0]

    def timed(k):
        _sync(dev, world)
        t = time.perf_counter()
        for _ in range(k):
            tr.step(next_batch())
        _sync(dev, world)
        return time.perf_counter() - t

    def ipc_guard() -> bool:
        from simclr_amd.comm import fallback_if_failed
        if fallback_if_failed(st, dev):
            args.bn_comm = "rccl(ipc-fallback)"
            return True
        return False

    auto = args.graph == "auto"
    t_eager = None
    if tr.hip and st.ipc is not None and os.environ.get("SIMCLR_BN_COMM", "auto") == "auto":
        # statistics-exchange autotune (N > 1): the IPC arena exchange (one-shot stores over
        # xGMI, spin on LL words) vs the RCCL all-reduce, 3 eager steps each after a warm-up,
        # the slower of the ranks decides (same choice everywhere)
        timed(2)
        if not ipc_guard():
            t_ipc = timed(3)
            ex, st.ipc = st.ipc, None
            t_rccl = timed(3)
            tt = torch.tensor([t_ipc, t_rccl, float(ex.failed())], dtype=torch.float64,
                              device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            if float(tt[0]) < float(tt[1]) and float(tt[2]) == 0.0:
                st.ipc = ex
            args.comm_probe_ms = [round(float(v) / 3 * 1000.0, 3) for v in tt.tolist()[:2]]
            args.bn_comm = "ipc" if st.ipc is not None else "rccl(probe)"
    if auto and tr.hip:
        timed(2)  # eager warm-up: autotuning, allocator, communicators
        if ipc_guard():
            timed(1)
        t_eager = 0.0  # measured below, interleaved with the graph replays
    if args.graph and tr.hip:
        try:
            tr.capture(next_batch())
        except Exception as e:  # deterministic across ranks: every rank falls back together
            print(f"[bench] rank {rank}: hipGraph capture failed ({e!r}); running eager",
                  file=sys.stderr, flush=True)
            tr.graph = None
            args.graph = False
    if tr.graph is not None and tr.sreplay is not None and tr.sreplay.pending:
        _set_mode(tr, tr.graph, "streams")
        timed(1)  # the executor's planning replay (one serial, per-node timed step)
    if auto and tr.graph is not None and t_eager is not None:
        # execution-mode autotune: eager issue vs replaying the captured step with the HIP graph
        # executor vs the native multi-stream executor over the same captured nodes
        # (runtime/graph_exec.py).  The HIP graph executor loses part of the side-stream overlap;
        # eager issue costs host time that grows with the ranks sharing the CPUs.
        # PROBE_ROUNDS interleaved rounds of 2 steps per arm (box drift hits every arm alike);
        # the slower rank decides, the same choice on every rank
        arms = ["eager", "graph"] + (["streams"] if tr.sreplay is not None else [])
        g = tr.graph
        tot = {a: 0.0 for a in arms}
        for _ in range(PROBE_ROUNDS):
            for a in arms:
                _set_mode(tr, g, a)
                tot[a] += timed(2)
        n = 2 * PROBE_ROUNDS
        tt = torch.tensor([tot[a] for a in arms], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        best = arms[int(torch.argmin(tt).item())]
        _set_mode(tr, g, best)
        args.mode_probe = {a: round(float(v) / n * 1000.0, 3) for a, v in zip(arms, tt.tolist())}
        args.mode_probe_ms = [args.mode_probe["eager"], args.mode_probe["graph"]]
    elif args.exec_mode in ("graph", "streams") and tr.graph is not None:
        _set_mode(tr, tr.graph, "streams" if (args.exec_mode == "streams"
                                              and tr.sreplay is not None) else "graph")
    args.graph = tr.graph is not None
    args.exec_used = _exec_mode(tr)
    if tr.graph is not None:
        loader.out = tr._static_x  # the augmentation writes the replayed step's input in place
    loss = None
    from simclr_amd.parallel import invariant as inv
    args.dp_invariant = {"dropped_modes": []}

    def replicas(where: str) -> bool:
        """Data-parallel invariant (parallel/invariant.py): master, shadow, momentum, step
        counter and BatchNorm buffers bitwise equal on every rank.  Untimed."""
        if world <= 1:
            args.dp_invariant[where] = "trivial(1 rank)"
            return True
        r = inv.check_replicas(tr.store, tr.opt, tr.model, group=st.group)
        args.dp_invariant[where] = inv.summary(r)
        return r["ok"]

    def drop_mode(where: str) -> None:
        """The replicas diverged under the current issue mode: every rank re-adopts rank 0's
        state and falls back to eager issue (the same decision everywhere: the check's answer
        is collective).  Divergence under eager issue is a bug, not a mode problem: raise."""
        mode = _exec_mode(tr)
        inv.resync(tr.store, tr.opt, group=st.group)
        if mode == "eager":
            raise inv.ReplicaDivergence(f"rank {rank}: replicas diverged under eager issue "
                                        f"({where}: {args.dp_invariant[where]})")
        print(f"[bench] rank {rank}: replicas diverged under {mode} replay ({where}); "
              "dropping it, issuing eagerly", file=sys.stderr, flush=True)
        args.dp_invariant["dropped_modes"].append(mode)
        tr.graph = None
        args.graph = False

    if not replicas("after_probe"):
        drop_mode("after_probe")

    def measure():
        nonlocal loss
        for _ in range(args.warmup):
            loss = tr.step(next_batch())
        _sync(dev, world)
        if ipc_guard():  # the captured graph (if any) holds the IPC exchange: issue eagerly
            tr.graph = None
            args.graph = False
            for _ in range(max(1, args.warmup)):
                loss = tr.step(next_batch())
            _sync(dev, world)
        t0 = time.perf_counter()
        host = 0.0
        for _ in range(args.steps):
            h0 = time.perf_counter()
            loss = tr.step(next_batch())
            host += time.perf_counter() - h0
        _sync(dev, world)
        t1 = time.perf_counter()
        # host time spent issuing the steps (≈ wall time means the run is launch/CPU bound; with
        # a replay the host also blocks whenever the device queue is full)
        args.host_issue_ms = host / args.steps * 1000.0
        # the issue cost itself: steps issued onto an idle device (untimed, after the K steps)
        idle = []
        for _ in range(3):
            _sync(dev, world)
            h0 = time.perf_counter()
            loss = tr.step(next_batch())
            idle.append(time.perf_counter() - h0)
        _sync(dev, world)
        args.host_issue_idle_ms = min(idle) * 1000.0
        return t0, t1

    t0, t1 = measure()
    if ipc_guard():
        # an IPC spin timed out inside the timed region: those steps ran on partial BatchNorm
        # statistics, so the measurement is void — every rank is on RCCL now (collective
        # decision) and the K steps are timed again
        print(f"[bench] rank {rank}: IPC statistics exchange timed out in the timed region; "
              "re-timing on RCCL", file=sys.stderr, flush=True)
        tr.graph = None
        args.graph = False
        args.bn_comm = "rccl(ipc-timeout, re-timed)"
        t0, t1 = measure()
    if not replicas("after_timed"):
        # the K timed steps ran on diverged replicas: void; re-time them under eager issue
        drop_mode("after_timed")
        t0, t1 = measure()
        if not replicas("after_retimed"):
            drop_mode("after_retimed")  # eager diverged: raises
    args.exec_used = _exec_mode(tr)
    if tr.sreplay is not None:
        args.sreplay_stats = tr.sreplay.stats()
    return t1 - t0, float(loss.item()) if loss is not None else float("nan")


def run_reference(args, rank, world, dev):
    from bench.torch_reference import (PlainContrastive, exclude_from_wt_decay, larc_step,
                                       nt_xent_reference)
    torch.manual_seed(7)
    ref_stem = "reference_cifar" if args.model == "resnet18" else "imagenet"
    model = PlainContrastive(args.model, stem="cifar" if args.cifar_stem else ref_stem).to(dev)
    if world > 1:
        model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    opt = torch.optim.SGD(exclude_from_wt_decay(model.named_parameters(), 1e-4),
                          lr=args.batch / 256, momentum=0.9, weight_decay=0.0)
    v0 = torch.rand(args.batch, 3, args.size, args.size, device=dev)
    v1 = torch.rand(args.batch, 3, args.size, args.size, device=dev)

    def step():
        opt.zero_grad()
        z0 = model(v0)
        z1 = model(v1)
        loss = nt_xent_reference(z0, z1, 0.5)
        loss.backward()
        larc_step(opt)
        return loss

    loss = None
    for _ in range(args.warmup):
        loss = step()
    _sync(dev, world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    _sync(dev, world)
    return time.perf_counter() - t0, float(loss.item())


def _stem_key(args) -> str:
    if args.cifar_stem:
        return "cifar"
    return "refstem" if args.model == "resnet18" else "imagenet"


def _stem_label(args) -> str:
    if args.cifar_stem:
        return "cifar-stem"
    return ("reference-stem(3x3/p3)" if args.model == "resnet18"
            else "imagenet-stem(7x7/s2+maxpool)")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--cifar-stem", dest="cifar_stem", action="store_true", default=True,
                    help="3x3/s1/p1 stem, no maxpool (the north star's CIFAR-ResNet; default)")
    ap.add_argument("--reference-stem", "--imagenet-stem", dest="cifar_stem",
                    action="store_false",
                    help="the stem the reference builds: r50 ImageNet 7x7/s2 + maxpool, "
                         "r18 3x3/s1/p3 (model.py:90-104)")
    ap.add_argument("--batch", type=int, default=512, help="images per GPU")
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--gather", dest="gather", action="store_true", default=None,
                    help="global negatives: NT-Xent over the all-gathered embeddings of every "
                         "rank (default at N > 1, the north star's loss)")
    ap.add_argument("--local-loss", dest="gather", action="store_false",
                    help="per-GPU NT-Xent, the reference's loss (loss.py has no collective)")
    ap.add_argument("--graph", action="store_true", default=None,
                    help="capture the step in a hipGraph and replay it")
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="issue every step eagerly (default: probe both, keep the faster)")
    ap.add_argument("--exec", dest="exec_mode", default="auto",
                    choices=["auto", "eager", "graph", "streams"],
                    help="step issue mode: auto (probe eager / hipGraph / native multi-stream "
                         "replay, keep the fastest), or one of them forced")
    ap.add_argument("--bucket-mb", dest="bucket_mb", type=float, default=32.0)
    ap.add_argument("--impl", choices=["ours", "reference"], default="ours")
    argv = list(sys.argv[1:] if argv is None else argv)
    args = ap.parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args, argv))
    rank, world, local, dev = _init()
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and "
                         "the flag disagree")
    if args.gather is None:
        args.gather = world > 1
    if args.exec_mode == "eager":
        args.graph = False
    elif args.exec_mode in ("graph", "streams"):
        args.graph = True
    if args.graph is None:
        # default: probe the eager step and the hipGraph replay of the whole step (RCCL
        # collectives included, thread-local capture mode) for 3 steps each and keep the faster
        # (same decision on every rank); gloo rehearsals on one GPU stay eager (host collectives
        # cannot be captured)
        args.graph = "auto" if (not dist.is_initialized() or dist.get_backend() == "nccl") \
            else False
    args.bn_comm = "none"
    if args.impl == "ours":
        dt, loss = run_ours(args, rank, world, dev)
    else:
        dt, loss = run_reference(args, rank, world, dev)
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / args.steps * 1000.0
    value = args.steps * args.batch * world / dt
    base = None
    bpath = ROOT / "profiles" / "reference_baseline.json"
    if bpath.exists():
        try:
            b = json.loads(bpath.read_text())
            key = f"{args.model}-{_stem_key(args)}-b{args.batch}" + (
                f"-s{args.size}" if args.size != 32 else "")
            per_gpu = b.get("images_per_sec_per_gpu", {}).get(key)
            if per_gpu:
                base = per_gpu * world
        except Exception:
            base = None
    flop = None
    try:
        from simclr_amd.utils.flops import step_flops
        flop = step_flops(args.model, True if args.cifar_stem else None, args.size, args.batch)
    except Exception as e:  # accounting only: never fails the bench
        print(f"[bench] FLOP count failed: {e!r}", file=sys.stderr, flush=True)
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(value / base, 3) if (base and args.impl == "ours") else None),
        "dtype": getattr(args, "dtype", args.precision) if args.impl == "ours" else "fp32",
        "data": (f"synthetic {args.size}x{args.size} uint8 "
                 f"{'CIFAR' if args.size == 32 else 'ImageNet'}-shape images, random-init "
                 "weights, on-device SimCLR augmentation"),
        "config": {
            "model": f"{args.model}-{_stem_label(args)}"
                     f"+projection-head({2048 if args.model == 'resnet50' else 512}-"
                     f"{2048 if args.model == 'resnet50' else 512}-128)",
            "global_batch": args.batch * world,
            "per_gpu_batch": args.batch,
            "views": 2,
            "seq_len": None,
            "image_size": args.size,
            "parallelism": f"dp{world}",
            "loss": "nt-xent tau=0.5" + (" global-negatives" if args.gather else " local"),
            "optimizer": "LARS(trust=1e-3)+SGD(m=0.9), warmup+cosine",
            "impl": args.impl,
            "hip_graph": bool(args.graph and args.impl == "ours"),
            "exec_mode_probe_ms_eager_graph": getattr(args, "mode_probe_ms", None),
            "exec_mode_probe_ms": getattr(args, "mode_probe", None),
            "exec_mode": getattr(args, "exec_used", None),
            "stream_replay": getattr(args, "sreplay_stats", None),
            "bn_stats_comm": args.bn_comm,
            "bn_comm_probe_ms_ipc_rccl": getattr(args, "comm_probe_ms", None),
            "host_issue_ms_per_step": (round(args.host_issue_ms, 3)
                                       if hasattr(args, "host_issue_ms") else None),
            "host_issue_ms_idle_device": (round(args.host_issue_idle_ms, 3)
                                          if hasattr(args, "host_issue_idle_ms") else None),
            "final_loss": loss,
            "dp_invariant": getattr(args, "dp_invariant", None),
        },
        # utilisation: model FLOPs of one step per GPU (3 x forward, counted from the real
        # conv / matmul shapes: simclr_amd/utils/flops.py) over the measured step time
        "model_tflop_per_step_per_gpu": round(flop / 1e12, 4) if flop else None,
        "achieved_tflops_per_gpu": round(flop / (ms / 1000.0) / 1e12, 1) if flop else None,
        "achieved_tflops_total": round(flop * world / (ms / 1000.0) / 1e12, 1) if flop else None,
        "mfu_vs_2p5pf_dense_bf16": round(flop / (ms / 1000.0) / 2.5e15, 4) if flop else None,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
