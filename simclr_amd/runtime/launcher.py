"""Fail-fast multi-process launcher (one process per GPU).

Reference: ``/root/reference/launch.py`` — a fork of ``torch.distributed.launch``
that sets MASTER_ADDR/PORT, WORLD_SIZE, RANK, LOCAL_RANK, OMP_NUM_THREADS=1 (nproc > 1) and
appends the Hydra overrides ``distributed.local_rank=<i> distributed.world_size=<W>`` (unless
``--use_env``), then waits on the children *sequentially* and never kills siblings, so one
crashed rank leaves the others blocked in a collective (Q13).

Here the children are polled together; the first non-zero exit terminates the remaining ranks
(SIGTERM, then SIGKILL after ``--kill_grace`` seconds) and the launcher exits with that code.
SIGINT/SIGTERM to the launcher are forwarded.  The global rank (``node_rank * nproc + i``) is
exported as RANK, so multi-node works (Q12).  Same command line as the reference.
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time
from argparse import REMAINDER, ArgumentParser
from typing import List, Optional


def parse_args(argv=None):
    p = ArgumentParser(description="spawn one training process per GPU (fail-fast)")
    p.add_argument("--nnodes", type=int, default=1)
    p.add_argument("--node_rank", type=int, default=0)
    p.add_argument("--nproc_per_node", type=int, default=1)
    p.add_argument("--master_addr", default="127.0.0.1", type=str)
    p.add_argument("--master_port", default=29500, type=int)
    p.add_argument("--use_env", default=False, action="store_true",
                   help="do not append the Hydra overrides; ranks come from the environment")
    p.add_argument("-m", "--module", default=False, action="store_true",
                   help="run the training script as a module (python -m)")
    p.add_argument("--no_python", default=False, action="store_true")
    p.add_argument("--kill_grace", type=float, default=10.0,
                   help="seconds between SIGTERM and SIGKILL of surviving ranks")
    p.add_argument("training_script", type=str)
    p.add_argument("training_script_args", nargs=REMAINDER)
    return p.parse_args(argv)


def build_commands(args) -> List[tuple]:
    world = args.nproc_per_node * args.nnodes
    base_env = os.environ.copy()
    base_env["MASTER_ADDR"] = args.master_addr
    base_env["MASTER_PORT"] = str(args.master_port)
    base_env["WORLD_SIZE"] = str(world)
    base_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if "OMP_NUM_THREADS" not in os.environ and args.nproc_per_node > 1:
        base_env["OMP_NUM_THREADS"] = "1"
    out = []
    for local in range(args.nproc_per_node):
        env = dict(base_env)
        env["RANK"] = str(args.nproc_per_node * args.node_rank + local)
        env["LOCAL_RANK"] = str(local)
        if args.no_python:
            if not args.use_env:
                raise ValueError("When using the '--no_python' flag, you must also set the "
                                 "'--use_env' flag.")
            if args.module:
                raise ValueError("Don't use both the '--no_python' flag and the '--module' flag.")
            cmd = []
        else:
            cmd = [sys.executable, "-u"] + (["-m"] if args.module else [])
        cmd.append(args.training_script)
        if not args.use_env:
            cmd += ["distributed.local_rank={}".format(local),
                    "distributed.world_size={}".format(world)]
        cmd += list(args.training_script_args)
        out.append((cmd, env))
    return out


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def visible_gpu_count(kfd_nodes: str = KFD_NODES) -> Optional[int]:
    """GPUs a child process will see, WITHOUT initialising HIP in this process (a launcher
    parent must never touch the GPU: ``torch.cuda.device_count()`` falls back to
    ``hipGetDeviceCount`` on ROCm when amdsmi is unavailable).  The visibility variables win
    when set; otherwise the KFD topology's GPU nodes (``simd_count > 0``; CPU nodes have 0) are
    counted.  None when neither source is available.

    The variables stack (ROCR filters the devices, HIP / CUDA filter what ROCR left), so the
    count is the minimum over the ones that are set; a set but empty variable hides every GPU
    (0, which callers treat as "no GPU visible", not "unknown")."""
    counts = []
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            counts.append(len([t for t in v.split(",") if t.strip() != ""]))
    if counts:
        return min(counts)
    try:
        n = 0
        for node in sorted(os.listdir(kfd_nodes)):
            try:
                with open(os.path.join(kfd_nodes, node, "properties")) as f:
                    for line in f:
                        k, _, val = line.partition(" ")
                        if k == "simd_count" and int(val) > 0:
                            n += 1
                            break
            except (OSError, ValueError):
                continue
        return n
    except OSError:
        return None


def _terminate(procs, grace: float) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                p.send_signal(signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + grace
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
    for p in procs:
        if p.poll() is None:
            try:
                p.kill()
            except ProcessLookupError:
                pass
            p.wait()


def launch(args) -> int:
    cmds = build_commands(args)
    procs = [subprocess.Popen(cmd, env=env) for cmd, env in cmds]

    def forward(signum, frame):
        _terminate(procs, args.kill_grace)
        sys.exit(128 + signum)

    old_int = signal.signal(signal.SIGINT, forward)
    old_term = signal.signal(signal.SIGTERM, forward)
    rc = 0
    try:
        alive = set(range(len(procs)))
        while alive:
            for i in list(alive):
                r = procs[i].poll()
                if r is None:
                    continue
                alive.discard(i)
                if r != 0:
                    sys.stderr.write(f"[launch] rank {i} exited with code {r}; terminating "
                                     f"{len(alive)} remaining rank(s)\n")
                    _terminate(procs, args.kill_grace)
                    return r
            time.sleep(0.05)
    finally:
        signal.signal(signal.SIGINT, old_int)
        signal.signal(signal.SIGTERM, old_term)
    return rc


def main(argv=None) -> None:
    sys.exit(launch(parse_args(argv)))
