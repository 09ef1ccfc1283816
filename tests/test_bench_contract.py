"""bench.py's driver contract on the CPU (gloo): ``--gpus N`` started WITHOUT a launcher spawns
the N ranks itself (fail-fast launcher, /root/reference/launch.py:202-259) and reports the
whole-job number; a launcher/flag mismatch is an error, never a silent 1-rank measurement."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _env():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


@pytest.mark.timeout(900)
def test_bench_gpus2_self_launches_two_ranks(tmp_path):
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--model", "resnet18",
           "--batch", "8", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=_env(), capture_output=True, text=True,
                       timeout=840)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2"
    assert j["config"]["global_batch"] == 16 and j["steps"] == 2 and j["warmup"] == 1
    assert j["value"] > 0 and j["dtype"] == "fp32"


def test_bench_world_mismatch_is_an_error(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port))
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--model", "resnet18",
           "--batch", "8", "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr
