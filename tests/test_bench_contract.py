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


def test_self_launch_never_touches_hip(monkeypatch):
    """The parent that forks every rank counts GPUs from the visibility variables / KFD
    topology only: torch.cuda.device_count() (which can fall back to hipGetDeviceCount) is never
    called and HIP stays uninitialised in the parent."""
    import argparse
    import torch
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_script", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)  # (the bench/ package shadows the name)
    spec.loader.exec_module(bench)
    from simclr_amd.runtime import launcher

    def boom(*a, **k):
        raise AssertionError("the launcher parent called into torch.cuda")
    monkeypatch.setattr(torch.cuda, "device_count", boom)
    monkeypatch.setattr(torch.cuda, "is_available", boom)
    seen = {}

    def fake_launch(la):
        seen["n"] = la.nproc_per_node
        return 0
    monkeypatch.setattr(launcher, "launch", fake_launch)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    rc = bench.self_launch(argparse.Namespace(gpus=8), ["--gpus", "8"])
    assert rc == 0 and seen["n"] == 8
    assert not torch.cuda.is_initialized()
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1")
    with pytest.raises(SystemExit, match="only 2 GPU"):
        bench.self_launch(argparse.Namespace(gpus=8), ["--gpus", "8"])


def test_visible_gpu_count_reads_kfd_topology(tmp_path, monkeypatch):
    from simclr_amd.runtime.launcher import visible_gpu_count
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    for i, simd in enumerate([0, 1024, 1024, 0]):  # CPU nodes have simd_count 0
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 8\nsimd_count {simd}\nmem_banks_count 1\n")
    assert visible_gpu_count(str(tmp_path)) == 2
    assert visible_gpu_count(str(tmp_path / "missing")) is None
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert visible_gpu_count(str(tmp_path)) == 0


def test_visible_gpu_count_stacks_variables(monkeypatch):
    """ROCR filters the devices and HIP / CUDA filter what it left: the count is the minimum
    over the variables that are set, and an empty one hides every GPU."""
    from simclr_amd.runtime.launcher import visible_gpu_count
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2,3")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert visible_gpu_count("/nonexistent") == 2
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")
    assert visible_gpu_count("/nonexistent") == 0
