"""The built extension registers every op schema (a bad schema aborts the process at load time,
which CPU-only runs would otherwise never notice: nothing launches a kernel there)."""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SO = ROOT / "simclr_amd" / "_C.so"


@pytest.mark.skipif(not SO.exists(), reason="extension not built")
def test_extension_loads_and_registers_ops():
    code = ("import torch; torch.ops.load_library(%r); o = torch.ops.simclr_amd; "
            "names = ['igemm', 'wgrad', 'bn_reduce_fused', 'ipc_open', 'maxpool_fwd', "
            "'ce_topk', 'class_sums', 'augment', 'lars_update', 'nt_forward']; "
            "[getattr(o, n).default for n in names]; print('ok')" % str(SO))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-3000:]
