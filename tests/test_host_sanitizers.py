"""AddressSanitizer + UndefinedBehaviorSanitizer build of the kernel launchers' host code
(SURVEY §5.2): tools/host_check.cpp drives the tile-variant admissibility, split planning and
workspace arithmetic of conv.hip / bn.hip / ntxent.hip / eval.hip / misc.hip over every conv of
ResNet-18/50 (CIFAR and ImageNet shapes, fwd / dgrad / wgrad).  GPU-side sanitizers are not
available on this pool, so only host code is instrumented (``-Xarch_host -fsanitize=...``).
The build (~2 min, dominated by conv.hip's device pass) is cached under tools/_host_check/,
keyed by the sources' contents."""
import concurrent.futures as cf
import hashlib
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "simclr_amd" / "csrc"
OUT = ROOT / "tools" / "_host_check"
UNITS = ["conv.hip", "bn.hip", "ntxent.hip", "eval.hip", "misc.hip"]
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-sanitize-recover=all"]


def _digest() -> str:
    h = hashlib.sha256()
    for p in [ROOT / "tools" / "host_check.cpp", CSRC / "kernels.h", CSRC / "common.h",
              *[CSRC / u for u in UNITS]]:
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")
@pytest.mark.timeout(900)
def test_host_code_clean_under_asan_ubsan():
    OUT.mkdir(parents=True, exist_ok=True)
    exe = OUT / f"host_check-{_digest()}"
    if not exe.exists():
        common = ["--offload-arch=gfx950", "-x", "hip", "-std=c++17", "-O1", "-g", *SAN,
                  f"-I{CSRC}"]
        srcs = [ROOT / "tools" / "host_check.cpp", *[CSRC / u for u in UNITS]]
        objs = [OUT / (s.stem + ".o") for s in srcs]

        def cc(pair):
            s, o = pair
            r = subprocess.run([HIPCC, *common, "-c", str(s), "-o", str(o)],
                               capture_output=True, text=True)
            assert r.returncode == 0, r.stderr[-4000:]
        with cf.ThreadPoolExecutor(max_workers=6) as ex:
            list(ex.map(cc, zip(srcs, objs)))
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", *SAN[:4], *map(str, objs), "-o",
                            str(exe)], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-4000:]
        for o in objs:
            o.unlink()
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env={"ASAN_OPTIONS": "detect_leaks=0", "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s)" in r.stdout
