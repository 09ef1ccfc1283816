"""Run bench.py against another build of the extension (one-box A/B of two builds).
Usage: python tools/bench_lib.py path/to/_C.so [bench.py arguments]"""
import runpy
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import simclr_amd.ops._ext as ext  # noqa: E402

ext._LIB = Path(sys.argv[1]).resolve()
assert ext._LIB.exists(), ext._LIB
sys.argv = [str(ROOT / "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
