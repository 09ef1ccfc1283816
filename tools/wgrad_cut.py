"""Run tools/wgrad_probe.py against an analysis build (_scratch/_C_cut<N>.so, tools/wgrad_cut.sh)
instead of the shipped _C.so.  Usage: python tools/wgrad_cut.py N <wgrad_probe.py arguments>"""
import runpy
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import simclr_amd.ops._ext as ext  # noqa: E402

ext._LIB = ROOT / "_scratch" / f"_C_cut{sys.argv[1]}.so"
assert ext._LIB.exists(), ext._LIB
sys.argv = [str(ROOT / "tools" / "wgrad_probe.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
