"""Build ``simclr_amd/_C.so`` in-tree with hipcc for gfx950 (no hipify, no JIT cache).

The kernel translation units (``*.hip``) include only HIP headers and compile in parallel in a
few seconds each; ``bindings.cpp`` and ``ipc.cpp`` are the only units that see the ATen headers.  Objects are
cached under ``csrc/_build`` and rebuilt when a source or a shared header is newer.

Usage:  python -m simclr_amd.csrc.build [--force] [--jobs N] [--debug]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
OUT = PKG / "_C.so"
BUILD = HERE / "_build"
KERNEL_SOURCES = ["conv.hip", "bn.hip", "misc.hip", "ntxent.hip", "lars.hip", "augment.hip",
                  "eval.hip", "comm.hip"]
BINDINGS = ["bindings.cpp", "ipc.cpp", "graphexec.cpp"]  # the units that see the ATen headers
HEADERS = ["common.h", "kernels.h"]
ARCH = os.environ.get("SIMCLR_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build simclr_amd kernels)")


def _torch_paths():
    import torch.utils.cpp_extension as ce
    import torch
    return ce.include_paths(), ce.library_paths(), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _stale(obj: Path, deps) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n  " + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build(force: bool = False, jobs: int = 0, debug: bool = False, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    BUILD.mkdir(exist_ok=True)
    opt = ["-O0", "-g"] if debug else ["-O3"]
    common = [f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", *opt, "-Wno-unused-result"]
    headers = [HERE / h for h in HEADERS]
    tasks = []
    objs = []
    for src in KERNEL_SOURCES:
        s = HERE / src
        o = BUILD / (s.stem + ".o")
        objs.append(o)
        if force or _stale(o, [s, *headers]):
            tasks.append([hipcc, *common, "-c", str(s), "-o", str(o)])
    incs, libdirs, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    for unit in BINDINGS:
        b = HERE / unit
        bo = BUILD / (b.stem + ".o")
        objs.append(bo)
        if force or _stale(bo, [b, *headers]):
            tasks.append([hipcc, *common, "-x", "hip", "-D__HIP_PLATFORM_AMD__=1",
                          "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                          *[f"-I{i}" for i in incs], f"-I{py_inc}", "-c", str(b), "-o", str(bo)])
    n = jobs or min(8, os.cpu_count() or 4)
    conv_rebuilt = any(str(BUILD / "conv.o") in t for t in tasks)
    if tasks:
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            for out in ex.map(_run, tasks):
                if verbose and out.strip():
                    print(out)
    if conv_rebuilt and not debug:
        # the LDS-DMA pipelines' ordering assumptions, verified on the emitted ISA
        sys.path.insert(0, str(PKG.parent / "tools"))
        import isa_check
        probs = isa_check.check(BUILD / "conv.o")
        if probs:
            (BUILD / "conv.o").unlink()
            raise RuntimeError("ISA check of conv.o failed:\n  " + "\n  ".join(probs[:20]))
    if force or tasks or not OUT.exists() or _stale(OUT, objs):
        tmp = OUT.with_suffix(".so.tmp")
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp),
              *[str(o) for o in objs], *[f"-L{d}" for d in libdirs],
              *[f"-Wl,-rpath,{d}" for d in libdirs],
              "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip"])
        os.replace(tmp, OUT)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--jobs", type=int, default=0)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    out = build(force=a.force, jobs=a.jobs, debug=a.debug, verbose=a.verbose)
    print(f"built {out}")


if __name__ == "__main__":
    main(sys.argv[1:])
