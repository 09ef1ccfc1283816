"""ISA checks of the LDS-DMA kernels in the built gfx950 code object (conv.o).

The LDS-DMA pipelines (``igemm_glds`` / ``wgrad_glds`` in csrc/conv.hip) rely on two facts the
source cannot express, so they are verified on the disassembly:

1. *No compiler drain.*  hipcc's wait-count pass inserts ``s_waitcnt vmcnt(0)`` before an LDS
   access it cannot prove disjoint from an in-flight ``buffer_load ... lds`` — which silently
   serialises the next tile's DMA behind the current tile's compute.  Flagged: a vmcnt wait
   that follows a DMA issue and precedes an LDS read/write with no barrier in between.
2. *M0 discipline.*  Kernels that issue the DMA through inline asm (``dma16_opaque``) write M0
   themselves; hipcc must not keep anything of its own in M0 there: every M0 write is the
   asm's ``s_mov_b32 m0`` + ``s_nop 0`` + DMA triple, and no other implicit M0 reader appears.
3. *Counted waits match the stores behind them* (PRO 3 ``vmcnt(2*BM*8/NT)``): the
   loop-head wait of the block-output prologue kernels may leave S VMEM ops in flight only if at
   least S VMEM ops were issued after the last DMA of the previous iteration (otherwise part
   of tile kt's DMA could still be landing when the prologue reads it).

Usage: python tools/isa_check.py [path/to/conv.o]   (exit 1 on a violation)
"""
from __future__ import annotations

import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LLVM = Path("/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

DMA = re.compile(r"buffer_load_dword\w*\s.*\blds\b")
VMEM = re.compile(r"^\s*(global_|buffer_|flat_)(load|store|atomic)")
WAIT_VM = re.compile(r"s_waitcnt\s.*vmcnt\((\d+)\)")
LDS_ACC = re.compile(r"^\s*ds_(read|write|load|store)")


def disassemble(obj: Path) -> str:
    with tempfile.TemporaryDirectory() as td:
        fat = Path(td) / "fat.bin"
        co = Path(td) / "co.elf"
        subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", str(obj)], check=True)
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o",
                        f"--targets={TARGET}", f"--input={fat}", f"--output={co}"], check=True)
        out = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)],
                             check=True, capture_output=True, text=True)
        return out.stdout


def kernels(asm: str, pattern: str):
    """Yield (symbol, [instruction lines]) of every kernel whose symbol matches ``pattern``."""
    for m in re.finditer(r"^[0-9a-f]+ <(\S+)>:\n(.*?)(?=^\s*$|\Z)", asm, re.M | re.S):
        if re.search(pattern, m.group(1)):
            lines = [ln.split("//")[0].rstrip() for ln in m.group(2).splitlines()]
            yield m.group(1), [ln for ln in lines if ln.strip()]


def template_args(sym: str):
    return [int(v) for v in re.findall(r"Li(\d+)E", sym)]


def drains(lines):
    """Indices of vmcnt waits between a DMA issue and an LDS access with no barrier between."""
    bad = []
    pending = False  # a DMA issued since the last barrier
    wait_at = None
    for i, ln in enumerate(lines):
        if DMA.search(ln):
            pending, wait_at = True, None
        elif "s_barrier" in ln or re.match(r"\s*s_branch\s", ln):
            # (an unconditional branch: the next line in layout order is not its successor)
            pending, wait_at = False, None
        elif pending and WAIT_VM.search(ln):
            wait_at = i
        elif pending and wait_at is not None and LDS_ACC.search(ln):
            bad.append(wait_at)
            pending, wait_at = False, None
    return bad


M0_READERS = re.compile(r"^\s*(s_movrel|v_movrel|s_sendmsg|ds_gws|ds_append|ds_consume|v_interp|"
                        r"ds_ordered_count|global_load_lds|s_set_gpr_idx)")


def m0_violations(lines):
    """Lines breaking the M0 discipline of an opaque-DMA kernel."""
    bad = []
    for i, ln in enumerate(lines):
        if M0_READERS.match(ln):
            bad.append(ln.strip())
        elif re.match(r"^\s*\S+\s+m0\b", ln):  # an instruction writing M0
            nxt = [x.strip() for x in lines[i + 1:i + 3]]
            if not (ln.strip().startswith("s_mov_b32 m0") and len(nxt) == 2 and
                    nxt[0] == "s_nop 0" and DMA.search(nxt[1])):
                bad.append(ln.strip())
    return bad


def opaque(lines) -> bool:
    """Does the kernel issue all its DMA through dma16_opaque (m0 write, s_nop, DMA triples)?"""
    dmas = [i for i, ln in enumerate(lines) if DMA.search(ln)]
    return bool(dmas) and all(i >= 2 and lines[i - 1].strip() == "s_nop 0" and
                              lines[i - 2].strip().startswith("s_mov_b32 m0") for i in dmas)


def counted_wait_ok(lines, expect: int):
    """Every ``vmcnt(expect)`` wait must have >= expect VMEM ops after the last DMA that
    precedes the loop back-edge into it (linear layout: DMA ... stores ... back-edge)."""
    idx = [i for i, ln in enumerate(lines) if (m := WAIT_VM.search(ln)) and int(m.group(1)) == expect]
    if not idx:
        return False, "counted wait not found"
    last_dma = max((i for i, ln in enumerate(lines) if DMA.search(ln)), default=-1)
    # the back-edge is the last branch after the last DMA
    tail = lines[last_dma + 1:]
    n = sum(1 for ln in tail[:next((k for k, ln in enumerate(tail)
                                    if re.match(r"^\s*s_branch", ln)), len(tail))]
            if VMEM.match(ln))
    return n >= expect, f"{n} VMEM ops behind the last DMA, wait allows {expect}"


def check(obj: Path) -> list:
    asm = disassemble(obj)
    problems = []
    for sym, lines in kernels(asm, r"(igemm|wgrad)_(glds|patch)"):
        for i in drains(lines):
            problems.append(f"{sym}: compiler vmcnt drain after a DMA issue: {lines[i].strip()}")
        if opaque(lines):
            for ln in m0_violations(lines):
                problems.append(f"{sym}: M0 used outside the opaque DMA: {ln}")
        if "igemm_glds" in sym:
            a = template_args(sym)  # BM, BN, WM, WN, PRO, EPI, NST
            if len(a) >= 7 and a[4] == 3:
                nt = 64 * a[2] * a[3]
                ok, msg = counted_wait_ok(lines, 2 * a[0] * 8 // nt)
                if not ok:
                    problems.append(f"{sym}: PRO 3 counted wait: {msg}")
    return problems


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    obj = Path(argv[0]) if argv else ROOT / "simclr_amd" / "csrc" / "_build" / "conv.o"
    probs = check(obj)
    for p in probs:
        print(p)
    print(f"[isa_check] {obj}: {len(probs)} problem(s)")
    return 1 if probs else 0


if __name__ == "__main__":
    sys.exit(main())
