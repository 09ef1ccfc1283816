"""ISA-level checks of the LDS-DMA kernels (tools/isa_check.py) on the built conv.o: no compiler
vmcnt drain of the DMA pipelines, M0 used only by the opaque DMA, and the block-output
prologue's counted wait (vmcnt(2*BM*8/NT)) backed by at least that many VMEM stores."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
OBJ = ROOT / "simclr_amd" / "csrc" / "_build" / "conv.o"
sys.path.insert(0, str(ROOT / "tools"))


@pytest.mark.skipif(not OBJ.exists(), reason="conv.o not built (run __graft_entry__.build())")
def test_lds_dma_isa_invariants():
    import isa_check
    assert isa_check.check(OBJ) == []


def test_drain_detector_on_synthetic_listing():
    import isa_check
    drained = ["buffer_load_dwordx4 v1, s[0:3], 0 offen lds", "s_waitcnt vmcnt(0)",
               "ds_read_b128 v[2:5], v6", "v_mfma_f32_16x16x32_bf16 v[0:3], v[2:5], v[2:5], v[0:3]"]
    assert isa_check.drains(drained) == [1]
    loop_head = ["buffer_load_dwordx4 v1, s[0:3], 0 offen lds", "s_waitcnt vmcnt(0)",
                 "s_waitcnt lgkmcnt(0)", "s_barrier", "ds_read_b128 v[2:5], v6"]
    assert isa_check.drains(loop_head) == []
    assert isa_check.template_args(
        "_ZN12_GLOBAL__N_110igemm_gldsILi256ELi64ELi8ELi1ELi3ELi0ELi2EEEvNS_9IgemmArgsE") == \
        [256, 64, 8, 1, 3, 0, 2]
    m0_ok = ["s_mov_b32 m0, s4", "s_nop 0", "buffer_load_dwordx4 v1, s[0:3], 0 offen lds"]
    assert isa_check.opaque(m0_ok) and isa_check.m0_violations(m0_ok) == []
    assert isa_check.m0_violations(m0_ok + ["s_mov_b32 m0, -1", "s_sendmsg sendmsg(MSG_GS)"])
