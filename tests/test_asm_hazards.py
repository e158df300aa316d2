"""Device-code hazard gate (CPU): no hand-written VMEM instruction may read an SGPR that a VALU op wrote fewer than
five wait states before (tools/sgpr_hazard.py). The compiler pads its own instructions but not inline asm; the one
such hazard found (gemm4w's direct-epilogue stores behind a v_readlane spill reload) faulted the GPU in round 4."""
import glob
import os
import shutil

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _objects():
    return sorted(glob.glob(os.path.join(ROOT, "build", "kernels", "*.o")))


@pytest.mark.skipif(not shutil.which("/opt/rocm/lib/llvm/bin/llvm-objdump"), reason="no ROCm LLVM tools")
def test_no_valu_sgpr_to_vmem_hazards():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import sgpr_hazard
    objs = _objects()
    if not objs:
        pytest.skip("kernel objects not built (make all)")
    found = []
    for o in objs:
        found += sgpr_hazard.scan(sgpr_hazard.disassemble(o), os.path.basename(o))
    assert not found, "\n".join(found[:20])


def test_scanner_flags_a_short_gap():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import sgpr_hazard
    bad = "\tv_readlane_b32 s3, v255, 5\n\ts_nop 1\n\tbuffer_store_dwordx4 v[4:7], v8, s[0:3], 0 offen\n"
    good = "\tv_readlane_b32 s3, v255, 5\n\ts_nop 4\n\tbuffer_store_dwordx4 v[4:7], v8, s[0:3], 0 offen\n"
    fixed = "\tv_readlane_b32 s3, v255, 5\n\ts_mov_b32 s3, 0\n\tbuffer_store_dwordx4 v[4:7], v8, s[0:3], 0 offen\n"
    assert len(sgpr_hazard.scan(bad)) == 1
    assert sgpr_hazard.scan(good) == []
    assert sgpr_hazard.scan(fixed) == []


def test_scanner_checks_lds_dma_and_source_only_salu():
    """the LDS-DMA form has three operands (vaddr, srsrc, soffset) and reads m0; s_cmp / s_bitcmp read
    their first operand, so they must not clear a pending VALU -> SGPR hazard"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import sgpr_hazard
    dma_bad = "\tv_readfirstlane_b32 s2, v0\n\ts_nop 0\n\tbuffer_load_dwordx4 v1, s[0:3], 0 offen lds\n"
    dma_ok = "\tv_readfirstlane_b32 s2, v0\n\ts_nop 4\n\tbuffer_load_dwordx4 v1, s[0:3], 0 offen lds\n"
    m0_bad = "\tv_readfirstlane_b32 m0, v0\n\tbuffer_load_dwordx4 v1, s[4:7], 0 offen lds\n"
    cmp_bad = ("\tv_readlane_b32 s3, v255, 5\n\ts_cmp_eq_u32 s3, 0\n"
               "\tbuffer_store_dwordx4 v[4:7], v8, s[0:3], 0 offen\n")
    assert len(sgpr_hazard.scan(dma_bad)) == 1
    assert sgpr_hazard.scan(dma_ok) == []
    assert len(sgpr_hazard.scan(m0_bad)) == 1
    assert len(sgpr_hazard.scan(cmp_bad)) == 1
