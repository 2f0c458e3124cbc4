"""ISA check of the shipped library (CPU, no GPU needed): no kernel that issues MFMAs also
issues packed-FP32 VALU (co-residency corruption; tools/isa_check.py)."""
import os
import sys

import pytest

from conftest import PKG, REPO

sys.path.insert(0, os.path.join(REPO, "tools"))
LIB = os.path.join(PKG, "qnn", "libqnn_hip.so")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"), reason="needs ROCm llvm-objdump")
def test_no_packed_fp32_in_mfma_kernels():
    import isa_check
    assert os.path.exists(LIB), "build the library first (make -C quantized.pytorch_amd)"
    n, bad = isa_check.check(LIB)
    assert n >= 100, f"only {n} MFMA kernels found: code-object extraction broken?"
    assert not bad, [f"{k[:100]}: {i}" for k, i in bad[:5]]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"), reason="needs ROCm llvm-objdump")
def test_no_counted_lgkm_wait_with_scalar_load_in_flight():
    """scalar-memory loads share LGKM_CNT with LDS ops but return out of order;
    no `s_waitcnt lgkmcnt(N > 0)` of the shipped kernels may be issued while one is in flight
    (tools/isa_check.py smem_lgkm_check; tools/asm_lgkm_check.py runs the same check on the
    assembly listings, where it also separates hand-counted waits from the compiler's)."""
    import isa_check
    n, bad = isa_check.smem_lgkm_check(LIB)
    assert n >= 100, f"only {n} kernels found: code-object extraction broken?"
    assert not bad, [f"{k[:100]}: {i}" for k, i in bad[:5]]


def test_lgkm_hazard_dataflow():
    """The check follows branches: a counted wait behind a scalar load is flagged on the path that
    reaches it, a wait only reachable after lgkmcnt(0) or past an unconditional branch is not."""
    import isa_check

    def prog(lines):
        return [f"{t}  // {0x1000 + 4 * k:012X}: 00000000" for k, t in enumerate(lines)]

    straight = prog(["s_load_dword s0, s[0:1], 0x0", "ds_read_b32 v0, v1", "s_waitcnt lgkmcnt(1)", "s_endpgm"])
    assert len(isa_check.lgkm_hazards(straight)) == 1
    cleared = prog(["s_load_dword s0, s[0:1], 0x0", "s_waitcnt lgkmcnt(0)", "s_waitcnt lgkmcnt(1)", "s_endpgm"])
    assert isa_check.lgkm_hazards(cleared) == []
    # k=1 branches over the load to the wait at k=4 (imm 2: next instruction + 2 dwords)
    skipped = prog(["s_nop 0", "s_branch 2", "s_load_dword s0, s[0:1], 0x0", "s_endpgm",
                    "s_waitcnt lgkmcnt(1)", "s_endpgm"])
    assert isa_check.lgkm_hazards(skipped) == []
    # a backward branch from a load's path into a wait
    looped = prog(["s_branch 3", "s_waitcnt lgkmcnt(2)", "s_endpgm", "s_nop 0",
                   "s_load_dword s0, s[0:1], 0x0", "s_branch 65531"])
    assert len(isa_check.lgkm_hazards(looped)) == 1
    assert isa_check.lgkm_hazards(prog(["s_load_dword s0, s[0:1], 0x0", "s_waitcnt lgkmcnt(15)", "s_endpgm"])) == []
