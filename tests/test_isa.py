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
