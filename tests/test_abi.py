"""The C-ABI library loads, exports every symbol include/qnn.h declares, and
validates arguments before touching the device (CPU-only checks)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO

HEADER = os.path.join(REPO, "include", "qnn.h")
LIB = os.path.join(PKG, "qnn", "libqnn_hip.so")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(qnn_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)
    from qnn import _lib
    return _lib.load()


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("qnn_qconv2d_fwd", "qnn_pack_weight_i8", "qnn_quantize_nchw_to_nhwc8", "qnn_fake_quant_f32",
              "qnn_rangebn_f32", "qnn_dwconv2d_fwd", "qnn_last_error", "qnn_abi_version"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True, text=True).stdout
    exported = set(re.findall(r"\sT\s(qnn_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_bindings_cover_every_symbol(lib):
    from qnn import _lib
    for s in declared_symbols():
        if s in ("qnn_last_error", "qnn_abi_version", "qnn_conv_tile_count", "qnn_conv_tile_kernel",
                 "qnn_measure_stats_work"):
            continue
        assert s in _lib.SIGNATURES, s


def test_abi_version(lib):
    from qnn import _lib
    assert lib.qnn_abi_version() == _lib.ABI_VERSION == 9


def test_header_constants_match_bindings():
    from qnn import _lib
    src = open(HEADER).read()
    defs = dict(re.findall(r"^#define\s+(QNN_\w+)\s+(\d+)", src, flags=re.M))
    assert int(defs["QNN_ABI_VERSION"]) == _lib.ABI_VERSION
    assert int(defs["QNN_MAX_RES"]) == _lib.MAX_RES
    assert int(defs["QNN_COMM_ID_BYTES"]) == _lib.COMM_ID_BYTES


def test_argument_validation_without_device(lib):
    import ctypes
    from qnn import _lib
    # invalid arguments are rejected before any HIP call, with a message
    rc = lib.qnn_fake_quant_f32(None, None, 16, 0.0, 0.0, 0.0, 255.0, None)
    assert rc == 1
    assert b"scale" in lib.qnn_last_error() or b"null" in lib.qnn_last_error()
    d = _lib.ConvDesc(n=1, hp=10, wp=10, cp=24, zero_off=0, cout=64, cout_pad=64, kh=3, kw=3, sh=1, sw=1, ho=8, wo=8,
                      kpad=256)
    e = _lib.Epilogue(mode=0, nwc=1, nclass=1)
    rc = lib.qnn_qconv2d_fwd(None, None, ctypes.byref(d), ctypes.byref(e), None)
    assert rc == 1 and b"cp" in lib.qnn_last_error()
    d.cp, d.ho = 16, 9
    rc = lib.qnn_qconv2d_fwd(None, None, ctypes.byref(d), ctypes.byref(e), None)
    assert rc == 1 and b"ho/wo" in lib.qnn_last_error()
    d.ho, d.kpad = 8, 100
    rc = lib.qnn_qconv2d_fwd(None, None, ctypes.byref(d), ctypes.byref(e), None)
    assert rc == 1 and b"kpad" in lib.qnn_last_error()
    rc = lib.qnn_fake_quant_vec_f32(None, None, 70000, 255.0, 0, None, None)
    assert rc == 1
    rc = lib.qnn_quantize_nchw_to_s2d8(None, None, 1, 5, 8, 8, 1, 5, 5, 0.0, 1.0, 255.0, None)
    assert rc == 1  # 4*c > 16
    # empty batches are a no-op success
    assert lib.qnn_fake_quant_f32(None, None, 0, 0.0, 0.0, 1.0, 255.0, None) == 0


def test_tile_kernel_families(lib):
    """qnn_conv_tile_kernel names every configuration's device function (no GPU work)."""
    from qnn import _lib
    fams = [_lib.tile_kernel(k) for k in range(_lib.CONV_TILES)]
    assert set(fams) == {"qconv_kernel", "qconv_pp_kernel", "qconv_band_kernel", "qconv16_kernel",
                         "qconv_rb_kernel", "qconv_direct_kernel", "qconv_rbp_kernel", "qconv_dtab_kernel",
                         "qconv_pb_kernel", "qconv_rs_kernel"}
    # families are contiguous id ranges; round 4 appended the two-team resident band, then the
    # table-epilogue direct configurations (ids of earlier families never move)
    runs = [f for i, f in enumerate(fams) if i == 0 or fams[i - 1] != f]
    # the ring family is split by the ping-pong ids 6-9 and again by ids 12-49 (round 5 appended
    # ring configurations 50-55), the direct family by ids 40-43 (the classifier head, 44, is a
    # direct-fragment configuration appended in round 4)
    assert len(runs) == len(set(runs)) + 3
    assert len(_lib.tile_ids("qconv_direct_kernel")) == 6 and _lib.tile_ids("qconv_direct_kernel")[-1] == 44
    assert _lib.tile_ids("qconv_rbp_kernel") == [40, 41]
    assert _lib.tile_ids("qconv_dtab_kernel") == [42, 43]
    assert fams[44] == "qconv_direct_kernel"
    # round 5 appended the persistent-band configurations 45-49
    assert _lib.tile_ids("qconv_pb_kernel") == [45, 46, 47, 48, 49]
    assert [fams[k] for k in range(50, 56)] == ["qconv_kernel"] * 6
    # round 6 appended the streamed resident-band configurations 56-63
    assert _lib.tile_ids("qconv_rs_kernel") == list(range(56, 64)) and len(fams) == 64
    assert lib.qnn_conv_tile_kernel(-1) is None and lib.qnn_conv_tile_kernel(_lib.CONV_TILES) is None


def test_struct_layout_matches_header():
    """ctypes mirrors of qnn_conv_desc / qnn_epilogue have the C field order."""
    import re as _re
    from qnn import _lib
    src = open(HEADER).read()
    for cname, py in (("qnn_conv_desc", _lib.ConvDesc), ("qnn_epilogue", _lib.Epilogue),
                      ("qnn_bn_params", _lib.BnParams), ("qnn_code_out", _lib.CodeOut),
                      ("qnn_res_link", _lib.ResLink)):
        body = _re.search(r"typedef struct " + cname + r" \{(.*?)\} " + cname, src, _re.S).group(1)
        body = _re.sub(r"/\*.*?\*/", "", body, flags=_re.S)
        names = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            decl = _re.sub(r"^(const\s+)?\w+\s*\*?\s*", "", decl)
            names += [_re.sub(r"\[.*\]", "", n.strip().lstrip("*")) for n in decl.split(",")]
        assert names == [f[0] for f in py._fields_], cname


def test_error_is_thread_local(lib):
    import threading
    lib.qnn_fake_quant_vec_f32(None, None, 0, 255.0, 0, None, None)
    mine = lib.qnn_last_error()
    seen = []

    def other():
        seen.append(lib.qnn_last_error())

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert mine and seen == [b""]


def test_built_for_gfx950_only():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", LIB], capture_output=True, text=True)
    blob = open(LIB, "rb").read()
    assert b"gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob


def test_conv_plan_every_configuration_host_only(lib):
    """qnn_conv_plan (host code only: configuration filters and the cost model) for the benched
    layer shapes, with the cost-model choice and with every configuration forced: returns a
    configuration or refuses it with a message, never crashes (a cost-model table indexed past its
    family's end once divided by zero here)."""
    import ctypes
    from qnn import _lib
    shapes = [  # (n, cin_pad, cout, k, stride, hw)
        (128, 64, 64, 3, 1, 56), (128, 512, 512, 3, 1, 7), (256, 256, 256, 3, 1, 14), (256, 64, 256, 1, 1, 56),
        (128, 256, 512, 1, 2, 14), (37, 2048, 1000, 1, 1, 1)]
    for n, cp, cout, k, st, hw in shapes:
        pad = k // 2
        ho = (hw + 2 * pad - k) // st + 1
        kpad = -(-k * k * cp // 128) * 128
        d = _lib.ConvDesc(n=n, hp=hw + 2 * pad, wp=hw + 2 * pad, cp=cp, zero_off=0, cout=cout, cout_pad=cout, kh=k,
                          kw=k, sh=st, sw=st, ho=ho, wo=ho, kpad=kpad)
        for mode in (0, 1):
            e = _lib.Epilogue(mode=mode, nwc=1, nclass=1)
            cfg, bm, bn, nb = (ctypes.c_int() for _ in range(4))
            for tile in range(_lib.CONV_TILES + 1):
                d.tile = tile
                rc = lib.qnn_conv_plan(ctypes.byref(d), ctypes.byref(e), ctypes.byref(cfg), ctypes.byref(bm),
                                       ctypes.byref(bn), ctypes.byref(nb))
                if tile == 0:
                    assert rc == 0 and 0 <= cfg.value < _lib.CONV_TILES
                if rc == 0:
                    assert bm.value > 0 and bn.value > 0 and nb.value > 0
                    assert tile == 0 or cfg.value == tile - 1
                else:
                    assert lib.qnn_last_error()
