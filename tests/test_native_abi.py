"""CPU-side checks of the C ABI: the library loads, exports every function
declared in include/movierec_ncf.h, validates shapes and sizes workspaces
(host-only entry points; no kernel launches)."""

import ctypes
import os
import re

import pytest

from movierec import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    text = open(os.path.join(ROOT, "include", "movierec_ncf.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(ncf_\w+)\s*\(", text, re.M)))


def test_header_and_binding_agree():
    assert _declared() == N.EXPORTED


def test_library_exports_every_symbol():
    L = N.lib()
    for name in _declared():
        assert hasattr(L, name), name
    assert L.ncf_abi_version() == N.ABI_VERSION == 11


def test_library_links_no_vendor_blas():
    """Every matrix product is a hand-written MFMA kernel: the library neither needs a BLAS
    library nor references one of its symbols (the rocBLAS layered path is gone)."""
    import subprocess
    needed = subprocess.run(["readelf", "-d", N.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "blas" not in needed.lower(), needed
    syms = subprocess.run(["nm", "-D", N.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "rocblas" not in syms.lower() and "hipblas" not in syms.lower()


def test_build_info_matches_the_tree():
    """The loaded library carries the SHA-256 of the sources it was built from (ncf_build_info);
    for the product library it equals the tree's hash and lists no experiment defines, so the
    benched binary is provably the committed code."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "ncf_build", os.path.join(ROOT, "movierecommender-tf-trt_amd", "csrc", "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    info = N.build_info()
    assert info["arch"] == "gfx950" and info["abi"] == N.ABI_VERSION
    assert info["src_sha256"] == b.embedded_hash(N.LIB_PATH)
    if not os.environ.get("NCF_LIB"):
        assert info["defines"] == ""
        assert info["src_sha256"] == b.source_hash(), "the library is stale: run __graft_entry__.build()"


def _shape(nu, ni, layers, g):
    s = N.NcfShape()
    arr = (ctypes.c_int32 * len(layers))(*layers)
    N.check(N.lib().ncf_shape_init(ctypes.byref(s), nu, ni, arr, len(layers), g))
    return s


def test_shape_init_derivations():
    s = _shape(138493, 27278, [128, 64, 32, 16], 64)
    assert (s.du, s.di, s.gmf_stride, s.row_width) == (64, 64, 64, 128)
    assert s.num_rows == 138493 + 27278
    assert s.out_features == 80
    assert s.mlp_params == 128 * 64 + 64 + 64 * 32 + 32 + 32 * 16 + 16 + 80 + 1
    s = _shape(5, 10, [7, 4], 3)   # odd split: du=3, di=4 (model.py:159-160)
    assert (s.du, s.di, s.gmf_stride, s.row_width) == (3, 4, 4, 8)


def test_shape_init_gmf_only():
    """BASELINE config A: ml-100k GMF-only (layers_sizes == [], gmf_dim 8): rows hold the GMF
    vectors only, the output layer reads the product alone; the host Layout agrees."""
    from movierec.layout import Layout
    s = _shape(943, 1682, [], 8)
    assert (s.num_layers, s.du, s.di, s.gmf_stride, s.row_width) == (0, 0, 0, 8, 8)
    assert (s.out_features, s.mlp_params, s.fast_path) == (8, 9, 0)
    lay = Layout(943, 1682, [], 8)
    assert (lay.row_width, lay.mlp_params, lay.out_features) == (s.row_width, s.mlp_params, s.out_features)
    assert lay.weight_names() == ["user_gmf_embedding", "item_gmf_embedding", "output/kernel", "output/bias"]
    assert N.lib().ncf_score_supported(ctypes.byref(s), N.NCF_SCORE_FP16) == 0
    s = _shape(10, 12, [], 5)   # gmf not a multiple of 4: padded rows
    assert (s.gmf_stride, s.row_width, s.mlp_params) == (8, 8, 6)


def test_shape_init_rejects_bad_dims():
    s = N.NcfShape()
    arr = (ctypes.c_int32 * 2)(0, 4)
    with pytest.raises(ValueError):
        N.check(N.lib().ncf_shape_init(ctypes.byref(s), 5, 10, arr, 2, 0))
    with pytest.raises(ValueError):
        N.check(N.lib().ncf_shape_init(ctypes.byref(s), 5, 10, arr, 0, 0))


def test_workspace_size_scales_with_batch():
    s = _shape(6040, 3952, [64, 32, 16, 8], 8)
    a, b = ctypes.c_size_t(), ctypes.c_size_t()
    N.check(N.lib().ncf_workspace_size(ctypes.byref(s), 1024, ctypes.byref(a)))
    N.check(N.lib().ncf_workspace_size(ctypes.byref(s), 4096, ctypes.byref(b)))
    assert b.value > a.value > 0
    with pytest.raises(ValueError):
        N.check(N.lib().ncf_workspace_size(ctypes.byref(s), 0, ctypes.byref(a)))


def test_score_support_and_workspace():
    L = N.lib()
    c = _shape(138493, 27278, [128, 64, 32, 16], 64)
    assert L.ncf_score_supported(ctypes.byref(c), N.NCF_SCORE_FP16) == 1
    assert L.ncf_score_supported(ctypes.byref(c), N.NCF_SCORE_FP32) == 1
    d = _shape(1000, 500, [256, 128, 64, 32], 128)   # config D widths: fp32 scorer only
    assert L.ncf_score_supported(ctypes.byref(d), N.NCF_SCORE_FP16) == 0
    a, b = ctypes.c_size_t(), ctypes.c_size_t()
    N.check(L.ncf_score_workspace_size(ctypes.byref(c), 32, ctypes.byref(a)))
    N.check(L.ncf_score_workspace_size(ctypes.byref(c), 138493, ctypes.byref(b)))
    assert b.value > a.value > 0
    with pytest.raises(ValueError):
        N.check(L.ncf_score_workspace_size(ctypes.byref(c), 0, ctypes.byref(a)))
