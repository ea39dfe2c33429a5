"""libyoloxhip.so loads on the CPU host and exports every symbol of include/yoloxhip.h.
No compute calls (no GPU here); only argument-validation paths that return before
touching the HIP runtime."""
import ctypes
import os
import re

import pytest

from conftest import REPO


def header_symbols():
    text = open(os.path.join(REPO, "include", "yoloxhip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|void|const char\*)\s+(yxh_\w+)\s*\(", text, re.M)))


def test_library_exports_every_header_symbol():
    from yolox_amd import _native as N
    lib = N.lib()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(N.EXPORTED)


def test_abi_and_struct_layout():
    from yolox_amd import _native as N
    lib = N.lib()
    assert lib.yxh_abi_version() == N.ABI_VERSION
    assert lib.yxh_sizeof_op() == ctypes.sizeof(N.Op)
    assert lib.yxh_sizeof_conv_desc() == ctypes.sizeof(N.ConvDesc)


def test_argument_errors_are_reported_without_a_device():
    from yolox_amd import _native as N
    lib = N.lib()
    assert lib.yxh_conv2d(None, None) == N.EINVAL
    assert b"null" in lib.yxh_last_error()
    d = N.ConvDesc()
    d.dtype = 7
    assert lib.yxh_conv2d(ctypes.byref(d), None) == N.EINVAL
    assert b"dtype" in lib.yxh_last_error()
    with pytest.raises(ValueError, match="dtype"):
        N.check(lib.yxh_conv2d(ctypes.byref(d), None), "conv")
    assert lib.yxh_graph_destroy(None) == N.OK
    assert lib.yxh_run_ops(None, 0, None) == N.OK


def test_postprocess_workspace_is_monotone():
    from yolox_amd import _native as N
    lib = N.lib()
    a = lib.yxh_postprocess_workspace_bytes(1, 336)
    b = lib.yxh_postprocess_workspace_bytes(32, 8400)
    c = lib.yxh_postprocess_workspace_bytes(32, 33600)
    assert 0 < a < b < c
    # the suppression matrix is built in budgeted row passes: linear in A past the budget
    # (was B * A * ceil(A/64) * 8 = 9.0 GB at 32 x 33600)
    assert c < 700 << 20
    assert lib.yxh_postprocess_workspace_bytes(1, 1 << 19) < 600 << 20
    lib.yxh_set_nms_mask_budget(1 << 16)
    try:
        assert lib.yxh_postprocess_workspace_bytes(32, 8400) < b
    finally:
        lib.yxh_set_nms_mask_budget(0)
    assert lib.yxh_postprocess_workspace_bytes(32, 8400) == b


def test_library_targets_gfx950_only():
    from yolox_amd import _native as N
    blob = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    for other in (b"gfx90a", b"gfx942", b"sm_"):
        assert b"amdgcn-amd-amdhsa--" + other not in blob


def test_no_shipped_kernel_uses_scratch():
    """Every gfx950 kernel in libyoloxhip.so keeps its state in registers / LDS: no kernel's
    code-object metadata reports a private segment (scratch spills cost vmcnt waits that drain
    the LDS-DMA pipelines).  tools/kernel_resources.py reads the metadata of every offload
    bundle in the library's .hip_fatbin section."""
    import importlib.util
    import shutil
    if not shutil.which("/opt/rocm/lib/llvm/bin/llvm-readelf"):
        pytest.skip("ROCm LLVM tools not installed")
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "kernel_resources.py")
    spec = importlib.util.spec_from_file_location("kernel_resources", path)
    kr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(kr)
    ks = kr.kernels()
    assert len(ks) > 300  # every translation unit's bundle was read
    spills = sorted((v["scratch"], k) for k, v in ks.items() if v.get("scratch", 0) > 0)
    assert not spills, spills[:10]
