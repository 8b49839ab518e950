"""CPU: the C-ABI library builds/loads, exports every entry point include/yolosod_hip.h declares, validates its
arguments before touching the GPU, and the product path refuses CPU tensors (no CPU fallback)."""
import ctypes
import re

import pytest
import torch

from conftest import ROOT
from yolosod_amd import _hip

HEADER = ROOT / "include" / "yolosod_hip.h"


def declared():
    txt = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(yolosod_\w+)\s*\(", txt, re.M)))


def test_header_declares_entry_points():
    names = declared()
    for n in ("yolosod_se_forward", "yolosod_cbam_forward", "yolosod_ca_forward", "yolosod_a2_forward",
              "yolosod_swin_forward", "yolosod_detect_decode", "yolosod_nms"):
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = _hip.load_library()
    for n in declared():
        assert hasattr(lib, n), n
        assert n in _hip.SIGNATURES, f"{n} has no ctypes signature"
    assert lib.yolosod_abi_version() == 1


def test_argument_validation_without_gpu():
    lib = _hip.load_library()
    rc = lib.yolosod_se_forward(None, None, 1, 8, 4, 4, None, None, None, None, 4, None, 0, None)
    assert rc != 0 and b"null" in lib.yolosod_last_error()
    rc = lib.yolosod_nms(ctypes.c_void_p(16), 1, 0, 10, 0.25, 0.7, None, 0, 0, 0, 300, 30000, 7680.0, 1,
                         ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16), None, 0, None)
    assert rc != 0 and b"nc=0" in lib.yolosod_last_error()
    rc = lib.yolosod_attention(ctypes.c_void_p(16), ctypes.c_void_p(16), 1, 400, 64, 2, None)
    assert rc != 0 and b"sequence length" in lib.yolosod_last_error()
    rc = lib.yolosod_detect_decode(5, None, None, None, None, 1, 10, 16, None, None)
    assert rc != 0 and b"nl=5" in lib.yolosod_last_error()


def test_workspace_queries():
    lib = _hip.load_library()
    assert lib.yolosod_se_workspace(32, 32, 320, 320) >= 32 * 32 * 4
    assert lib.yolosod_swin_workspace(32, 64, 160, 160, 7, 128) >= 32 * 529 * 49 * 64 * 4 * 2
    assert lib.yolosod_nms_workspace(32, 10, 34000, 1) >= 32 * 34000 * 10 * 16


def test_product_ops_refuse_cpu_tensors():
    from yolosod_amd.nn import modules as M
    x = torch.randn(1, 32, 8, 8)
    se = M.SE_Block(16)
    with pytest.raises(RuntimeError, match="GPU"):
        se(x)
    with pytest.raises(RuntimeError, match="GPU"):
        M.CBAM_Block(32, None, 8).eval()(x)
    from yolosod_amd.utils.ops import non_max_suppression
    with pytest.raises(RuntimeError, match="GPU"):
        non_max_suppression(torch.rand(1, 14, 100))
