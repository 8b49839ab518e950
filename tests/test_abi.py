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


OPS = ("se_fwd", "cbam_fwd", "ca_fwd", "a2_fwd", "swin_fwd", "detect_head_fwd", "detect_decode_fwd", "nms_batched")


def test_torch_op_library_registers_the_kernel_families():
    """one torch op per kernel family (csrc/torch_ops.cpp, a cpp_extension over the C ABI); Meta
    kernels give output shapes without a GPU, and a CPU tensor reaches no kernel (no CPU implementation)."""
    ops = _hip.ops()
    for n in OPS:
        assert hasattr(ops, n), n
    m = torch.empty(2, 64, 20, 20, device="meta")
    assert ops.se_fwd(m, m, m, m, m, None).shape == m.shape
    assert ops.swin_fwd(m, 2, 7, *([m] * 3), 1e-5, *([m] * 6), 1e-5, *([m] * 9), 1e-3).shape == m.shape
    feats = [torch.empty(3, 64, s, s, device="meta") for s in (16, 8, 4, 2)]
    y = ops.detect_head_fwd(feats, feats, feats, feats, feats, feats, [4.0, 8.0, 16.0, 32.0], 10, 16)
    assert tuple(y.shape) == (3, 14, 16 * 16 + 8 * 8 + 4 * 4 + 2 * 2)
    out, counts, index = ops.nms_batched(torch.empty(3, 14, 100, device="meta"), 0.25, 0.7, None, False, False, 300,
                                         30000, 7680.0)
    assert tuple(out.shape) == (3, 300, 6) and tuple(counts.shape) == (3,) and tuple(index.shape) == (3, 300)
    with pytest.raises((RuntimeError, NotImplementedError)):
        ops.se_fwd(torch.zeros(1, 8, 4, 4), *[torch.zeros(1)] * 4, None)
