"""GPU: the Detect head's 3x3 tower convs on the fp16 two-term split implicit-GEMM kernel (csrc/conv3x3.hip) against
the exact (fp64) conv + bias + SiLU of the same fp32 weights (ultralytics/nn/modules/head.py:43-57, conv.py:37-55),
next to the MIOpen fp32 path's own error; ragged tiles, every tower input width, the split-range guard, and the
whole tower module path (Conv.tower -> conv_epilogue)."""
import pytest
import torch
import torch.nn.functional as F

from oplib import tol_close
from yolosod_amd import _hip

pytestmark = pytest.mark.gpu


def _ref64(x, w, b):
    return F.silu(F.conv2d(x.double(), w.double(), b.double(), padding=1))


@pytest.mark.parametrize("shape", [(2, 64, 37, 45), (1, 128, 20, 20), (2, 32, 9, 7), (1, 512, 20, 20),
                                   (2, 256, 40, 40), (1, 64, 160, 160), (3, 64, 8, 32), (1, 96, 1, 1)])
def test_conv3x3_matches_fp64(shape, cuda):
    g = torch.Generator().manual_seed(sum(shape))
    B, cin, H, W = shape
    x = torch.randn(shape, generator=g)
    w = torch.randn(64, cin, 3, 3, generator=g) * (1.0 / (3 * cin ** 0.5))
    b = torch.randn(64, generator=g) * 0.1
    ref = _ref64(x, w, b)
    wd = w.to(cuda)
    y = _hip.conv3x3_silu(x.to(cuda), b.to(cuda), lambda: _hip.conv3x3_prepare(wd)).cpu().double()
    miopen = F.silu(F.conv2d(x.to(cuda), wd, b.to(cuda), padding=1)).cpu().double()
    err, err_m = float((y - ref).abs().max()), float((miopen - ref).abs().max())
    ok, e, ratio = tol_close(y, ref, 5e-5, 1e-4)
    assert ok, f"{shape}: max abs err {e:.3g} (MIOpen fp32 {err_m:.3g})"
    # fp32 accumulation of Cin * 9 products per output: within a few times MIOpen's own error (its Winograd / direct
    # kernels sum in a different order), e.g. 7.5e-6 vs 1.5e-6 at Cin = 512
    assert err <= 8 * err_m + 1e-5, (err, err_m)


def test_conv3x3_range_guard(cuda):
    x = torch.randn(1, 64, 16, 16, device=cuda)
    w = torch.randn(64, 64, 3, 3, device=cuda) * 0.05
    b = torch.zeros(64, device=cuda)
    prep = _hip.conv3x3_prepare(w)
    _hip.split_range_flag(reset=True)
    _hip.conv3x3_silu(x, b, lambda: prep)
    assert not _hip.split_range_flag(reset=True)
    _hip.conv3x3_silu(x * 1e5, b, lambda: prep)  # activations beyond fp16's range
    assert _hip.split_range_flag(reset=True)
    big = _hip.conv3x3_prepare(w * 2e4)  # 64 W beyond 65504: flagged by the preparation and by every later launch
    _hip.split_range_flag(reset=True)
    for _ in range(2):
        _hip.conv3x3_silu(x, b, lambda: big)
        assert _hip.split_range_flag(reset=True)


def test_tower_convs_take_the_kernel(cuda, monkeypatch):
    """The Detect tower convs route to the kernel (op_timer records 'conv3x3' launches) and match the MIOpen path
    (YOLOSOD_CONV3X3=0) within fp32 accuracy."""
    from yolosod_amd.nn import modules as M
    from yolosod_amd.nn.tasks import build_model
    m = build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=cuda)
    x = torch.rand(2, 3, 256, 256, generator=torch.Generator().manual_seed(4)).to(cuda)
    monkeypatch.setattr(M, "CONV3X3", "1")  # the tower convs on the fp16-split kernel (the default)
    monkeypatch.setattr(M, "S1_NECK", False)  # (the neck's Bottleneck convs: test_neck_c2f_convs_take_the_kernel)
    with torch.inference_mode():
        with _hip.op_timer() as t:
            y = m(x)[0]
        keys = [k[0] for k, _ in t.durations_ms()]
        monkeypatch.setattr(M, "CONV3X3", "0")
        y0 = m(x)[0]
    assert keys.count("conv3x3") == 16  # 4 levels x (box, class) x 2 convs
    ok, e, _ = tol_close(y.cpu().double(), y0.cpu().double(), 1e-3, 1e-4)
    assert ok, e


@pytest.mark.parametrize("shape,cout", [((2, 32, 40, 48), 32), ((2, 128, 24, 24), 128), ((1, 256, 20, 20), 256),
                                        ((2, 64, 17, 28), 64)])
def test_conv3x3_groups_out_res_match_fp64(shape, cout, cuda):
    """Cout 32 / multiples of 64 (output groups of 32 / 64 channels), the residual added after the activation and the
    output written into a concat slice (the neck's C2f Bottleneck cv2: x + SiLU(conv(cv1(x))), block.py:343)."""
    g = torch.Generator().manual_seed(sum(shape) + cout)
    B, cin, H, W = shape
    x = torch.randn(shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * (1.0 / (3 * cin ** 0.5))
    b = torch.randn(cout, generator=g) * 0.1
    r = torch.randn(B, cout, H, W, generator=g)
    ref = F.silu(F.conv2d(x.double(), w.double(), b.double(), padding=1))
    wd = w.to(cuda)
    prep = _hip.conv3x3_prepare(wd)
    y = _hip.conv3x3_silu(x.to(cuda), b.to(cuda), lambda: prep, cout).cpu().double()
    miopen = F.silu(F.conv2d(x.to(cuda), wd, b.to(cuda), padding=1)).cpu().double()
    err, err_m = float((y - ref).abs().max()), float((miopen - ref).abs().max())
    ok, e, _ = tol_close(y, ref, 5e-5, 1e-4)
    assert ok, f"{shape}: max abs err {e:.3g} (MIOpen fp32 {err_m:.3g})"
    assert err <= 8 * err_m + 1e-5, (err, err_m)
    if W % 4 == 0:  # residual + concat slice: bit-identical to the plain output + res (the add is the last op)
        buf = torch.full((B, cout + 64, H, W), float("nan"), device=cuda)
        out = buf[:, 32:32 + cout]
        _hip.conv3x3_silu(x.to(cuda), b.to(cuda), lambda: prep, cout, out=out, res=r.to(cuda))
        y0 = _hip.conv3x3_silu(x.to(cuda), b.to(cuda), lambda: prep, cout)
        assert torch.equal(out, y0 + r.to(cuda))
        assert torch.isnan(buf[:, :32]).all() and torch.isnan(buf[:, 32 + cout:]).all()


def test_neck_c2f_convs_take_the_kernel(cuda, monkeypatch):
    """The neck C2fs' Bottleneck 3x3 convs (12 at the paper scale) route to the stride-1 kernel and the model matches
    the MIOpen path (YOLOSOD_S1_NECK=0) within fp32 accuracy."""
    from yolosod_amd.nn import modules as M
    from yolosod_amd.nn.tasks import build_model
    m = build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=cuda)
    x = torch.rand(2, 3, 640, 640, generator=torch.Generator().manual_seed(5)).to(cuda)  # (at 320, P5 is 10 wide)
    with torch.inference_mode():
        with _hip.op_timer() as t:
            y = m(x)[0]
        n1 = sum(1 for k, _ in t.durations_ms() if k[0] == "conv3x3")
        monkeypatch.setattr(M, "S1_NECK", False)
        with _hip.op_timer() as t:
            y0 = m(x)[0]
        n0 = sum(1 for k, _ in t.durations_ms() if k[0] == "conv3x3")  # the Detect towers only
    assert n1 - n0 == 12, (n1, n0)
    ok, e, _ = tol_close(y.cpu().double(), y0.cpu().double(), 1e-3, 1e-4)
    assert ok, e


@pytest.mark.parametrize("cout,res", [(64, False), (32, True), (128, True)])
def test_conv3x3_slice_input_bit_identical(cout, res, cuda):
    """The input as a channel slice of a wider buffer (yolosod_conv3x3_silu_xs: the neck C2f's Bottleneck reading its
    input inside the C2f buffer), residual a slice too: bit-identical to the packed input."""
    g = torch.Generator().manual_seed(cout + res)
    cin = cout if res else 64
    buf = torch.randn(2, cin + 96, 24, 40, generator=g).to(cuda)
    x = buf[:, 32:32 + cin]
    w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(cuda)
    b = (torch.randn(cout, generator=g) * 0.1).to(cuda)
    prep = _hip.conv3x3_prepare(w)
    r = x if res else None
    y0 = _hip.conv3x3_silu(x.contiguous(), b, lambda: prep, cout, res=None if r is None else r.contiguous())
    y = _hip.conv3x3_silu(x, b, lambda: prep, cout, res=r)
    assert torch.equal(y, y0)


def test_model_neck_c2f_slices_bit_identical(cuda, monkeypatch):
    """The neck C2fs' Bottlenecks reading their inputs as slices of the C2f buffer (modules.C2F_SLICES) give the
    dual-store form's output bit for bit."""
    from yolosod_amd.nn import modules as M
    from yolosod_amd.nn.tasks import build_model
    m = build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=cuda)
    x = torch.rand(2, 3, 640, 640, generator=torch.Generator().manual_seed(12)).to(cuda)
    torch.backends.cudnn.deterministic = True
    try:
        with torch.inference_mode():
            monkeypatch.setattr(M, "C2F_SLICES", True)
            y = m(x)[0]
            monkeypatch.setattr(M, "C2F_SLICES", False)
            y0 = m(x)[0]
    finally:
        torch.backends.cudnn.deterministic = False
    assert torch.equal(y, y0), float((y - y0).abs().max())
