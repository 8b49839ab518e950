"""GPU: the PAN neck's wide 1x1 convs on the fp16 two-term split kernel (csrc/conv1x1x2.hip) against the exact
(fp64) conv + bias + SiLU of the same fp32 weights (ultralytics/nn/modules/conv.py:37-55), next to MIOpen's own fp32
error: Cout groups of 128, Cin padded to 128 (192), pixel tails (HW not a multiple of 64), concat-slice input and
output, C2f's dual store; and the model's routing (YOLOSOD_N1_NECK) against the MIOpen path."""
import pytest
import torch
import torch.nn.functional as F

from oplib import tol_close
from yolosod_amd import _hip

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,cout", [((2, 256, 40, 40), 128), ((2, 192, 20, 20), 128), ((1, 768, 40, 40), 256),
                                        ((2, 1024, 20, 20), 512), ((1, 384, 12, 12), 256), ((3, 96, 8, 8), 128)])
def test_conv1x1x2_matches_fp64(shape, cout, cuda):
    g = torch.Generator().manual_seed(sum(shape) + cout)
    B, cin, H, W = shape
    x = torch.randn(shape, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) * (1.0 / cin ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    ref = F.silu(F.conv2d(x.double(), w.double(), b.double()))
    wd = w.to(cuda)
    y = _hip.conv1x1x2_silu(x.to(cuda), b.to(cuda), lambda: _hip.conv1x1x2_prepare(wd), cout).cpu().double()
    miopen = F.silu(F.conv2d(x.to(cuda), wd, b.to(cuda))).cpu().double()
    err, err_m = float((y - ref).abs().max()), float((miopen - ref).abs().max())
    ok, e, _ = tol_close(y, ref, 5e-5, 1e-4)
    assert ok, f"{shape}: max abs err {e:.3g} (MIOpen fp32 {err_m:.3g})"
    assert err <= 8 * err_m + 1e-5, (err, err_m)


def test_conv1x1x2_slices_and_dual_store(cuda):
    """Input and output as channel slices of concat buffers and the dual store of channels [c2lo, Cout): bit-identical
    to the contiguous form, the rest of the buffers untouched."""
    g = torch.Generator().manual_seed(9)
    xb = torch.randn(2, 320, 16, 20, generator=g).to(cuda)
    x = xb[:, 32:288]  # 256 channels, batch stride 320 * HW
    w = (torch.randn(256, 256, generator=g) * 0.06).to(cuda)
    b = (torch.randn(256, generator=g) * 0.1).to(cuda)
    prep = _hip.conv1x1x2_prepare(w)
    y0 = _hip.conv1x1x2_silu(x.contiguous(), b, lambda: prep, 256)
    z = torch.full((2, 384, 16, 20), float("nan"), device=cuda)
    t = torch.empty((2, 128, 16, 20), device=cuda)
    _hip.conv1x1x2_silu(x, b, lambda: prep, 256, out=z[:, :256], out2=t, c2lo=128)
    assert torch.equal(z[:, :256], y0) and torch.equal(t, y0[:, 128:])
    assert torch.isnan(z[:, 256:]).all()


def test_neck_wide_1x1_convs_take_the_kernel(cuda, monkeypatch):
    """The neck's wide 1x1 convs route to the kernel (those without a gate-statistics epilogue) and the model matches
    the MIOpen path (YOLOSOD_N1_NECK=0) within fp32 accuracy."""
    from yolosod_amd.nn import modules as M
    from yolosod_amd.nn.tasks import build_model
    m = build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=cuda)
    x = torch.rand(2, 3, 640, 640, generator=torch.Generator().manual_seed(6)).to(cuda)
    with torch.inference_mode():
        with _hip.op_timer() as t:
            y = m(x)[0]
        n = sum(1 for k, _ in t.durations_ms() if k[0] == "conv1x1x2")
        monkeypatch.setattr(M, "N1_NECK", False)
        y0 = m(x)[0]
    assert n >= 8, n
    ok, e, _ = tol_close(y.cpu().double(), y0.cpu().double(), 1e-3, 1e-4)
    assert ok, e


@pytest.mark.parametrize("shape,k1,cout", [((2, 256, 16, 20), 128, 128), ((1, 512, 20, 20), 256, 256),
                                           ((2, 384, 8, 8), 128, 256), ((1, 1024, 10, 10), 512, 512)])
def test_conv1x1x2_virtual_concat_bit_identical(shape, k1, cout, cuda):
    """A CatView (two parts read in place, the second from a channel slice) gives the materialised concat's output
    bit for bit, dual store included."""
    g = torch.Generator().manual_seed(k1 + cout)
    B, cin, H, W = shape
    a = torch.randn(B, k1, H, W, generator=g).to(cuda)
    bb = torch.randn(B, cin - k1 + 64, H, W, generator=g).to(cuda)[:, 32:32 + cin - k1]  # a slice: batch stride
    w = (torch.randn(cout, cin, generator=g) * (1.0 / cin ** 0.5)).to(cuda)
    b = (torch.randn(cout, generator=g) * 0.1).to(cuda)
    prep = _hip.conv1x1x2_prepare(w)
    y0 = _hip.conv1x1x2_silu(torch.cat([a, bb], 1), b, lambda: prep, cout)
    cv = _hip.CatView([a, bb])
    assert _hip.conv1x1x2_ok(cv, torch.nn.Conv2d(cin, cout, 1))
    y = _hip.conv1x1x2_silu(cv, b, lambda: prep, cout)
    assert torch.equal(y, y0)
    t = torch.empty((B, cout // 2, H, W), device=cuda)
    _hip.conv1x1x2_silu(cv, b, lambda: prep, cout, out2=t, c2lo=cout // 2)
    assert torch.equal(t, y0[:, cout // 2:])


@pytest.mark.parametrize("k1,cin", [(64, 128), (32, 96), (128, 256)])
def test_conv1x1_thin_virtual_concat_bit_identical(k1, cin, cuda):
    """The thin 1x1 kernel over a CatView (any split) = over the materialised concat, bit for bit."""
    g = torch.Generator().manual_seed(cin + k1)
    a = torch.randn(2, k1, 32, 32, generator=g).to(cuda)
    bb = torch.randn(2, cin - k1, 32, 32, generator=g).to(cuda)
    w = (torch.randn(64, cin, generator=g) * (1.0 / cin ** 0.5)).to(cuda)
    b = (torch.randn(64, generator=g) * 0.1).to(cuda)
    y0 = _hip.conv1x1_thin(torch.cat([a, bb], 1), w, b)
    cv = _hip.CatView([a, bb])
    assert _hip.conv1x1_thin_ok(cv, 64)
    assert torch.equal(_hip.conv1x1_thin(cv, w, b), y0)
    t = torch.empty((2, 32, 32, 32), device=cuda)
    _hip.conv1x1_thin(cv, w, b, out2=t, c2lo=32)
    assert torch.equal(t, y0[:, 32:])


def test_model_neck_concats_as_virtual_concats_bit_identical(cuda, monkeypatch):
    """The executor hands the neck Concats to their C2f as CatViews (tasks.CATVIEW): every neck Concat does (the skip
    inputs are never copied) and the model output is bit-identical to the concat-buffer form."""
    from yolosod_amd.nn import tasks as T
    m = T.build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=cuda)
    x = torch.rand(2, 3, 640, 640, generator=torch.Generator().manual_seed(8)).to(cuda)
    torch.backends.cudnn.deterministic = True
    try:
        with torch.inference_mode():
            monkeypatch.setattr(T, "CATVIEW", True)
            with _hip.op_timer() as t:
                y = m(x)[0]
            cats = sum(1 for k, _ in t.durations_ms() if k[0] in ("conv1x1x2", "conv1x1_thin") and "cat" in k[2])
            monkeypatch.setattr(T, "CATVIEW", False)
            y0 = m(x)[0]
    finally:
        torch.backends.cudnn.deterministic = False
    assert cats == 6, cats
    assert torch.equal(y, y0), float((y - y0).abs().max())


@pytest.mark.parametrize("shape", [(2, 128, 40, 40), (2, 96, 20, 24), (1, 256, 16, 16)])
def test_conv1x1x2_cout64_matches_fp64(shape, cuda):
    """The 64-channel-group form (the neck's Cout-64 1x1 convs) against fp64, and its dual store bit-identical."""
    g = torch.Generator().manual_seed(sum(shape))
    B, cin, H, W = shape
    x = torch.randn(shape, generator=g)
    w = torch.randn(64, cin, 1, 1, generator=g) * (1.0 / cin ** 0.5)
    b = torch.randn(64, generator=g) * 0.1
    ref = F.silu(F.conv2d(x.double(), w.double(), b.double()))
    wd = w.to(cuda)
    prep = _hip.conv1x1x2_prepare(wd)
    y = _hip.conv1x1x2_silu(x.to(cuda), b.to(cuda), lambda: prep, 64)
    miopen = F.silu(F.conv2d(x.to(cuda), wd, b.to(cuda))).cpu().double()
    err, err_m = float((y.cpu().double() - ref).abs().max()), float((miopen - ref).abs().max())
    assert err <= 8 * err_m + 1e-5, (err, err_m)
    t = torch.empty((B, 32, H, W), device=cuda)
    _hip.conv1x1x2_silu(x.to(cuda), b.to(cuda), lambda: prep, 64, out2=t, c2lo=32)
    assert torch.equal(t, y[:, 32:])
