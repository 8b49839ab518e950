"""GPU: the stride-2 3x3 conv with the producing gate applied at staging (csrc/conv3x3s2.hip) against the exact
(fp64) conv + bias + SiLU of the gated input formed in fp32 as the reference does (SE: x * a, smallobj_modules.py:92;
CBAM: (x * ca) * sa, cbam_block.py:53-54; then Conv, conv.py:37-55), next to the MIOpen fp32 path's own error: Cout 64
and 128, one and several input chunks, ragged tiles and odd input sizes, every gate combination, the range guard."""
import pytest
import torch
import torch.nn.functional as F

from oplib import tol_close
from yolosod_amd import _hip

pytestmark = pytest.mark.gpu


def _gated(x, gc, gp):
    y = x
    if gc is not None:
        y = y * gc[:, :, None, None]
    if gp is not None:
        y = y * gp[:, None]
    return y


@pytest.mark.parametrize("gates", ["none", "c", "p", "cp"])
@pytest.mark.parametrize("shape,cout", [((2, 32, 40, 40), 64), ((2, 64, 24, 56), 128), ((1, 32, 17, 39), 64),
                                        ((2, 96, 16, 64), 128), ((1, 32, 320, 320), 64), ((1, 64, 160, 160), 128)])
def test_conv3x3s2_matches_fp64(shape, cout, gates, cuda):
    g = torch.Generator().manual_seed(sum(shape) + cout + len(gates))
    B, cin, H, W = shape
    x = torch.randn(shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * (1.0 / (3 * cin ** 0.5))
    b = torch.randn(cout, generator=g) * 0.1
    gc = torch.sigmoid(torch.randn(B, cin, generator=g)) if "c" in gates else None
    gp = torch.sigmoid(torch.randn(B, H, W, generator=g)) if "p" in gates else None
    xg = _gated(x, gc, gp)  # fp32 products, as the reference's gate output
    ref = F.silu(F.conv2d(xg.double(), w.double(), b.double(), stride=2, padding=1))
    wd = w.to(cuda)
    d = lambda t: None if t is None else t.to(cuda)  # noqa: E731
    y = _hip.conv3x3s2_silu(x.to(cuda), b.to(cuda), lambda: _hip.conv3x3s2_prepare(wd), cout, d(gc), d(gp))
    y = y.cpu().double()
    miopen = F.silu(F.conv2d(xg.to(cuda), wd, b.to(cuda), stride=2, padding=1)).cpu().double()
    assert y.shape == ref.shape
    err, err_m = float((y - ref).abs().max()), float((miopen - ref).abs().max())
    ok, e, _ = tol_close(y, ref, 5e-5, 1e-4)
    assert ok, f"{shape}: max abs err {e:.3g} (MIOpen fp32 {err_m:.3g})"
    assert err <= 8 * err_m + 1e-5, (err, err_m)


def test_conv3x3s2_gated_input_is_the_reference_product(cuda):
    """The staged values are exactly the reference's fp32 gate products: feeding the materialised (x * ca) * sa with
    no gates gives bit-identical outputs to feeding x with the gates."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 64, 32, 40, generator=g).to(cuda)
    ca = torch.sigmoid(torch.randn(2, 64, generator=g)).to(cuda)
    sa = torch.sigmoid(torch.randn(2, 32, 40, generator=g)).to(cuda)
    w = (torch.randn(128, 64, 3, 3, generator=g) * 0.05).to(cuda)
    b = torch.zeros(128, device=cuda)
    prep = _hip.conv3x3s2_prepare(w)
    y1 = _hip.conv3x3s2_silu(x, b, lambda: prep, 128, ca, sa)
    y0 = _hip.conv3x3s2_silu((x * ca[:, :, None, None]) * sa[:, None], b, lambda: prep, 128)
    assert torch.equal(y1, y0)


def test_conv3x3s2_range_guard(cuda):
    x = torch.randn(1, 32, 16, 16, device=cuda)
    w = torch.randn(64, 32, 3, 3, device=cuda) * 0.05
    b = torch.zeros(64, device=cuda)
    prep = _hip.conv3x3s2_prepare(w)
    _hip.split_range_flag(reset=True)
    _hip.conv3x3s2_silu(x, b, lambda: prep, 64)
    assert not _hip.split_range_flag(reset=True)
    _hip.conv3x3s2_silu(x, b, lambda: prep, 64, torch.full((1, 32), 1e5, device=cuda))  # gated values beyond fp16
    assert _hip.split_range_flag(reset=True)
    big = _hip.conv3x3s2_prepare(w * 2e4)
    _hip.split_range_flag(reset=True)
    for _ in range(2):
        _hip.conv3x3s2_silu(x, b, lambda: big, 64)
        assert _hip.split_range_flag(reset=True)


@pytest.mark.parametrize("shape,cout", [((2, 64, 40, 40), 256), ((2, 128, 24, 24), 512), ((1, 256, 40, 40), 384)])
def test_conv3x3s2_channel_groups_match_fp64(shape, cout, cuda):
    """Cout a multiple of 128 above 128 (the PAN neck's stride-2 convs): work items (tile, 128-channel group)."""
    g = torch.Generator().manual_seed(sum(shape) + cout)
    B, cin, H, W = shape
    x = torch.randn(shape, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * (1.0 / (3 * cin ** 0.5))
    b = torch.randn(cout, generator=g) * 0.1
    ref = F.silu(F.conv2d(x.double(), w.double(), b.double(), stride=2, padding=1))
    wd = w.to(cuda)
    y = _hip.conv3x3s2_silu(x.to(cuda), b.to(cuda), lambda: _hip.conv3x3s2_prepare(wd), cout).cpu().double()
    miopen = F.silu(F.conv2d(x.to(cuda), wd, b.to(cuda), stride=2, padding=1)).cpu().double()
    err, err_m = float((y - ref).abs().max()), float((miopen - ref).abs().max())
    ok, e, _ = tol_close(y, ref, 5e-5, 1e-4)
    assert ok, f"{shape}: max abs err {e:.3g} (MIOpen fp32 {err_m:.3g})"
    assert err <= 8 * err_m + 1e-5, (err, err_m)


@pytest.mark.parametrize("cin,cout", [(32, 64), (64, 128), (64, 256)])
def test_conv3x3s2_into_concat_slice(cin, cout, cuda):
    """out= a channel slice of a concat buffer (batch stride > Cout*Ho*Wo): bit-identical to the contiguous output, and
    the rest of the buffer untouched."""
    g = torch.Generator().manual_seed(cin + cout)
    x = torch.randn(3, cin, 24, 40, generator=g).to(cuda)
    w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(cuda)
    b = (torch.randn(cout, generator=g) * 0.1).to(cuda)
    prep = _hip.conv3x3s2_prepare(w)
    y = _hip.conv3x3s2_silu(x, b, lambda: prep, cout)
    buf = torch.full((3, cout + 96, 12, 20), float("nan"), device=cuda)
    _hip.conv3x3s2_silu(x, b, lambda: prep, cout, out=buf[:, 32:32 + cout])
    assert torch.equal(buf[:, 32:32 + cout], y)
    assert torch.isnan(buf[:, :32]).all() and torch.isnan(buf[:, 32 + cout:]).all()
