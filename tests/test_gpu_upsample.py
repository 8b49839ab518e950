"""Neck glue: the nearest 2x upsample written straight into a Concat slice (yolosod_upsample2x,
nn/tasks._predict_once_planned) against torch's nearest interpolation of the same tensor - a pure copy, so bit-exact.
Reference semantics: nn.Upsample(None, 2, 'nearest') + Concat rows of the neck YAML (ultralytics/nn/tasks.py parse)."""
import pytest
import torch
import torch.nn.functional as F

from yolosod_amd import _hip

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,ctot,off", [((2, 3, 20, 20), 7, 2), ((1, 5, 8, 12), 5, 0), ((3, 16, 40, 40), 48, 32)])
def test_upsample2x_into_concat_slice(dtype, shape, ctot, off):
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    B, C, h, w = shape
    x = torch.randn(shape, generator=g).to(dev, dtype)
    buf = torch.full((B, ctot, 2 * h, 2 * w), 7.0, device=dev, dtype=dtype)
    out = buf[:, off:off + C]
    assert _hip.upsample2x_into(x, out)
    torch.cuda.synchronize()
    ref = F.interpolate(x.float(), scale_factor=2, mode="nearest").to(dtype)
    assert torch.equal(out, ref)
    # the rest of the buffer is untouched
    mask = torch.ones(ctot, dtype=torch.bool)
    mask[off:off + C] = False
    assert torch.all(buf[:, mask] == 7.0)


def test_upsample2x_unsupported_shape_launches_nothing():
    dev = torch.device("cuda")
    x = torch.randn(2, 3, 5, 6, device=dev)  # w % 4 != 0: the caller keeps its strided copy
    out = torch.zeros(2, 3, 10, 12, device=dev)
    assert not _hip.upsample2x_into(x, out)
    assert torch.all(out == 0)
