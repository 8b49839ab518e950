"""Test helper: a "trained-like" paper model and structured synthetic scenes for end-to-end parity.

Why: at seed-0 random init the backbone's per-layer gain is ~0.6, so at the Detect head the input signal is gone -
neighbouring anchors carry near-identical (often bit-identical) scores, nothing passes conf 0.25, and the kept
indices after NMS are decided by ties that any fp32 re-association can flip. A trained network keeps its
activations near unit variance. This model gets that property the way training would:

1. seed-0 paper model (reference RNG order, ``tests/golden/model_manifest.json``);
2. BatchNorm recalibration - one train-mode forward of a calibration batch with ``momentum = 1`` sets every
   Conv's BN running statistics to the batch statistics of its input (unit-variance, zero-mean activations);
3. the class branch's last 1x1 conv (``Detect.cv3[i][2]``) scaled by 0.4 with its bias + 2 (logits in a moderate
   range: no score saturates at exactly 1.0 in fp32, ~1 % of anchors pass conf 0.25).

The result is saved in the reference trainer's checkpoint layout (``nn/checkpoint.save_checkpoint``), so both the
GPU path and the CPU oracle load it through ``attempt_load_one_weight`` (``nn/tasks.py:941-975``).
"""
from __future__ import annotations

import torch

CFG = "yolov12-sod-fusion-v5-simple.yaml"


def scene(gen: torch.Generator, size: int, n_rect: int | None = None) -> torch.Tensor:
    """[3, size, size] in [0, 1]: a flat background with ``n_rect`` random flat-coloured rectangles (edges give
    the network something to respond to; uniform noise averages out)."""
    n_rect = n_rect or max(8, size * 3 // 16)
    x = torch.rand(3, 1, 1, generator=gen).expand(3, size, size).clone()
    for _ in range(n_rect):
        w, h = torch.randint(4, max(5, size // 3), (2,), generator=gen).tolist()
        x0, y0 = torch.randint(0, size - 4, (2,), generator=gen).tolist()
        x[:, y0:y0 + h, x0:x0 + w] = torch.rand(3, 1, 1, generator=gen)
    return x


def scenes(seed: int, n: int, size: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.stack([scene(g, size) for _ in range(n)])


def noisy_scenes(seed: int, n: int, size: int, sigma: float = 0.06) -> torch.Tensor:
    """The rectangle scenes with per-pixel Gaussian noise on top (clamped to [0, 1]): no flat region is left, so no
    two neighbouring anchors see identical receptive fields and their scores are never exactly tied in fp32 (the flat
    scenes produce such ties, which any re-association can flip)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.stack([scene(g, size) for _ in range(n)])
    return (x + sigma * torch.randn(x.shape, generator=g)).clamp_(0.0, 1.0)


def make_trained_like_checkpoint(path, cal_size: int = 320, cls_scale: float = 0.4, cls_shift: float = 2.0):
    from oracle.model_ref import REGISTRY
    from yolosod_amd.nn.checkpoint import save_checkpoint
    from yolosod_amd.nn.tasks import DetectionModel

    torch.manual_seed(0)
    m = DetectionModel(CFG, registry=REGISTRY)  # oracle operator classes: the calibration forward runs on the CPU
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.momentum = 1.0
    m.train()
    with torch.no_grad():
        m(scenes(12345, 2, cal_size))
    m.eval()
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.momentum = 0.03  # initialize_weights' value (utils/torch_utils.py:410-420)
    det = m.model[-1]
    with torch.no_grad():
        for i in range(det.nl):
            c = det.cv3[i][2]
            c.weight.mul_(cls_scale)
            c.bias.add_(cls_shift)
    torch.manual_seed(0)
    p = DetectionModel(CFG)  # the product classes (their reference class paths go into the checkpoint)
    p.load_state_dict(m.state_dict())
    return save_checkpoint(p, path)
