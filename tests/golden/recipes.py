"""Deterministic recipes shared by ``make_golden.py`` (which runs the *reference* modules) and the tests (which run
this build's modules): module configurations, seeded parameter perturbation and seeded inputs.

Default random init gives near-constant attention outputs, so every per-op fixture uses
perturbed parameters and unit-scale inputs. Parameters are regenerated from the recipe (torch's CPU generator is
platform independent); the fixture stores their sha256 so any drift is caught, plus the inputs and the reference
outputs.
"""
from __future__ import annotations

import hashlib

import numpy as np
import torch

# name -> (op, constructor args as the reference's parse_model would inject them, input shape)
OPS = {
    "se_c32_r64": ("SE_Block", (64,), (2, 32, 24, 24)),
    "se_c128_r256": ("SE_Block", (256,), (2, 128, 12, 12)),
    "se_c64_r4_odd": ("SE_Block", (4,), (2, 64, 9, 7)),
    "cbam_c64": ("CBAM_Block", (64, 128, 16), (2, 64, 24, 24)),
    "cbam_c256": ("CBAM_Block", (256, 512, 16), (2, 256, 12, 12)),
    "cbam_c32_odd": ("CBAM_Block", (32, None, 8), (2, 32, 13, 11)),
    "ca_c128": ("CA_Block", (128, 256, 32), (2, 128, 16, 12)),
    "ca_c64_odd": ("CA_Block", (64, None, 4), (2, 64, 9, 7)),
    "a2_c64_h20": ("A2_Attn", (64, None, 8, 8), (2, 64, 20, 20)),
    "a2_c128_h16": ("A2_Attn", (128, None, 8, 2), (2, 128, 16, 12)),
    "a2_c64_h4": ("A2_Attn", (64, None, 8, 4), (1, 64, 4, 8)),
    "a2_c512_h20": ("A2_Attn", (512, None, 8, 8), (1, 512, 20, 20)),
    "swin_c64_h20": ("SwinBlock", (64, 2, 7), (2, 64, 20, 20)),
    "swin_c64_h14": ("SwinBlock", (64, 2, 7), (1, 64, 14, 14)),
    "swin_c64_h6": ("SwinBlock", (64, 2, 7), (2, 64, 6, 6)),
    "swin_c64_h16x12": ("SwinBlock", (64, 2, 7), (1, 64, 16, 12)),
    "swin_c64_h20x5": ("SwinBlock", (64, 2, 7), (1, 64, 20, 5)),
    "swin_c256_h9": ("SwinBlock", (256, 4, 7), (1, 256, 9, 9)),
    # MambaBlock(c, c_hidden, seq_reduction) (GLU fallback): fusion-v5 L7 is (128, 256, 2) at P3
    "mamba_c128_h16": ("MambaBlock", (128, 256, 2), (1, 128, 16, 16)),
    "mamba_c64_h15x13": ("MambaBlock", (64, 64, 2), (2, 64, 15, 13)),
    "mamba_c32_r1": ("MambaBlock", (32, 64, 1), (2, 32, 10, 12)),
    "mamba_c64_r3": ("MambaBlock", (64, 32, 3), (1, 64, 14, 17)),
}


def seed_of(name: str) -> int:
    return int(hashlib.sha256(name.encode()).hexdigest()[:8], 16)


def perturb_(module: torch.nn.Module, seed: int) -> None:
    """Overwrite every float parameter/buffer in state_dict order from a seeded generator."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for k, v in module.state_dict().items():
            if not v.is_floating_point():
                continue
            if k.endswith("running_var"):
                v.copy_(torch.rand(v.shape, generator=g) * 0.5 + 0.5)
            elif k.endswith("running_mean"):
                v.copy_(torch.randn(v.shape, generator=g) * 0.2)
            elif v.dim() >= 2:
                fan_in = v[0].numel()
                v.copy_(torch.randn(v.shape, generator=g) * (1.5 / fan_in ** 0.5))
            elif k.endswith("weight"):  # norm scales
                v.copy_(1.0 + torch.randn(v.shape, generator=g) * 0.2)
            else:
                v.copy_(torch.randn(v.shape, generator=g) * 0.2)


def make_input(name: str, shape) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed_of(name) + 1)
    return torch.randn(shape, generator=g)


def params_sha256(module: torch.nn.Module) -> str:
    h = hashlib.sha256()
    for k, v in module.state_dict().items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


# ---- decode / NMS synthetic inputs ----
DECODE = {"name": "decode_128", "B": 2, "nc": 10, "shapes": [(32, 32), (16, 16), (8, 8), (4, 4)],
          "strides": [4.0, 8.0, 16.0, 32.0]}


def decode_maps(spec=DECODE):
    g = torch.Generator().manual_seed(seed_of(spec["name"]))
    maps = []
    for h, w in spec["shapes"]:
        box = torch.randn(spec["B"], 64, h, w, generator=g) * 2.0
        cls = torch.randn(spec["B"], spec["nc"], h, w, generator=g) * 3.0 - 2.0
        maps.append(torch.cat([box, cls], 1))
    return maps


def synthetic_predictions(seed: int, B: int, A: int, nc: int, n_clusters: int = 40, img: float = 640.0,
                          tie_scores: bool = False, degenerate: bool = False) -> np.ndarray:
    """(B, 4+nc, A) xywh + class scores: clustered, heavily overlapping boxes, a few classes per cluster, scores
    spread over [0, 1) with no exact ties (unless tie_scores). ``degenerate``: also zero-area boxes (w = 0 or h = 0:
    two of them give IoU 0 / 0 = NaN, which torchvision's ``ovr > thr`` treats as no suppression) and exact duplicates
    of other anchors' boxes and class scores with the main score lowered (identical boxes: IoU exactly 1; identical
    zero-area boxes: NaN), the scores kept distinct so that every kept row names one anchor."""
    rng = np.random.default_rng(seed)
    out = np.zeros((B, 4 + nc, A), np.float32)
    for b in range(B):
        cx = rng.uniform(0, img, n_clusters)
        cy = rng.uniform(0, img, n_clusters)
        cw = rng.uniform(8, 120, n_clusters)
        ch = rng.uniform(8, 120, n_clusters)
        k = rng.integers(0, n_clusters, A)
        jit = rng.normal(0, 0.08, (4, A))
        out[b, 0] = cx[k] + jit[0] * cw[k]
        out[b, 1] = cy[k] + jit[1] * ch[k]
        out[b, 2] = cw[k] * np.exp(jit[2])
        out[b, 3] = ch[k] * np.exp(jit[3])
        s = rng.uniform(0, 1, (nc, A)) ** 3
        main = rng.integers(0, nc, n_clusters)[k]
        s[main, np.arange(A)] = rng.uniform(0.05, 1.0, A)
        if tie_scores:
            s = np.round(s * 16) / 16
        out[b, 4:] = s
        if degenerate:
            n_dup = A // 10
            src, dst = rng.choice(A, n_dup, replace=False), rng.choice(A, n_dup, replace=False)
            ok = src != dst
            src, dst = src[ok], dst[ok]
            out[b, :, dst] = out[b, :, src]
            out[b, 4:, dst] *= np.float32(0.97)  # same box and best class, lower (distinct) scores
            zw = rng.choice(A, A // 7, replace=False)
            out[b, 2, zw] = 0.0
            zh = rng.choice(A, A // 10, replace=False)
            out[b, 3, zh] = 0.0
            both = dst[: len(dst) // 3]  # some duplicate pairs become identical zero-area boxes
            out[b, 2, both] = 0.0
            out[b, 2, src[: len(dst) // 3]] = 0.0
    return out


def nms_case(name):
    """(prediction, non_max_suppression kwargs) of NMS fixture ``name``."""
    seed, B, A, nc, kw = NMS_CASES[name]
    kw = dict(kw)
    tie, deg = kw.pop("tie", False), kw.pop("degenerate", False)
    return synthetic_predictions(seed, B, A, nc, tie_scores=tie, degenerate=deg), kw


NMS_CASES = {
    # name: (pred seed, B, A, nc, kwargs)
    "nms_predict": (11, 3, 3000, 10, dict(conf_thres=0.25, iou_thres=0.7)),
    "nms_val": (11, 3, 3000, 10, dict(conf_thres=0.001, iou_thres=0.7, multi_label=True)),
    "nms_agnostic": (12, 2, 2000, 10, dict(conf_thres=0.25, iou_thres=0.5, agnostic=True)),
    "nms_classes": (13, 2, 2000, 10, dict(conf_thres=0.2, iou_thres=0.6, classes=[1, 3, 7])),
    "nms_cuts": (14, 2, 4000, 10, dict(conf_thres=0.1, iou_thres=0.45, max_nms=500, max_det=50)),
    "nms_empty": (15, 2, 500, 10, dict(conf_thres=0.999999, iou_thres=0.7)),
    "nms_ties": (16, 2, 1500, 10, dict(conf_thres=0.25, iou_thres=0.7, tie=True)),
    "nms_iou0": (17, 1, 800, 4, dict(conf_thres=0.3, iou_thres=0.0)),
    "nms_degenerate": (18, 2, 2000, 10, dict(conf_thres=0.25, iou_thres=0.7, degenerate=True)),
}


def synthetic_eval_set(seed: int, n_img: int = 24, nc: int = 6, img: float = 640.0):
    """Synthetic ground truth + detections for the mAP harness: per image 0-14 labelled xyxy boxes; each label is
    detected with prob 0.85 (jittered box, IoU spread over ~0.3-0.99, wrong class 10 %), plus 0-6 false positives,
    confidences in (0.001, 1). Image 0 has labels but no detections, image 1 detections but no labels, image 2
    neither. Returns (gt: list of (cls [m], boxes [m, 4]) float32, preds: list of [n, 6] float32)."""
    rng = np.random.default_rng(seed)
    gt, preds = [], []
    for i in range(n_img):
        m = 0 if i in (1, 2) else int(rng.integers(1, 15))
        c = rng.integers(0, nc, m).astype(np.float32)
        xy = rng.uniform(0, img - 40, (m, 2))
        wh = rng.uniform(8, 160, (m, 2))
        boxes = np.concatenate([xy, np.minimum(xy + wh, img)], 1).astype(np.float32)
        rows = []
        if i not in (0, 2):
            for j in range(m):
                if rng.uniform() < 0.85:
                    w, h = boxes[j, 2] - boxes[j, 0], boxes[j, 3] - boxes[j, 1]
                    s = rng.uniform(0.0, 0.25)
                    jit = rng.normal(0, s, 4) * np.array([w, h, w, h])
                    b = boxes[j] + jit
                    b = np.array([min(b[0], b[2] - 1), min(b[1], b[3] - 1), max(b[2], b[0] + 1), max(b[3], b[1] + 1)])
                    cls = c[j] if rng.uniform() > 0.1 else float(rng.integers(0, nc))
                    rows.append([*b, rng.uniform(0.001, 1.0), cls])
            for _ in range(int(rng.integers(0, 7))):
                xy0 = rng.uniform(0, img - 40, 2)
                wh0 = rng.uniform(8, 160, 2)
                rows.append([*xy0, *(xy0 + wh0), rng.uniform(0.001, 1.0), float(rng.integers(0, nc))])
        gt.append((c, boxes))
        preds.append(np.array(rows, np.float32).reshape(-1, 6))
    return gt, preds
