"""Detection post-processing API (``ultralytics/utils/ops.py`` surface for this path).

:func:`non_max_suppression` keeps the reference signature and semantics (``ops.py:167-316``) including the
in-place xywh->xyxy rewrite of the caller's tensor, the best-class / multi-label candidate rules, the class offset
``cls * max_wh``, the ``max_nms`` pre-cut and ``[:max_det]``; the per-image greedy NMS is ``torchvision.ops.nms``
semantics (stable descending sort, strict ``IoU > iou_thres``) - all of it in one batched HIP launch pair with no
per-image Python loop. Differences: the wall-clock ``time_limit`` break (``ops.py:312-314``) is not reproduced
(every image is processed); masks (nm > 0), ``labels`` and ``rotated`` are not supported and raise.
"""
from __future__ import annotations

import torch

from .. import _hip


def xywh2xyxy(x: torch.Tensor) -> torch.Tensor:
    """ops.py:416-434."""
    assert x.shape[-1] == 4
    y = torch.empty_like(x)
    xy = x[..., :2]
    wh = x[..., 2:] / 2
    y[..., :2] = xy - wh
    y[..., 2:] = xy + wh
    return y


_CLIP_BOUNDS = {}


def clip_boxes(boxes: torch.Tensor, shape):
    """ops.py:319-338 (tensor branch). On the GPU the four per-column clamps (eight kernels) run as one clamp
    against cached [0,0,0,0] / [w,h,w,h] bound tensors: min(max(v, 0), bound) per element, the same values."""
    if boxes.device.type == "cuda" and boxes.dtype == torch.float32 and boxes.shape[-1] == 4:
        key = (boxes.device, float(shape[0]), float(shape[1]))
        lim = _CLIP_BOUNDS.get(key)
        if lim is None:
            lim = _CLIP_BOUNDS[key] = (torch.zeros(4, device=boxes.device),
                                       torch.tensor([shape[1], shape[0], shape[1], shape[0]], dtype=torch.float32,
                                                    device=boxes.device))
        return boxes.clamp_(min=lim[0], max=lim[1])
    boxes[..., 0] = boxes[..., 0].clamp(0, shape[1])
    boxes[..., 1] = boxes[..., 1].clamp(0, shape[0])
    boxes[..., 2] = boxes[..., 2].clamp(0, shape[1])
    boxes[..., 3] = boxes[..., 3].clamp(0, shape[0])
    return boxes


def scale_boxes(img1_shape, boxes, img0_shape, ratio_pad=None, padding=True, xywh=False):
    """ops.py:92-128."""
    if ratio_pad is None:
        gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
        pad = (round((img1_shape[1] - img0_shape[1] * gain) / 2 - 0.1),
               round((img1_shape[0] - img0_shape[0] * gain) / 2 - 0.1))
    else:
        gain = ratio_pad[0][0]
        pad = ratio_pad[1]
    if padding:
        boxes[..., 0] -= pad[0]
        boxes[..., 1] -= pad[1]
        if not xywh:
            boxes[..., 2] -= pad[0]
            boxes[..., 3] -= pad[1]
    if boxes.device.type == "cuda":
        # a Python-scalar divisor would run as a multiply by its reciprocal on the GPU (not bit-equal to the
        # reference's CPU division): divide by a device tensor instead
        boxes[..., :4] /= torch.full((), gain, dtype=boxes.dtype, device=boxes.device)
    else:
        boxes[..., :4] /= gain
    return clip_boxes(boxes, img0_shape)


def _validate(prediction, conf_thres, iou_thres, labels, rotated, nc):
    assert 0 <= conf_thres <= 1, f"Invalid Confidence threshold {conf_thres}, valid values are between 0.0 and 1.0"
    assert 0 <= iou_thres <= 1, f"Invalid IoU {iou_thres}, valid values are between 0.0 and 1.0"
    if isinstance(prediction, (list, tuple)):
        prediction = prediction[0]
    if rotated:
        raise NotImplementedError("rotated (OBB) NMS is not on this path")
    if labels is not None and len(labels):
        raise NotImplementedError("apriori labels (autolabelling) are not supported")
    if prediction.dim() != 3:
        raise ValueError(f"prediction must be [B, 4+nc, A], got {tuple(prediction.shape)}")
    nc = nc or (prediction.shape[1] - 4)
    if prediction.shape[1] - nc - 4:
        raise NotImplementedError("mask coefficients (nm > 0) are not supported")
    return prediction, nc


def non_max_suppression_padded(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                               multi_label=False, labels=(), max_det=300, nc=0, max_time_img=0.05, max_nms=30000,
                               max_wh=7680, in_place=True, rotated=False):
    """Same semantics as :func:`non_max_suppression`, returning fixed-shape device tensors and never syncing:
    ``(out [B, max_det, 6], counts [B] int32, index [B, max_det] int32 anchor ids, -1 padded)``."""
    prediction, nc = _validate(prediction, conf_thres, iou_thres, labels, rotated, nc)
    if prediction.shape[-1] == 6:
        raise NotImplementedError("end-to-end (B, N, 6) predictions are not on this path")
    multi_label = bool(multi_label) and nc > 1
    return _hip.nms(prediction, conf_thres, iou_thres, classes, agnostic, multi_label, max_det, max_nms, max_wh,
                    in_place)


def non_max_suppression(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                        multi_label=False, labels=(), max_det=300, nc=0, max_time_img=0.05, max_nms=30000,
                        max_wh=7680, in_place=True, rotated=False):
    """Reference-compatible NMS (ops.py:167-316): list of [n_i, 6] tensors (x1, y1, x2, y2, conf, cls)."""
    out, counts, _ = non_max_suppression_padded(prediction, conf_thres, iou_thres, classes, agnostic, multi_label,
                                                labels, max_det, nc, max_time_img, max_nms, max_wh, in_place,
                                                rotated)
    n = counts.cpu().tolist()  # the one host sync (the reference's output sizes are data dependent too)
    return [out[i, : n[i]] for i in range(len(n))]
