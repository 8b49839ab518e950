"""ORACLE - TEST INFRASTRUCTURE ONLY (see oracle/ops_ref.py header for the rules).

numpy restatement of ``ultralytics.utils.ops.non_max_suppression`` (ops.py:167-316) around the C restatement of
``torchvision.ops.nms`` (oracle/nms_ref.c). Returns the reference's per-image rows plus the anchor index of each
kept row. Pinned by tests/golden/nms_*.npz, produced by running the *reference's* wrapper.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "libnms_ref.so"
_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def _load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        lib = ctypes.CDLL(str(LIB))
        lib.nms_ref.restype = ctypes.c_int64
        lib.nms_ref.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p]
        _lib = lib
    return _lib


def torchvision_nms(boxes: np.ndarray, scores: np.ndarray, iou_threshold: float) -> np.ndarray:
    """torchvision.ops.nms restated (CPU kernel semantics): int64 indices of kept boxes, descending score."""
    boxes = np.ascontiguousarray(boxes, dtype=np.float32)
    scores = np.ascontiguousarray(scores, dtype=np.float32)
    n = boxes.shape[0]
    keep = np.empty(max(n, 1), dtype=np.int64)
    k = _load().nms_ref(boxes.ctypes.data, scores.ctypes.data, n, float(iou_threshold), keep.ctypes.data)
    return keep[:k].copy()


def xywh2xyxy_np(x: np.ndarray) -> np.ndarray:
    """ops.py:416-434 in fp32."""
    y = np.empty_like(x)
    xy = x[..., :2]
    wh = x[..., 2:] / np.float32(2)
    y[..., :2] = xy - wh
    y[..., 2:] = xy + wh
    return y


def clip_boxes_ref(boxes: np.ndarray, shape) -> np.ndarray:
    """ops.py:319-338 (numpy branch, in place): x to [0, w], y to [0, h]."""
    boxes[..., [0, 2]] = boxes[..., [0, 2]].clip(0, shape[1])
    boxes[..., [1, 3]] = boxes[..., [1, 3]].clip(0, shape[0])
    return boxes


def scale_boxes_ref(img1_shape, boxes: np.ndarray, img0_shape, ratio_pad=None, padding=True, xywh=False):
    """ops.py:92-128 in fp32 (in place): undo letterbox gain / pad, then clip to img0_shape.
    Called per image by DetectionPredictor.postprocess (models/yolo/detect/predict.py:39) on pred[:, :4]."""
    if ratio_pad is None:
        gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
        pad = (round((img1_shape[1] - img0_shape[1] * gain) / 2 - 0.1),
               round((img1_shape[0] - img0_shape[0] * gain) / 2 - 0.1))
    else:
        gain = ratio_pad[0][0]
        pad = ratio_pad[1]
    if padding:
        boxes[..., 0] -= np.float32(pad[0])
        boxes[..., 1] -= np.float32(pad[1])
        if not xywh:
            boxes[..., 2] -= np.float32(pad[0])
            boxes[..., 3] -= np.float32(pad[1])
    boxes[..., :4] /= np.float32(gain)
    return clip_boxes_ref(boxes, img0_shape)


def non_max_suppression_ref(prediction: np.ndarray, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                            multi_label=False, max_det=300, nc=0, max_nms=30000, max_wh=7680, in_place=True):
    """Returns (rows: list of [n_i, 6] float32, anchors: list of [n_i] int64). Mutates ``prediction`` (B, 4+nc, A)
    to xyxy in place when ``in_place`` (ops.py:241-244)."""
    pred = prediction
    bs = pred.shape[0]
    nc = nc or (pred.shape[1] - 4)
    mi = 4 + nc
    conf32 = np.float32(conf_thres)
    xc = pred[:, 4:mi].max(1) > conf32
    multi_label = bool(multi_label) and nc > 1
    t = np.ascontiguousarray(np.swapaxes(pred, 1, 2))  # (B, A, 4+nc)
    t[..., :4] = xywh2xyxy_np(t[..., :4])
    if in_place:
        pred[:, :4, :] = np.swapaxes(t[..., :4], 1, 2)
    rows_out, idx_out = [], []
    for xi in range(bs):
        anchors = np.nonzero(xc[xi])[0]
        x = t[xi][anchors]
        if not x.shape[0]:
            rows_out.append(np.zeros((0, 6), np.float32))
            idx_out.append(np.zeros((0,), np.int64))
            continue
        box, cls = x[:, :4], x[:, 4:mi]
        if multi_label:
            i, j = np.nonzero(cls > conf32)  # row-major (anchor, class) order, as torch.where
            x = np.concatenate([box[i], cls[i, j][:, None], j[:, None].astype(np.float32)], 1)
            aidx = anchors[i]
        else:
            j = cls.argmax(1)  # first maximal index
            conf = cls[np.arange(cls.shape[0]), j]
            keepc = conf > conf32
            x = np.concatenate([box, conf[:, None], j[:, None].astype(np.float32)], 1)[keepc]
            aidx = anchors[keepc]
        if classes is not None:
            m = (x[:, 5:6] == np.asarray(classes, dtype=np.float32)[None]).any(1)
            x, aidx = x[m], aidx[m]
        n = x.shape[0]
        if not n:
            rows_out.append(np.zeros((0, 6), np.float32))
            idx_out.append(np.zeros((0,), np.int64))
            continue
        if n > max_nms:
            o = np.argsort(-x[:, 4], kind="stable")[:max_nms]
            x, aidx = x[o], aidx[o]
        c = x[:, 5:6] * np.float32(0 if agnostic else max_wh)
        boxes = (x[:, :4] + c).astype(np.float32)
        i = torchvision_nms(boxes, x[:, 4], iou_thres)[:max_det]
        rows_out.append(x[i].astype(np.float32))
        idx_out.append(aidx[i].astype(np.int64))
    return rows_out, idx_out
