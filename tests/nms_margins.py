"""Test helper: decision margins of the reference NMS on one image, for end-to-end kept-index parity.

Two forwards of the same model on the same input (the HIP path and the CPU oracle) differ by fp32 rounding, so
their Detect outputs ``y`` differ by a small perturbation. The reference's post-processing
(``ultralytics/utils/ops.py:167-316`` around ``torchvision.ops.nms``) turns ``y`` into kept anchor indices through
discrete decisions; each is a comparison whose two sides both move with the perturbation:

* the candidate filter ``max_c score > conf`` (ops.py:234, 275)                       -> margin |score - conf|
* the best class ``argmax_c`` (ops.py:274)                                            -> top-1 minus top-2 score
* the greedy suppression ``IoU(kept i, j) > iou_thres`` (torchvision CPU nms)         -> |max_i IoU(i, j) - thr|
* the processing order of two boxes that overlap past the threshold (sorted scores)   -> |s_i - s_j|
* the output order and the ``[:max_det]`` cut (ops.py:297)                            -> consecutive kept gaps

Rule used by the parity tests: an image is *decision-stable* when every one of these margins, measured on the
oracle's ``y``, exceeds twice the perturbation of its inputs actually measured between the two outputs (score
margins against 2 max|d score|; IoU margins, computed in fp32 on the class-offset boxes like the oracle, against
2 max|d IoU| over the same-class candidate pairs + 1e-6). On a decision-stable image no decision can flip, so
the kept anchor indices must be bit-identical, in order. Images that are not decision-stable are counted and
reported; their indices may legitimately differ at the flipping decision (test-side only, not product code).
"""
from __future__ import annotations

import numpy as np


def _xyxy(b):
    """ops.py:416-434 in fp32, as the oracle (xy -/+ wh / 2)."""
    b = b.astype(np.float32)
    xy, wh = b[:, :2], b[:, 2:] / np.float32(2)
    return np.concatenate([xy - wh, xy + wh], 1)


def _iou(b):
    """Pairwise IoU of xyxy boxes [n, 4] exactly as the oracle's torchvision restatement computes it: fp32 areas
    (no +1), fp32 clamped intersection, fp32 ratio (returned as float64 for the margins)."""
    b = b.astype(np.float32)
    area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    lt = np.maximum(b[:, None, :2], b[None, :, :2])
    rb = np.minimum(b[:, None, 2:], b[None, :, 2:])
    wh = np.maximum(rb - lt, np.float32(0))
    inter = wh[..., 0] * wh[..., 1]
    return (inter / ((area[:, None] + area[None, :]) - inter)).astype(np.float64)


def nms_stability(y_ref: np.ndarray, y_oth: np.ndarray, conf=0.25, iou_thres=0.7, max_det=300, max_nms=30000,
                  max_wh=7680):
    """Decision margins of predict-mode NMS (single label, class-aware) for one image.

    ``y_ref`` / ``y_oth``: [4 + nc, A] float32 Detect outputs (xywh boxes, class probabilities) of the oracle and of
    the other path. Returns a dict with each margin, the measured perturbations, the greedy keep list of the oracle
    (anchor indices, output order) and ``stable``."""
    s_r = np.ascontiguousarray(y_ref[4:].T)  # [A, nc]
    s_o = np.ascontiguousarray(y_oth[4:].T)
    d_s = float(np.abs(s_r.astype(np.float64) - s_o).max())
    best = s_r.max(1)
    m_conf = float(np.abs(best.astype(np.float64) - np.float32(conf)).min())
    cand = np.nonzero(best > np.float32(conf))[0]
    res = {"d_score": d_s, "m_conf": m_conf, "n_cand": int(cand.size)}
    if cand.size == 0:
        res.update(m_cls=np.inf, m_iou=np.inf, m_order=np.inf, m_out=np.inf, d_iou=0.0, keep=np.zeros(0, np.int64))
        res["stable"] = m_conf > 2 * d_s
        return res
    sc = s_r[cand]
    top2 = np.sort(sc, 1)[:, -2:] if sc.shape[1] > 1 else np.concatenate([np.full((len(cand), 1), -np.inf), sc], 1)
    m_cls = float((top2[:, 1].astype(np.float64) - top2[:, 0]).min())
    cls = sc.argmax(1)
    score = sc[np.arange(len(cand)), cls]
    if cand.size > max_nms:
        o = np.argsort(-score, kind="stable")
        cut = float(score[o[max_nms - 1]]) - float(score[o[max_nms]])
        o = o[:max_nms]
        cand, cls, score = cand[o], cls[o], score[o]
    else:
        cut = np.inf
    off = (cls.astype(np.float32) * np.float32(max_wh))[:, None]  # class offset (ops.py:289-295), in fp32
    b_r = (_xyxy(y_ref[:4, cand].T) + off).astype(np.float32)
    b_o = (_xyxy(y_oth[:4, cand].T) + off).astype(np.float32)
    order = np.argsort(-score, kind="stable")  # torchvision: descending score, stable
    # per class (the class offset max_wh keeps different classes apart), greedy with margins
    m_iou, m_order, d_iou = np.inf, np.inf, 0.0
    keep_mask = np.zeros(len(cand), bool)
    for c in np.unique(cls):
        sel = order[cls[order] == c]  # this class, in processing order
        ir, io = _iou(b_r[sel]), _iou(b_o[sel])
        n = len(sel)
        if n > 1:
            iu = np.triu_indices(n, 1)
            d_iou = max(d_iou, float(np.abs(ir[iu] - io[iu]).max()))
        kept = []
        for t in range(n):
            mx = float(ir[kept, t].max()) if kept else 0.0
            m_iou = min(m_iou, abs(mx - iou_thres))
            if not (mx > iou_thres):
                kept.append(t)
        keep_mask[sel[kept]] = True
        res.setdefault("_pairs", []).append((sel, ir, io))
    d_iou_tol = 2 * d_iou + 1e-6
    for sel, ir, io in res.pop("_pairs"):
        n = len(sel)
        if n > 1:
            close = np.maximum(ir, io) > iou_thres - d_iou_tol
            np.fill_diagonal(close, False)
            if close.any():
                a, b = np.nonzero(close)
                m_order = min(m_order, float(np.abs(score[sel[a]].astype(np.float64) - score[sel[b]]).min()))
    kept_idx = order[keep_mask[order]]  # output order: descending score over all classes
    ks = score[kept_idx].astype(np.float64)
    m_out = float((ks[:-1] - ks[1:]).min()) if len(ks) > 1 else np.inf
    if len(ks) > max_det:
        m_out = min(m_out, float(ks[max_det - 1] - ks[max_det]))
    m_out = min(m_out, cut)
    res.update(m_cls=m_cls, m_iou=m_iou, m_order=m_order, m_out=m_out, d_iou=d_iou,
               keep=cand[kept_idx[:max_det]].astype(np.int64))
    res["stable"] = bool(m_conf > 2 * d_s and m_cls > 2 * d_s and m_order > 2 * d_s and m_out > 2 * d_s
                         and m_iou > d_iou_tol)
    return res


def first_divergence(y_ref: np.ndarray, y_oth: np.ndarray, conf=0.25, iou_thres=0.7, max_nms=30000, max_wh=7680):
    """The first decision at which predict-mode NMS on ``y_oth`` departs from NMS on ``y_ref`` (single label,
    class-aware; ``ultralytics/utils/ops.py:274-297`` around torchvision's greedy NMS), or None when every decision
    agrees - the kept anchor lists are then identical.

    Both outputs are replayed side by side, stage by stage, in the order the reference takes its decisions: the
    candidate filter (ops.py:234, 275), the best class (:274), the descending-score processing order and the
    ``max_nms`` cut (:284-286), then the greedy IoU tests box by box (torchvision CPU nms). Everything before the
    returned decision is identical in both runs, so it is the cause of the first difference in the kept lists. The
    result holds the decision's margin measured on ``y_ref`` and the tolerance it is held to: twice the measured
    perturbation of that decision's inputs (score decisions: 2 max|d score| over the image; IoU tests: 2 max|d IoU|
    over the same-class candidate pairs + 1e-6)."""
    s_r = np.ascontiguousarray(y_ref[4:].T)
    s_o = np.ascontiguousarray(y_oth[4:].T)
    tol_s = 2 * float(np.abs(s_r.astype(np.float64) - s_o).max())
    best_r, best_o = s_r.max(1), s_o.max(1)
    c_r, c_o = best_r > np.float32(conf), best_o > np.float32(conf)
    if (c_r != c_o).any():
        x = np.nonzero(c_r != c_o)[0]
        margin = float(np.abs(best_r[x].astype(np.float64) - np.float32(conf)).max())
        return {"kind": "conf", "anchors": x.tolist(), "margin": margin, "tol": tol_s}
    cand = np.nonzero(c_r)[0]
    if cand.size == 0:
        return None
    cls_r, cls_o = s_r[cand].argmax(1), s_o[cand].argmax(1)
    if (cls_r != cls_o).any():
        x = np.nonzero(cls_r != cls_o)[0]
        top2 = np.sort(s_r[cand[x]], 1)[:, -2:].astype(np.float64)
        return {"kind": "class", "anchors": cand[x].tolist(), "margin": float((top2[:, 1] - top2[:, 0]).max()),
                "tol": tol_s}
    sc_r = s_r[cand, cls_r]
    sc_o = s_o[cand, cls_o]
    ord_r = np.argsort(-sc_r, kind="stable")
    ord_o = np.argsort(-sc_o, kind="stable")
    n_proc = min(cand.size, max_nms)
    if not np.array_equal(ord_r[:n_proc], ord_o[:n_proc]):
        j = int(np.nonzero(ord_r[:n_proc] != ord_o[:n_proc])[0][0])
        a, b = ord_r[j], ord_o[j]
        return {"kind": "order", "position": j, "anchors": [int(cand[a]), int(cand[b])],
                "margin": abs(float(sc_r[a]) - float(sc_r[b])), "tol": tol_s}
    order = ord_r[:n_proc]
    off = (cls_r.astype(np.float32) * np.float32(max_wh))[:, None]
    b_r = (_xyxy(y_ref[:4, cand].T) + off).astype(np.float32)
    b_o = (_xyxy(y_oth[:4, cand].T) + off).astype(np.float32)
    # per class (the offsets keep classes apart): pairwise IoU of both runs and the IoU perturbation
    ious, d_iou = {}, 0.0
    for c in np.unique(cls_r[order]):
        sel = order[cls_r[order] == c]
        ir, io = _iou(b_r[sel]), _iou(b_o[sel])
        if len(sel) > 1:
            iu = np.triu_indices(len(sel), 1)
            d_iou = max(d_iou, float(np.abs(ir[iu] - io[iu]).max()))
        ious[int(c)] = (sel, ir, io, [])
    tol_iou = 2 * d_iou + 1e-6
    pos = {int(t): i for c in ious for i, t in enumerate(ious[c][0])}
    for t in order:  # global processing order = per-class order interleaved by score
        sel, ir, io, kept = ious[int(cls_r[t])]
        i = pos[int(t)]
        mx_r = float(ir[kept, i].max()) if kept else 0.0
        mx_o = float(io[kept, i].max()) if kept else 0.0
        if (mx_r > iou_thres) != (mx_o > iou_thres):
            return {"kind": "iou", "anchors": [int(cand[t])], "margin": abs(mx_r - iou_thres), "tol": tol_iou}
        if not (mx_r > iou_thres):
            kept.append(i)
    return None
