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
    (no +1), fp32 clamped intersection, fp32 ratio (returned as float64 for the margins). Two zero-area boxes give
    0 / 0 = NaN, as in torchvision (its ``ovr > thr`` is then false: a NaN IoU never suppresses)."""
    b = b.astype(np.float32)
    area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    lt = np.maximum(b[:, None, :2], b[None, :, :2])
    rb = np.minimum(b[:, None, 2:], b[None, :, 2:])
    wh = np.maximum(rb - lt, np.float32(0))
    inter = wh[..., 0] * wh[..., 1]
    with np.errstate(invalid="ignore", divide="ignore"):
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
        res.update(m_cls=np.inf, m_iou=np.inf, m_order=np.inf, m_out=np.inf, d_iou=0.0, nan_pairs=0,
                   keep=np.zeros(0, np.int64))
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
    nan_pairs = 0  # same-class pairs whose IoU is NaN (0 / 0) in one run only: such a pair has no margin
    keep_mask = np.zeros(len(cand), bool)
    for c in np.unique(cls):
        sel = order[cls[order] == c]  # this class, in processing order
        ir, io = _iou(b_r[sel]), _iou(b_o[sel])
        n = len(sel)
        if n > 1:
            iu = np.triu_indices(n, 1)
            a_r, a_o = ir[iu], io[iu]
            nr, no = np.isnan(a_r), np.isnan(a_o)
            nan_pairs += int((nr != no).sum())
            both = ~nr & ~no  # NaN in both runs: neither suppresses (ovr > thr is false), the same decision
            if both.any():
                d_iou = max(d_iou, float(np.abs(a_r[both] - a_o[both]).max()))
        kept = []
        for t in range(n):
            col = ir[kept, t]
            col = col[~np.isnan(col)]  # torchvision's ovr > thr: a NaN IoU never suppresses
            mx = float(col.max()) if col.size else 0.0
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
    res["nan_pairs"] = nan_pairs
    res["stable"] = bool(m_conf > 2 * d_s and m_cls > 2 * d_s and m_order > 2 * d_s and m_out > 2 * d_s
                         and m_iou > d_iou_tol and nan_pairs == 0)
    return res


# Bounds on the perturbation of the inputs of a decision that is allowed to flip (replay_divergences): a flip is only
# a near-tie if the two runs' outputs for the anchors it involves agree to within the forward's own accuracy.
SCORE_PERT_MAX = 1e-3  # north_star: outputs within 1e-3 abs of the CPU reference
BOX_PERT_MAX = 0.25    # px: twice the reference fp32 CPU path's own worst box error vs fp64 on the trained-like model
                       # (0.12 px, tests/test_gpu_e2e.py::test_e2e_forward_within_tolerance)


def _rank_before(key_a, idx_a, key_b, idx_b):
    """True where a is processed before b in torchvision's order: descending score, stable (lower index first)."""
    return (key_a > key_b) | ((key_a == key_b) & (idx_a < idx_b))


def replay_divergences(y_ref: np.ndarray, y_oth: np.ndarray, conf=0.25, iou_thres=0.7, max_det=300, max_nms=30000,
                       max_wh=7680):
    """Replay predict-mode NMS (single label, class-aware: ``ultralytics/utils/ops.py:234-297`` around torchvision's
    greedy CPU nms) on ``y_oth``, decision by decision, and at every decision evaluate what ``y_ref`` decides in the
    SAME state. Where they differ the replay records the decision and adopts ``y_oth``'s choice, then keeps going, so
    every divergent decision of the image is found (not only the first one) and the replay ends with NMS(y_oth)'s own
    kept list (``keep``; the caller checks it against the real NMS of y_oth).

    Decisions, each with its margin on y_ref and the perturbation ``pert`` of its own inputs between the two runs:
      * conf    - candidate filter ``max_c score > conf`` (ops.py:234, 275) of one anchor;
      * class   - best class ``argmax_c`` (ops.py:274) of one anchor: top score minus the adopted class's score;
      * max_nms - an anchor crossing the ``max_nms`` cut (ops.py:284-286);
      * order   - processing order of two SAME-class boxes that suppress one another in either run (different
                  classes never interact: the max_wh class offset keeps their boxes apart, ops.py:289-295);
      * iou     - the greedy test ``any IoU(kept, t) > thr`` of one box (torchvision: ``ovr > thr``, so an IoU of
                  0 / 0 = NaN from two zero-area boxes never suppresses; a pair that is NaN in one run only and above
                  the threshold in the other is recorded as kind ``nan``, never justified);
      * out_order - output order / the ``[:max_det]`` cut (ops.py:297): a pair of kept boxes (any classes) in
                  inverted order, the earlier one within max_det.
    A decision is justified (``ok``) when its margin is within twice its own perturbation and the perturbation is
    within the forward's accuracy: every score involved moved by <= SCORE_PERT_MAX, every box coordinate involved by
    <= BOX_PERT_MAX."""
    s_r = np.ascontiguousarray(y_ref[4:].T)
    s_o = np.ascontiguousarray(y_oth[4:].T)
    d_s = np.abs(s_r.astype(np.float64) - s_o)  # [A, nc]
    d_box = np.abs(y_ref[:4].astype(np.float64) - y_oth[:4]).max(0)  # [A]
    dec = []

    def add(kind, anchors, margin, pert, score_anchors=(), box_anchors=(), **kw):
        sp = float(d_s[list(score_anchors)].max()) if len(score_anchors) else 0.0
        bp = float(d_box[list(box_anchors)].max()) if len(box_anchors) else 0.0
        ok = bool(margin <= 2 * pert and sp <= SCORE_PERT_MAX and bp <= BOX_PERT_MAX and kind != "nan")
        dec.append(dict(kind=kind, anchors=[int(a) for a in anchors], margin=float(margin), tol=float(2 * pert),
                        score_pert=sp, box_pert=bp, ok=ok, **kw))

    best_r, best_o = s_r.max(1), s_o.max(1)
    c_r, c_o = best_r > np.float32(conf), best_o > np.float32(conf)
    for a in np.nonzero(c_r != c_o)[0]:
        add("conf", [a], abs(float(best_r[a]) - conf), abs(float(best_r[a]) - float(best_o[a])), score_anchors=[a])
    cand = np.nonzero(c_o)[0]
    res = {"decisions": dec, "keep": np.zeros(0, np.int64)}
    if cand.size == 0:
        res["ok"] = all(d["ok"] for d in dec)
        return res
    cls_o = s_o[cand].argmax(1)
    cls_r = s_r[cand].argmax(1)
    for i in np.nonzero(cls_r != cls_o)[0]:
        a, cr, co = cand[i], cls_r[i], cls_o[i]
        add("class", [a], float(s_r[a, cr]) - float(s_r[a, co]), max(d_s[a, cr], d_s[a, co]), score_anchors=[a])
    sc_o = s_o[cand, cls_o]
    sc_r = s_r[cand, cls_o]  # y_ref's score of the adopted class: the key of its processing order
    order = np.argsort(-sc_o, kind="stable")
    if cand.size > max_nms:
        o_r = np.argsort(-sc_r, kind="stable")
        top_o, top_r = set(order[:max_nms].tolist()), set(o_r[:max_nms].tolist())
        edge = float(sc_r[o_r[max_nms - 1]])
        for i in sorted(top_o ^ top_r):
            add("max_nms", [cand[i]], abs(float(sc_r[i]) - edge), float(d_s[cand[i]].max()), score_anchors=[cand[i]])
        order = order[:max_nms]
    off = (cls_o.astype(np.float32) * np.float32(max_wh))[:, None]
    b_r = (_xyxy(y_ref[:4, cand].T) + off).astype(np.float32)
    b_o = (_xyxy(y_oth[:4, cand].T) + off).astype(np.float32)
    keep_mask = np.zeros(len(cand), bool)
    with np.errstate(invalid="ignore", divide="ignore"):
        for c in np.unique(cls_o[order]):
            sel = order[cls_o[order] == c]  # this class, in y_oth's processing order
            ir, io = _iou(b_r[sel]), _iou(b_o[sel])
            kept = []
            for t in range(len(sel)):
                if kept:
                    rr, ro = ir[kept, t], io[kept, t]
                    nan_r, nan_o = np.isnan(rr), np.isnan(ro)
                    for k in np.nonzero((nan_r != nan_o) & (np.where(nan_r, ro, rr) > iou_thres))[0]:
                        ka, ta = cand[sel[kept[k]]], cand[sel[t]]
                        add("nan", [ka, ta], np.inf, 0.0, box_anchors=[ka, ta])
                    sup_r, sup_o = bool((rr > iou_thres).any()), bool((ro > iou_thres).any())
                    # processing order of the boxes that suppress t in either run
                    for k in np.nonzero((rr > iou_thres) | (ro > iou_thres))[0]:
                        i, j = sel[kept[k]], sel[t]
                        if not _rank_before(sc_r[i], cand[i], sc_r[j], cand[j]):
                            add("order", [cand[i], cand[j]], abs(float(sc_r[i]) - float(sc_r[j])),
                                max(abs(float(sc_r[i]) - float(sc_o[i])), abs(float(sc_r[j]) - float(sc_o[j]))),
                                score_anchors=[cand[i], cand[j]])
                    if sup_r != sup_o:  # (a NaN-only difference is already recorded above)
                        flip = np.nonzero(~nan_r & ~nan_o & ((rr > iou_thres) != (ro > iou_thres)))[0]
                        ks = [cand[sel[kept[k]]] for k in flip]
                        if len(flip):
                                add("iou", ks + [cand[sel[t]]], float(np.abs(rr[flip] - iou_thres).max()),
                                float(np.abs(rr[flip] - ro[flip]).max()), box_anchors=ks + [cand[sel[t]]])
                    if sup_o:
                        continue
                kept.append(t)
            keep_mask[sel[kept]] = True
    kept_idx = order[keep_mask[order]]  # output order: y_oth's processing order (descending score, all classes)
    # output order / max_det cut: pairs of kept boxes whose order y_ref would invert, the earlier one within max_det
    n = len(kept_idx)
    if n > 1:
        kr, ka = sc_r[kept_idx].astype(np.float64), cand[kept_idx]
        ii, jj = np.triu_indices(n, 1)
        m = ii < max_det
        ii, jj = ii[m], jj[m]
        inv = ~_rank_before(kr[ii], ka[ii], kr[jj], ka[jj])
        if inv.any():
            ii, jj = ii[inv], jj[inv]
            pert_k = np.abs(kr - sc_o[kept_idx])
            add("out_order", sorted(set(ka[ii].tolist()) | set(ka[jj].tolist())),
                float(np.abs(kr[ii] - kr[jj]).max()), float(np.maximum(pert_k[ii], pert_k[jj]).max()),
                score_anchors=sorted(set(ka[ii].tolist()) | set(ka[jj].tolist())), pairs=int(inv.sum()))
    res["keep"] = cand[kept_idx[:max_det]].astype(np.int64)
    res["ok"] = all(d["ok"] for d in dec)
    return res


def tie_level(d, rel=2.0 ** -21):
    """A decision whose margin on y_ref is at the level of an fp32 rounding tie of its operands (<= 16 units in the
    last place of a score in [0.5, 1)): the flat scenes' identical receptive fields give exact ties by construction."""
    return d["margin"] <= rel
