"""Detection metrics for the mAP@0.5:0.95 parity harness (host side, numpy / torch-CPU).

Restates the reference's evaluation arithmetic so GPU detections and CPU-reference detections can be scored the same
way (quitedob/yolo-sod = Ultralytics 8.3.63):
  box_iou            ultralytics/utils/metrics.py:52-71     (fp32, eps 1e-7, torchvision formula)
  match_predictions  ultralytics/engine/validator.py:222-262 (greedy, use_scipy=False path)
  smooth             ultralytics/utils/metrics.py:447-452
  compute_ap         ultralytics/utils/metrics.py:505-533   (101-point COCO interpolation)
  ap_per_class       ultralytics/utils/metrics.py:536-622   (max-F1 operating point)
  DetMetrics         ultralytics/utils/metrics.py:640-870   (mp, mr, mAP50, mAP50-95, fitness 0.1/0.9)
Plots / curves output are not reproduced (they do not feed the metrics).
"""
from __future__ import annotations

import numpy as np
import torch

IOU_THRESHOLDS = torch.linspace(0.5, 0.95, 10)  # detect/val.py:41
_trapezoid = getattr(np, "trapezoid", None) or np.trapz


def box_iou(box1: torch.Tensor, box2: torch.Tensor, eps: float = 1e-7) -> torch.Tensor:
    """Pairwise IoU [N, M] of xyxy boxes in fp32, evaluated in the reference's operation order."""
    a = box1.float()[:, None, :]
    b = box2.float()[None, :, :]
    wh = (torch.minimum(a[..., 2:], b[..., 2:]) - torch.maximum(a[..., :2], b[..., :2])).clamp_(0)
    inter = wh.prod(2)
    area1 = (a[..., 2:] - a[..., :2]).prod(2)
    area2 = (b[..., 2:] - b[..., :2]).prod(2)
    return inter / (area1 + area2 - inter + eps)


def match_predictions(pred_classes: torch.Tensor, true_classes: torch.Tensor, iou: torch.Tensor,
                      iouv: torch.Tensor = IOU_THRESHOLDS) -> np.ndarray:
    """[N_pred, len(iouv)] bool: prediction j is a true positive at threshold t. ``iou`` is [N_true, N_pred].

    Per threshold: candidate (label, detection) pairs with class match and IoU >= t, ranked by IoU descending
    (stable order of the flattened nonzero scan for ties), then each detection keeps its best pair and each label its
    first remaining pair (np.unique first-occurrence semantics, as the reference)."""
    correct = np.zeros((pred_classes.shape[0], iouv.shape[0]), dtype=bool)
    same = (true_classes[:, None] == pred_classes[None, :])
    iou = (iou * same).cpu().numpy()
    for ti, thr in enumerate(iouv.tolist()):
        li, di = np.nonzero(iou >= thr)
        if li.size == 0:
            continue
        pairs = np.stack([li, di], 1)
        if pairs.shape[0] > 1:
            pairs = pairs[iou[pairs[:, 0], pairs[:, 1]].argsort()[::-1]]
            pairs = pairs[np.unique(pairs[:, 1], return_index=True)[1]]
            pairs = pairs[np.unique(pairs[:, 0], return_index=True)[1]]
        correct[pairs[:, 1].astype(int), ti] = True
    return correct


def smooth(y: np.ndarray, f: float = 0.05) -> np.ndarray:
    """Box filter over a fraction f of the samples, edge-padded."""
    nf = round(len(y) * f * 2) // 2 + 1
    pad = np.ones(nf // 2)
    yp = np.concatenate((pad * y[0], y, pad * y[-1]))
    return np.convolve(yp, np.ones(nf) / nf, mode="valid")


def compute_ap(recall: np.ndarray, precision: np.ndarray):
    """Area under the precision envelope, sampled at 101 recall points. Returns (ap, envelope, recall axis)."""
    mrec = np.concatenate(([0.0], recall, [1.0]))
    mpre = np.concatenate(([1.0], precision, [0.0]))
    mpre = np.flip(np.maximum.accumulate(np.flip(mpre)))
    x = np.linspace(0, 1, 101)
    return _trapezoid(np.interp(x, mrec, mpre), x), mpre, mrec


def ap_per_class(tp, conf, pred_cls, target_cls, eps: float = 1e-16):
    """Per-class AP over the IoU thresholds and the max-F1 operating point.

    Returns (tp, fp, p, r, f1, ap [nc, T], unique_classes, p_curve, r_curve, f1_curve, x, prec_values)."""
    order = np.argsort(-conf)
    tp, conf, pred_cls = tp[order], conf[order], pred_cls[order]
    classes, n_true = np.unique(target_cls, return_counts=True)
    nc = classes.shape[0]
    x = np.linspace(0, 1, 1000)
    prec_values = []
    ap = np.zeros((nc, tp.shape[1]))
    p_curve, r_curve = np.zeros((nc, 1000)), np.zeros((nc, 1000))
    for ci, c in enumerate(classes):
        sel = pred_cls == c
        n_l, n_p = n_true[ci], sel.sum()
        if n_p == 0 or n_l == 0:
            continue
        fpc = (1 - tp[sel]).cumsum(0)
        tpc = tp[sel].cumsum(0)
        recall = tpc / (n_l + eps)
        r_curve[ci] = np.interp(-x, -conf[sel], recall[:, 0], left=0)
        precision = tpc / (tpc + fpc)
        p_curve[ci] = np.interp(-x, -conf[sel], precision[:, 0], left=1)
        for j in range(tp.shape[1]):
            ap[ci, j], mpre, mrec = compute_ap(recall[:, j], precision[:, j])
            if j == 0:
                prec_values.append(np.interp(x, mrec, mpre))
    prec_values = np.array(prec_values)
    f1_curve = 2 * p_curve * r_curve / (p_curve + r_curve + eps)
    i = smooth(f1_curve.mean(0), 0.1).argmax()
    p, r, f1 = p_curve[:, i], r_curve[:, i], f1_curve[:, i]
    tp_n = (r * n_true).round()
    fp_n = (tp_n / (p + eps) - tp_n).round()
    return tp_n, fp_n, p, r, f1, ap, classes.astype(int), p_curve, r_curve, f1_curve, x, prec_values


class DetMetrics:
    """Box metrics with the reference's keys and means (mp, mr, mAP50, mAP50-95, fitness = 0.1 mAP50 + 0.9 mAP)."""

    keys = ["metrics/precision(B)", "metrics/recall(B)", "metrics/mAP50(B)", "metrics/mAP50-95(B)"]

    def __init__(self):
        self.p = self.r = self.f1 = np.zeros(0)
        self.all_ap = np.zeros((0, 10))
        self.ap_class_index = np.zeros(0, int)

    def process(self, tp, conf, pred_cls, target_cls):
        res = ap_per_class(tp, conf, pred_cls, target_cls)
        self.p, self.r, self.f1, self.all_ap, self.ap_class_index = res[2], res[3], res[4], res[5], res[6]

    @property
    def map50(self):
        return float(self.all_ap[:, 0].mean()) if len(self.all_ap) else 0.0

    @property
    def map75(self):
        return float(self.all_ap[:, 5].mean()) if len(self.all_ap) else 0.0

    @property
    def map(self):
        return float(self.all_ap.mean()) if len(self.all_ap) else 0.0

    def mean_results(self):
        mp = float(self.p.mean()) if len(self.p) else 0.0
        mr = float(self.r.mean()) if len(self.r) else 0.0
        return [mp, mr, self.map50, self.map]

    @property
    def fitness(self):
        return float((np.array(self.mean_results()) * [0.0, 0.0, 0.1, 0.9]).sum())

    @property
    def results_dict(self):
        return dict(zip(self.keys + ["fitness"], self.mean_results() + [self.fitness]))
