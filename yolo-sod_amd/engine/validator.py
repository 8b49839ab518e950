"""Detection evaluator: accumulates per-image statistics and reports mAP like the reference's DetectionValidator.

Mirrors ultralytics/models/yolo/detect/val.py:125-187 (update_metrics, _process_batch, get_stats) for the tensor
path, where predictions and labels live in the same image space (scale_boxes with gain 1, pad 0: predict.py:39,
val.py:113-123), so no rescaling is applied. NMS for validation is the reference's val mode
(val.py:92-102: conf 0.001, iou 0.7, multi_label=True, max_det 300) and runs on the GPU via
``yolosod_amd.utils.ops.non_max_suppression``; matching and AP are host-side (utils/metrics.py).
"""
from __future__ import annotations

import numpy as np
import torch

from ..utils.metrics import IOU_THRESHOLDS, DetMetrics, box_iou, match_predictions

VAL_NMS = dict(conf_thres=0.001, iou_thres=0.7, multi_label=True, max_det=300)


class DetectionEvaluator:
    def __init__(self, nc: int, iouv: torch.Tensor = IOU_THRESHOLDS):
        self.nc = nc
        self.iouv = iouv
        self.niou = iouv.numel()
        self.seen = 0
        self.stats = dict(tp=[], conf=[], pred_cls=[], target_cls=[], target_img=[])
        self.metrics = DetMetrics()

    def update(self, preds, targets):
        """preds: list of [n_i, 6] (x1, y1, x2, y2, conf, cls); targets: list of (cls [m_i], boxes_xyxy [m_i, 4])."""
        for pred, (cls, bbox) in zip(preds, targets):
            self.seen += 1
            pred = pred.detach().float().cpu()
            cls = torch.as_tensor(cls).float().cpu().reshape(-1)
            bbox = torch.as_tensor(bbox).float().cpu().reshape(-1, 4)
            npr, nl = len(pred), len(cls)
            stat = dict(conf=np.zeros(0, np.float32), pred_cls=np.zeros(0, np.float32),
                        tp=np.zeros((npr, self.niou), bool), target_cls=cls.numpy(), target_img=cls.unique().numpy())
            if npr == 0:
                if nl:
                    for k in self.stats:
                        self.stats[k].append(stat[k])
                continue
            stat["conf"] = pred[:, 4].numpy()
            stat["pred_cls"] = pred[:, 5].numpy()
            if nl:
                stat["tp"] = match_predictions(pred[:, 5], cls, box_iou(bbox, pred[:, :4]), self.iouv)
            for k in self.stats:
                self.stats[k].append(stat[k])

    def get_stats(self):
        """Concatenate and score; same gate as the reference (metrics only when any prediction is a TP)."""
        if not self.stats["tp"]:
            return self.metrics.results_dict
        st = {k: np.concatenate(v, 0) for k, v in self.stats.items()}
        st.pop("target_img")
        if len(st) and st["tp"].any():
            self.metrics.process(st["tp"], st["conf"], st["pred_cls"], st["target_cls"])
        return self.metrics.results_dict
