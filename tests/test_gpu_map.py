"""GPU: mAP@0.5:0.95 parity of the hot path. Synthetic raw Detect maps go through (a) the HIP decode + HIP NMS in the
reference's val mode and (b) the CPU oracle decode + oracle NMS; both detection sets are scored with the same
evaluator against the same synthetic labels (jittered predict-mode detections of the oracle plus random boxes).
Bar: identical kept-box counts per image and |mAP_gpu - mAP_cpu| <= 1e-3 (the decode differs by fp32 rounding only,
which can flip an IoU-threshold crossing in rare cases); in practice the two agree exactly."""
import numpy as np
import pytest
import torch

from oracle import ops_ref as R
from oracle.nms import non_max_suppression_ref
from yolosod_amd import _hip
from yolosod_amd.engine.validator import VAL_NMS, DetectionEvaluator
from yolosod_amd.utils.ops import non_max_suppression

pytestmark = pytest.mark.gpu

STRIDES = [4.0, 8.0, 16.0, 32.0]


def _maps(B, img, nc, seed):
    g = torch.Generator().manual_seed(seed)
    maps = []
    for s in STRIDES:
        h = w = int(img // s)
        box = torch.randn(B, 64, h, w, generator=g) * 2.0
        cls = torch.randn(B, nc, h, w, generator=g) * 2.5 - 3.0
        maps.append(torch.cat([box, cls], 1))
    return maps


def _labels(dets_predict, B, nc, img, seed):
    rng = np.random.default_rng(seed)
    out = []
    for b in range(B):
        d = dets_predict[b]
        keep = d[rng.uniform(size=len(d)) < 0.6]
        boxes = keep[:, :4] + rng.normal(0, 2.0, (len(keep), 4)).astype(np.float32)
        cls = keep[:, 5].copy()
        m = int(rng.integers(0, 8))
        xy = rng.uniform(0, img - 30, (m, 2))
        rnd = np.concatenate([xy, xy + rng.uniform(6, 60, (m, 2))], 1).astype(np.float32)
        out.append((np.concatenate([cls, rng.integers(0, nc, m).astype(np.float32)]),
                    np.concatenate([boxes, rnd]).astype(np.float32)))
    return out


@pytest.mark.parametrize("B,img,nc,seed", [(4, 256, 10, 0), (2, 640, 10, 1)])
def test_map_parity_gpu_vs_cpu_reference(B, img, nc, seed, cuda):
    maps = _maps(B, img, nc, seed)
    y_cpu = R.decode_ref(maps, STRIDES, nc).float()
    y_gpu = _hip.detect_decode([m.to(cuda) for m in maps], STRIDES, nc)
    # labels from the oracle's predict-mode detections
    rows_p, _ = non_max_suppression_ref(y_cpu.numpy().copy(), conf_thres=0.25, iou_thres=0.7)
    labels = _labels(rows_p, B, nc, img, seed)
    # val-mode detections, both paths
    rows_cpu, _ = non_max_suppression_ref(y_cpu.numpy().copy(), **VAL_NMS)
    dets_gpu = non_max_suppression(y_gpu, **VAL_NMS)
    assert [len(d) for d in dets_gpu] == [len(r) for r in rows_cpu]
    e_gpu, e_cpu = DetectionEvaluator(nc), DetectionEvaluator(nc)
    e_gpu.update(dets_gpu, labels)
    e_cpu.update([torch.from_numpy(r) for r in rows_cpu], labels)
    m_gpu, m_cpu = e_gpu.get_stats(), e_cpu.get_stats()
    assert m_cpu["metrics/mAP50-95(B)"] > 0.05, m_cpu  # a non-trivial workload
    for k in m_cpu:
        assert abs(m_gpu[k] - m_cpu[k]) <= 1e-3, (k, m_gpu[k], m_cpu[k])
