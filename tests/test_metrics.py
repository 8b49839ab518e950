"""CPU: the mAP harness (yolosod_amd.utils.metrics / engine.validator) against the reference's own box_iou,
match_predictions and DetMetrics on a synthetic label + detection set (tests/golden/metrics_eval.npz, made by
make_golden.py gen_metrics from the reference)."""
import json

import numpy as np
import torch

import recipes
from conftest import golden
from yolosod_amd.engine.validator import DetectionEvaluator
from yolosod_amd.utils.metrics import ap_per_class, box_iou, compute_ap, match_predictions


def _split(z):
    gi = np.cumsum(np.r_[0, z["gt_n"]])
    pi = np.cumsum(np.r_[0, z["pred_n"]])
    gt = [(z["gt_cls"][gi[i]:gi[i + 1]], z["gt_boxes"][gi[i]:gi[i + 1]]) for i in range(len(z["gt_n"]))]
    preds = [z["pred"][pi[i]:pi[i + 1]] for i in range(len(z["pred_n"]))]
    return gt, preds


def test_fixture_inputs_regenerate():
    z = golden("metrics_eval")
    gt, preds = recipes.synthetic_eval_set(21)
    assert np.array_equal(np.concatenate([g[1] for g in gt]), z["gt_boxes"])
    assert np.array_equal(np.concatenate(preds), z["pred"])


def test_match_predictions_bit_exact():
    z = golden("metrics_eval")
    gt, preds = _split(z)
    tps = []
    for (cls, boxes), pred in zip(gt, preds):
        if len(pred) and len(cls):
            p = torch.from_numpy(pred)
            tps.append(match_predictions(p[:, 5], torch.from_numpy(cls), box_iou(torch.from_numpy(boxes), p[:, :4])))
        elif len(pred):
            tps.append(np.zeros((len(pred), 10), bool))
    assert np.array_equal(np.concatenate(tps), z["tp"])


def test_evaluator_matches_reference_metrics():
    z = golden("metrics_eval")
    gt, preds = _split(z)
    ev = DetectionEvaluator(nc=6)
    ev.update([torch.from_numpy(p) for p in preds], gt)
    res = ev.get_stats()
    ref = json.loads(str(z["results"]))
    for k, v in ref.items():
        assert abs(res[k] - v) <= 1e-12, (k, res[k], v)
    np.testing.assert_allclose(ev.metrics.all_ap, z["all_ap"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(ev.metrics.p, z["p"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(ev.metrics.r, z["r"], rtol=0, atol=1e-12)
    assert ev.metrics.ap_class_index.tolist() == z["ap_class_index"].tolist()
    assert 0.2 < res["metrics/mAP50-95(B)"] < res["metrics/mAP50(B)"] < 1


def test_edge_cases():
    # the 101-point interpolation loses the last half step: the reference scores a perfect detector 0.995
    assert abs(compute_ap(np.array([1.0]), np.array([1.0]))[0] - 0.995) < 1e-12
    ev = DetectionEvaluator(nc=3)
    ev.update([torch.zeros(0, 6)], [(np.zeros(0), np.zeros((0, 4)))])
    assert ev.get_stats()["metrics/mAP50-95(B)"] == 0.0
    tp = np.zeros((4, 10), bool)
    out = ap_per_class(tp, np.array([0.9, 0.8, 0.7, 0.1]), np.zeros(4), np.zeros(2))
    assert out[5].sum() == 0.0
