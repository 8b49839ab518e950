"""GPU NMS: bit-exact kept rows, counts, anchor indices and in-place rewrite vs the reference fixtures and the
oracle (including ties, class filter, agnostic, multi-label, max_nms / max_det cuts, empty, IoU threshold 0)."""
import json

import numpy as np
import pytest
import torch

import recipes
from conftest import golden
from oracle.nms import non_max_suppression_ref

pytestmark = pytest.mark.gpu


def _run_gpu(pred_np, cuda, **kw):
    from yolosod_amd.utils.ops import non_max_suppression_padded
    p = torch.from_numpy(pred_np.copy()).to(cuda)
    out, counts, index = non_max_suppression_padded(p, **kw)
    return p.cpu().numpy(), out.cpu().numpy(), counts.cpu().numpy(), index.cpu().numpy()


@pytest.mark.parametrize("name", list(recipes.NMS_CASES))
def test_nms_matches_reference_fixture(name, cuda):
    z = golden(name)
    kw = json.loads(str(z["kwargs"]))
    p_after, out, counts, index = _run_gpu(z["pred"], cuda, **kw)
    assert np.array_equal(p_after, z["pred_after"]), "in-place xyxy rewrite differs"
    assert counts.tolist() == z["counts"].tolist()
    rows = np.concatenate([out[b, :c] for b, c in enumerate(counts)]) if counts.sum() else np.zeros((0, 6))
    idx = np.concatenate([index[b, :c] for b, c in enumerate(counts)]) if counts.sum() else np.zeros((0,))
    assert np.array_equal(rows, z["rows"]), "kept rows differ (must be bit-exact)"
    assert np.array_equal(idx, z["index"]), "kept anchor indices differ"


def test_nms_list_api(cuda):
    from yolosod_amd.utils.ops import non_max_suppression
    z = golden("nms_predict")
    res = non_max_suppression(torch.from_numpy(z["pred"].copy()).to(cuda), 0.25, 0.7)
    assert [len(r) for r in res] == z["counts"].tolist()
    assert np.array_equal(torch.cat(res).cpu().numpy(), z["rows"])


@pytest.mark.parametrize("B,A,clusters,kw", [
    (8, 34000, 200, dict(conf_thres=0.25, iou_thres=0.7)),
    (4, 34000, 60, dict(conf_thres=0.001, iou_thres=0.7, multi_label=True)),
    (2, 34000, 3000, dict(conf_thres=0.05, iou_thres=0.5, max_det=1000)),
    (2, 136000, 400, dict(conf_thres=0.25, iou_thres=0.7)),
    # max_det above the 1024 LDS kept-list (the reference has no cap, ops.py:297): workspace kept lists
    (2, 34000, 8000, dict(conf_thres=0.05, iou_thres=0.5, max_det=4000)),
    (1, 34000, 6000, dict(conf_thres=0.001, iou_thres=0.6, multi_label=True, max_det=3000)),
])
def test_nms_full_size_vs_oracle(B, A, clusters, kw, cuda):
    pred = recipes.synthetic_predictions(1000 + B + A, B, A, 10, n_clusters=clusters)
    p_after, out, counts, index = _run_gpu(pred, cuda, **kw)
    ref = pred.copy()
    rows, idx = non_max_suppression_ref(ref, **kw)
    assert np.array_equal(p_after, ref)
    assert counts.tolist() == [len(r) for r in rows]
    for b in range(B):
        assert np.array_equal(out[b, :counts[b]], rows[b]), b
        assert np.array_equal(index[b, :counts[b]], idx[b]), b


@pytest.mark.parametrize("B,A,clusters,kw", [
    (2, 34000, 200, dict(conf_thres=0.25, iou_thres=0.7)),
    (2, 34000, 3000, dict(conf_thres=0.05, iou_thres=0.45, max_det=1000)),
    (1, 34000, 30, dict(conf_thres=0.001, iou_thres=0.7, multi_label=True, max_nms=5000)),
])
def test_nms_full_size_ties_vs_oracle(B, A, clusters, kw, cuda):
    """Scores quantised to 1/16: huge tie groups straddle the prefix threshold of the top-KCAP selection and the
    remainder path; stable (index) order among equal scores must match the reference."""
    pred = recipes.synthetic_predictions(2000 + B + clusters, B, A, 10, n_clusters=clusters, tie_scores=True)
    p_after, out, counts, index = _run_gpu(pred, cuda, **kw)
    ref = pred.copy()
    rows, idx = non_max_suppression_ref(ref, **kw)
    assert np.array_equal(p_after, ref)
    assert counts.tolist() == [len(r) for r in rows]
    for b in range(B):
        assert np.array_equal(out[b, :counts[b]], rows[b]), b
        assert np.array_equal(index[b, :counts[b]], idx[b]), b


@pytest.mark.parametrize("kw", [
    dict(conf_thres=0.25, iou_thres=0.7),
    dict(conf_thres=0.25, iou_thres=0.45, multi_label=True, max_det=600),
])
def test_nms_remainder_class_lists_out_of_band(kw, cuda):
    """Three clusters (the remainder path past the 2048-row prefix), 40 % of the boxes moved across x = max_wh (7680)
    and 10 % to negative x: boxes outside their class's x band overlap boxes of the next class in the reference's
    offset space (cross-class suppression), which any class-partitioned shortcut of the remainder's kept-list test
    would have to handle. Must equal the all-pairs reference."""
    B, A = 2, 34000
    pred = recipes.synthetic_predictions(3131, B, A, 10, n_clusters=3)
    rng = np.random.default_rng(9)
    for b in range(B):
        u = rng.uniform(0, 1, A)
        pred[b, 0, u < 0.4] += 7680.0 - 320.0
        pred[b, 0, (u >= 0.4) & (u < 0.5)] -= 640.0
    p_after, out, counts, index = _run_gpu(pred, cuda, **kw)
    ref = pred.copy()
    rows, idx = non_max_suppression_ref(ref, **kw)
    assert np.array_equal(p_after, ref)
    assert counts.tolist() == [len(r) for r in rows]
    for b in range(B):
        assert np.array_equal(out[b, :counts[b]], rows[b]), b
        assert np.array_equal(index[b, :counts[b]], idx[b]), b


@pytest.mark.parametrize("mode", ["all_equal", "low_byte", "low_byte_multi"])
def test_nms_prefix_select_shared_key_digits(mode, cuda):
    """The top-KCAP select skips the key digits all candidates share: 5000 candidates per image whose scores are all
    equal (nothing below the threshold key: everything goes through the remainder path) or differ only in the lowest
    mantissa byte (the select runs its last digit pass only); multi-label takes the global-memory select (n > the
    register path's capacity)."""
    B, A, nc = 2, 34000, 10
    pred = recipes.synthetic_predictions(4242, B, A, nc, n_clusters=300)
    rng = np.random.default_rng(5)
    pred[:, 4:] = 0.0
    multi = mode == "low_byte_multi"
    for b in range(B):
        sel = rng.choice(A, 5000, replace=False)
        for j in (range(nc) if multi else (0,)):
            cls = (sel + j) % nc
            if mode == "all_equal":
                pred[b, 4 + cls, sel] = 0.5
            else:
                bits = np.float32(0.5).view(np.uint32) + rng.integers(0, 256, sel.size).astype(np.uint32)
                pred[b, 4 + cls, sel] = bits.view(np.float32)
    kw = dict(conf_thres=0.25, iou_thres=0.6, max_det=300, multi_label=multi)
    p_after, out, counts, index = _run_gpu(pred, cuda, **kw)
    ref = pred.copy()
    rows, idx = non_max_suppression_ref(ref, **kw)
    assert np.array_equal(p_after, ref)
    assert counts.tolist() == [len(r) for r in rows]
    for b in range(B):
        assert np.array_equal(out[b, :counts[b]], rows[b]), b
        assert np.array_equal(index[b, :counts[b]], idx[b]), b


def test_torch_ops_reject_wrong_sized_partials_and_devices(cuda):
    """Public torch.ops boundary: producer partials of the wrong size raise (TORCH_CHECK) instead of being read out
    of bounds on the GPU."""
    from yolosod_amd import _hip
    ops = _hip.ops()
    x = torch.randn(2, 32, 40, 40, device=cuda)
    w1, b1 = torch.randn(4, 32, device=cuda), torch.randn(4, device=cuda)
    w2, b2 = torch.randn(32, 4, device=cuda), torch.randn(32, device=cuda)
    bad = torch.zeros(7, device=cuda)
    with pytest.raises(RuntimeError, match="psum"):
        ops.se_fwd(x, w1, b1, w2, b2, bad)
    sa = torch.randn(98, device=cuda)
    with pytest.raises(RuntimeError, match="psum"):
        ops.cbam_fwd(x, w1, w2, sa, bad, bad)


@pytest.mark.parametrize("kw", [dict(conf_thres=0.25, iou_thres=0.7), dict(conf_thres=0.001, iou_thres=0.6,
                                                                           multi_label=True)])
def test_nms_not_in_place_leaves_prediction_untouched(kw, cuda):
    """in_place=False (DetectionPredictor's call: its Detect output is local) gives the same rows / indices as the
    in-place call and leaves the prediction tensor bit-identical, without a copy."""
    from yolosod_amd.utils.ops import non_max_suppression_padded
    pred = recipes.synthetic_predictions(77, 4, 34000, 10, n_clusters=300)
    p = torch.from_numpy(pred.copy()).to(cuda)
    out, counts, index = non_max_suppression_padded(p, in_place=False, **kw)
    assert np.array_equal(p.cpu().numpy(), pred)
    p_after, out2, counts2, index2 = _run_gpu(pred, cuda, **kw)
    assert torch.equal(counts.cpu(), torch.from_numpy(counts2)) and torch.equal(index.cpu(), torch.from_numpy(index2))
    assert np.array_equal(out.cpu().numpy(), out2)


def test_nms_empty_and_sparse_blocks(cuda):
    """Images without candidates (random-init heads: nothing clears conf) and images whose candidates sit in a few
    256-anchor blocks only: nms_prep stores masks / boxes for candidate blocks only and nms_scatter skips the
    rest; results equal the oracle on a workspace filled with garbage first."""
    from yolosod_amd.utils.ops import non_max_suppression_padded
    g = np.random.default_rng(8)
    B, A, nc = 6, 34000, 10
    pred = np.zeros((B, 4 + nc, A), np.float32)
    pred[:, 0:2] = g.uniform(0, 640, (B, 2, A))
    pred[:, 2:4] = g.uniform(4, 90, (B, 2, A))
    pred[:, 4:] = g.uniform(0, 0.2, (B, nc, A))  # below conf everywhere
    for b, blocks in ((1, [0]), (3, [7, 8, 132]), (5, list(range(0, 133, 11)))):
        for blk in blocks:
            a = np.arange(blk * 256, min(A, blk * 256 + 256))[g.uniform(size=min(256, A - blk * 256)) < 0.3]
            pred[b, 4 + g.integers(0, nc, a.size), a] = g.uniform(0.3, 1.0, a.size).astype(np.float32)
    torch.empty(64 << 20, dtype=torch.uint8, device=cuda).fill_(0xA5)  # recycled by the caching allocator: garbage
    p_after, out, counts, index = _run_gpu(pred, cuda, conf_thres=0.25, iou_thres=0.7)
    ref = pred.copy()
    rows, idx = non_max_suppression_ref(ref, 0.25, 0.7)
    assert np.array_equal(p_after, ref)
    assert counts.tolist() == [len(r) for r in rows] and counts[0] == 0 and counts[3] > 0
    for b in range(B):
        assert np.array_equal(out[b, :counts[b]], rows[b]), b
        assert np.array_equal(index[b, :counts[b]], idx[b]), b
        assert (out[b, counts[b]:] == 0).all() and (index[b, counts[b]:] == -1).all()
