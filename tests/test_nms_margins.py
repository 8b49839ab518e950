"""CPU: the decision-margin analysis used by the end-to-end parity test (tests/nms_margins.py) replays the oracle's
greedy NMS exactly (same kept anchors, same order), flags perturbations that flip a decision, and the side-by-side
replay (replay_divergences) finds EVERY divergent decision of an image, each with its own perturbation, while ending
on the second run's own NMS result."""
import warnings

import numpy as np
import pytest

import recipes
from nms_margins import SCORE_PERT_MAX, nms_stability, replay_divergences
from oracle.nms import non_max_suppression_ref


@pytest.mark.parametrize("seed,max_det", [(11, 300), (12, 300), (13, 40)])
def test_margin_replay_matches_oracle_nms(seed, max_det):
    pred = recipes.synthetic_predictions(seed, 2, 3000, 10)
    _, idx = non_max_suppression_ref(pred.copy(), 0.25, 0.7, max_det=max_det)
    for b in range(2):
        st = nms_stability(pred[b], pred[b], max_det=max_det)
        assert np.array_equal(st["keep"], idx[b])
        assert st["d_score"] == 0.0 and st["d_iou"] == 0.0


def test_margin_flags_a_flipping_perturbation():
    pred = recipes.synthetic_predictions(11, 1, 3000, 10)[0]
    st = nms_stability(pred, pred)
    assert st["n_cand"] > 0
    # perturb by more than the smallest score margin: the analysis must call the image unstable
    d = 4 * min(st["m_conf"], st["m_order"], st["m_out"])
    other = pred.copy()
    other[4:] += np.float32(d)
    assert not nms_stability(pred, other)["stable"]
    # and a perturbation far below every margin keeps it stable when the margins are large
    tiny = pred.copy()
    tiny[4:] = np.nextafter(tiny[4:], np.float32(2))
    st2 = nms_stability(pred, tiny)
    assert st2["stable"] == (min(st2["m_conf"], st2["m_cls"], st2["m_order"], st2["m_out"]) > 2 * st2["d_score"]
                             and st2["m_iou"] > 1e-6)


def _flip(kind, seed=22):
    """(pred, oth): one image whose two versions differ by a tiny perturbation that flips one decision of ``kind``."""
    pred = recipes.synthetic_predictions(seed, 1, 3000, 10)[0].copy()
    s = pred[4:].T  # view [A, nc]
    best = s.max(1)
    cand = np.nonzero(best > 0.25)[0]
    oth = pred.copy()
    so = oth[4:].T
    eps = np.float32(1e-6)
    if kind == "conf":  # a non-candidate moved just below / above the threshold
        x = int(np.nonzero(best <= 0.25)[0][0])
        c = int(s[x].argmax())
        s[x, c] = np.float32(0.25) - eps
        so[x, c] = np.float32(0.25) + eps
    elif kind == "class":  # a candidate with two near-equal top classes
        x = int(cand[0])
        c = int(s[x].argmax())
        c2 = (c + 1) % s.shape[1]
        s[x, c2] = s[x, c] - eps
        so[x, c2] = s[x, c] + eps
        so[x, c] = s[x, c]
    elif kind in ("order", "iou"):  # two same-class boxes over the IoU threshold (order: their scores swap)
        x, y = int(cand[0]), int(cand[1])
        cx = int(s[x].argmax())
        s[:, :] = np.minimum(s, np.float32(0.2))
        s[x, cx], s[y, cx] = np.float32(0.9), np.float32(0.8)
        pred[:4, x] = [100.0, 100.0, 40.0, 40.0]
        if kind == "order":
            pred[:4, y] = [101.0, 100.0, 40.0, 40.0]
            s[y, cx] = np.float32(0.9) - eps
            so[:, :] = s
            so[y, cx] = np.float32(0.9) + eps
            oth[:4] = pred[:4]
        else:
            so[:, :] = s
            oth[:4, x] = pred[:4, x]
            # IoU of two 40x40 boxes offset by dx along x: (40 - dx) / (40 + dx); 0.7 at dx = 40 * 0.3 / 1.7
            dx = np.float32(40 * 0.3 / 1.7)
            pred[:4, y] = [100.0 + dx + 0.01, 100.0, 40.0, 40.0]  # +-0.01: the flip survives the class offset
            oth[:4, y] = [100.0 + dx - 0.01, 100.0, 40.0, 40.0]
    return pred, oth


def _nms(p, **kw):
    kw = dict(dict(max_det=300), **kw)
    return non_max_suppression_ref(p[None].copy(), 0.25, 0.7, **kw)[1][0]


def test_replay_no_decisions_when_outputs_agree():
    pred = recipes.synthetic_predictions(21, 2, 3000, 10)
    for b in range(2):
        r = replay_divergences(pred[b], pred[b].copy())
        assert r["decisions"] == [] and r["ok"]
        assert np.array_equal(r["keep"], _nms(pred[b]))


@pytest.mark.parametrize("kind", ["conf", "class", "order", "iou"])
def test_replay_finds_the_flipped_decision(kind):
    """Each kind of decision flipped by a tiny perturbation is found and justified; the replay ends on the second
    run's own NMS result; an IoU flip changes the kept lists."""
    pred, oth = _flip(kind)
    r = replay_divergences(pred, oth)
    kinds = [d["kind"] for d in r["decisions"]]
    assert kind in kinds, r["decisions"]
    assert r["ok"], r["decisions"]
    assert np.array_equal(r["keep"], _nms(oth))
    if kind in ("iou", "order"):
        assert not np.array_equal(_nms(pred), _nms(oth))


def test_replay_keeps_going_past_the_first_divergence():
    """Two flips in one image (a candidate-filter flip, then an IoU flip later in the processing order): both are
    recorded, not only the first."""
    pred, oth = _flip("iou")
    s, so = pred[4:].T, oth[4:].T
    x = int(np.nonzero(s.max(1) <= 0.25)[0][-1])
    s[x, 0] = np.float32(0.25) - np.float32(1e-6)
    so[x, 0] = np.float32(0.25) + np.float32(1e-6)
    r = replay_divergences(pred, oth)
    kinds = [d["kind"] for d in r["decisions"]]
    assert "conf" in kinds and "iou" in kinds, kinds
    assert np.array_equal(r["keep"], _nms(oth))


def test_replay_cross_class_order_swap_is_not_a_processing_decision():
    """Two kept boxes of different classes that swap places: no processing-order decision (class offsets keep them
    apart), only the output order of the kept list."""
    pred = recipes.synthetic_predictions(23, 1, 3000, 10)[0].copy()
    keep = _nms(pred)
    s = pred[4:].T
    a, b = int(keep[0]), int(keep[1])
    ca, cb = int(s[a].argmax()), int(s[b].argmax())
    if ca == cb:
        b = int(next(k for k in keep if int(s[k].argmax()) != ca))
        cb = int(s[b].argmax())
    oth = pred.copy()
    so = oth[4:].T
    s[b, cb] = s[a, ca] - np.float32(1e-6)
    so[b, cb] = s[a, ca] + np.float32(1e-6)
    r = replay_divergences(pred, oth)
    kinds = {d["kind"] for d in r["decisions"]}
    assert "order" not in kinds and "out_order" in kinds, r["decisions"]
    assert r["ok"] and np.array_equal(r["keep"], _nms(oth))


def test_replay_rejects_a_flip_with_a_large_perturbation():
    """A flip is a near-tie only if the anchors it involves moved by no more than the forward's accuracy: a score
    moved by 2e-2 across the threshold is not justified, whatever its margin."""
    pred = recipes.synthetic_predictions(24, 1, 3000, 10)[0].copy()
    s = pred[4:].T
    oth = pred.copy()
    so = oth[4:].T
    x = int(np.nonzero(s.max(1) <= 0.25)[0][0])
    c = int(s[x].argmax())
    s[x, c] = np.float32(0.24)
    so[x, c] = np.float32(0.26)
    r = replay_divergences(pred, oth)
    d = [d for d in r["decisions"] if d["kind"] == "conf"]
    assert d and d[0]["margin"] <= d[0]["tol"] and d[0]["score_pert"] > SCORE_PERT_MAX and not r["ok"]


def test_replay_nan_iou_of_zero_area_boxes():
    """Two identical zero-area boxes: IoU 0 / 0 = NaN never suppresses (torchvision ``ovr > thr``), so both are kept
    in both runs; if the second run gives one of them a width that puts the pair over the threshold, the NaN / non-NaN
    split is recorded as kind "nan" and never justified."""
    pred, _ = _flip("iou")
    s = pred[4:].T
    x, y = [int(a) for a in np.argsort(-s.max(1))[:2]]
    c = int(s[x].argmax())
    s[y, :] = s[x] * np.float32(0.99)
    pred[:4, x] = pred[:4, y] = [300.0, 300.0, 0.0, 30.0]
    keep = _nms(pred)
    assert x in keep and y in keep
    assert not replay_divergences(pred, pred.copy())["decisions"]
    oth = pred.copy()
    oth[:4, x] = oth[:4, y] = [300.0, 300.0, 0.5, 30.0]  # same boxes, now 0.5 px wide (survives the class offset): IoU 1
    r = replay_divergences(pred, oth)
    assert "nan" in {d["kind"] for d in r["decisions"]} and not r["ok"]
    assert np.array_equal(r["keep"], _nms(oth))
    assert c == int(s[y].argmax())
    # the margin analysis: a pair NaN in one run only has no margin, so the image is not decision-stable (min(inf,
    # nan) used to fold it away as stable), and no RuntimeWarning escapes
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        st = nms_stability(pred, oth)
        same = nms_stability(pred, pred.copy())
    assert st["nan_pairs"] >= 1 and not st["stable"]
    assert same["nan_pairs"] == 0 and np.isfinite(same["m_iou"])
    assert np.array_equal(same["keep"], keep)


@pytest.mark.parametrize("case", ["nms_degenerate", "nms_ties", "nms_predict"])
@pytest.mark.parametrize("max_det", [300, 40])
def test_replay_ends_on_the_second_runs_nms(case, max_det):
    """Random tiny perturbations of scores and boxes (zero-area and duplicate boxes, exact score ties): whatever
    decisions flip, the replay ends exactly on the oracle NMS of the perturbed output, and every recorded decision is
    justified."""
    pred, kw = recipes.nms_case(case)
    rng = np.random.default_rng(5)
    for b in range(pred.shape[0]):
        p = pred[b]
        o = p.copy()
        o[4:] += (rng.normal(0, 2e-6, o[4:].shape)).astype(np.float32)
        o[:4] += (rng.normal(0, 1e-4, o[:4].shape) * (o[:4] != 0)).astype(np.float32)
        r = replay_divergences(p, o, max_det=max_det)
        assert np.array_equal(r["keep"], _nms(o, max_det=max_det)), case
        assert r["ok"], [d for d in r["decisions"] if not d["ok"]]
        r0 = replay_divergences(p, p.copy(), max_det=max_det)
        assert not r0["decisions"] and np.array_equal(r0["keep"], _nms(p, max_det=max_det))
