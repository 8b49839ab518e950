"""CPU: the decision-margin analysis used by the end-to-end parity test (tests/nms_margins.py) replays the oracle's
greedy NMS exactly (same kept anchors, same order), and flags perturbations that flip a decision."""
import numpy as np
import pytest

import recipes
from nms_margins import first_divergence, nms_stability
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


def test_first_divergence_none_when_kept_lists_agree():
    pred = recipes.synthetic_predictions(21, 2, 3000, 10)
    for b in range(2):
        assert first_divergence(pred[b], pred[b].copy()) is None


@pytest.mark.parametrize("kind", ["conf", "class", "order", "iou"])
def test_first_divergence_locates_the_flipped_decision(kind):
    """Each kind of decision flipped by a tiny perturbation is found, with its small margin; the kept lists of the
    two runs (oracle NMS) differ when the flipped IoU test un-suppresses a box."""
    pred = recipes.synthetic_predictions(22, 1, 3000, 10)[0].copy()
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
    elif kind == "order":  # two candidates whose scores swap
        a, b = int(cand[0]), int(cand[1])
        ca, cb = int(s[a].argmax()), int(s[b].argmax())
        s[b, :] = np.minimum(s[b], np.float32(0.2))  # b's best class stays cb
        so[b, :] = s[b]
        s[b, cb] = s[a, ca] - eps
        so[b, cb] = s[a, ca] + eps
    else:  # a box moved across the IoU threshold against the box that would suppress it
        x, y = int(cand[0]), int(cand[1])
        cx = int(s[x].argmax())
        s[:, :] = np.minimum(s, np.float32(0.2))
        s[x, cx], s[y, cx] = np.float32(0.9), np.float32(0.8)
        so[:, :] = s
        pred[:4, x] = oth[:4, x] = [100.0, 100.0, 40.0, 40.0]
        # IoU of two 40x40 boxes offset by dx along x: (40 - dx) / (40 + dx); 0.7 at dx = 40 * 0.3 / 1.7
        dx = np.float32(40 * 0.3 / 1.7)
        pred[:4, y] = [100.0 + dx + 0.01, 100.0, 40.0, 40.0]  # +-0.01: the flip survives the class offset
        oth[:4, y] = [100.0 + dx - 0.01, 100.0, 40.0, 40.0]
    fd = first_divergence(pred, oth)
    assert fd is not None and fd["kind"] == kind, fd
    assert fd["margin"] <= fd["tol"], fd
    _, ir = non_max_suppression_ref(pred[None].copy(), 0.25, 0.7, max_det=300)
    _, io = non_max_suppression_ref(oth[None].copy(), 0.25, 0.7, max_det=300)
    if kind == "iou":  # the box the perturbation un-suppresses is kept by the second run only
        assert not np.array_equal(ir[0], io[0])
