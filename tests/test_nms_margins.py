"""CPU: the decision-margin analysis used by the end-to-end parity test (tests/nms_margins.py) replays the oracle's
greedy NMS exactly (same kept anchors, same order), and flags perturbations that flip a decision."""
import numpy as np
import pytest

import recipes
from nms_margins import nms_stability
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
