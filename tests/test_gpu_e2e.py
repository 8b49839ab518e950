"""GPU: end-to-end parity of the whole path - GPU forward -> HIP NMS against oracle forward -> oracle NMS.

north_star: "matching the reference PyTorch-CPU forward on identical weights/inputs ... and bit-exact kept-box
indices after NMS" (``ultralytics/utils/ops.py:296-297`` after ``nn/modules/head.py:100-131``). Unlike
test_gpu_checkpoint.py / test_gpu_nms.py, which feed one tensor to both NMS implementations, here each side runs
its own forward, so the kept indices are compared across two fp32 computations of the Detect output.

Workload: the trained-like paper model (tests/trained_like.py: BN recalibrated to unit-variance activations, class
logits in a moderate range) on structured 640x640 scenes; the GPU runs the bench's batch of 32, the oracle 8 of its
images. Rule for the indices (tests/nms_margins.py): an image is *decision-stable* when every NMS decision on the
oracle's output - candidate filter, best class, greedy IoU test, processing order of overlapping boxes, output
order / max_det cut - has a margin of more than twice the perturbation measured between the two forwards. Every
image's kept anchor indices must be bit-identical, in order, except where a decision is that close: such an
exception is allowed only on an image that is not decision-stable, must keep >= 90 % of its kept anchors in common,
and is counted (at most 2 of the 8 images). The GPU's indices always equal the oracle NMS of the GPU's own output. The mAP test scores val-mode detections of both full paths (production fused head, not the
raw-map decode) against the same synthetic labels: |mAP50-95 difference| <= 1e-3
(``models/yolo/detect/val.py:92-102`` -> ``engine/validator.py:222-262``)."""
import os

import numpy as np
import pytest
import torch

from nms_margins import nms_stability
from trained_like import make_trained_like_checkpoint, scenes

pytestmark = pytest.mark.gpu

B_GPU, IMG = 32, 640
ORACLE_IMAGES = list(range(0, B_GPU, 4))  # 8 of the batch


def _log(msg):
    log = os.environ.get("YOLOSOD_PARITY_LOG")
    if log:
        with open(log, "a") as f:
            f.write(f"{os.environ.get('PYTEST_CURRENT_TEST', '?')}: {msg}\n")


@pytest.fixture(scope="module")
def e2e(tmp_path_factory, cuda):
    from oracle.model_ref import REGISTRY
    from yolosod_amd.nn.checkpoint import attempt_load_one_weight
    path = make_trained_like_checkpoint(tmp_path_factory.mktemp("e2e") / "trained_like.pt")
    gm, _ = attempt_load_one_weight(path, device=cuda)
    cm, _ = attempt_load_one_weight(path, device="cpu", registry=REGISTRY)
    x = scenes(777, B_GPU, IMG)
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True  # MIOpen split-K atomics otherwise vary run to run
    try:
        with torch.inference_mode():
            y_gpu = gm(x.to(cuda))[0]
            y_cpu = cm(x[ORACLE_IMAGES])[0]
            y_64 = cm.double()(x[ORACLE_IMAGES].double())[0]  # the exact answer (fp64), for the forward bound
            cm.float()
    finally:
        torch.backends.cudnn.deterministic = det
    return gm, cm, x, y_gpu, y_cpu, y_64


def test_e2e_forward_within_tolerance(e2e):
    """Forward accuracy of the GPU path against the exact (fp64) forward of the same weights, next to the
    reference's own fp32 CPU forward. With unit-variance activations through 40 layers this model is far less
    well conditioned than the random-init one: the reference's fp32 forward itself is 0.12 px off the fp64 one on
    the worst box coordinate (large-box DFL sides at P5) and 1.2e-4 on the scores, so the north-star 1e-3 absolute
    (met at random init, test_gpu_model.py) cannot hold here for any fp32 implementation. Bar: the GPU path is at
    least as close to the exact forward as the reference's fp32 path, within a factor 2 (+1e-3 abs)."""
    _, _, _, y_gpu, y_cpu, y_64 = e2e
    yg = y_gpu[ORACLE_IMAGES].cpu().double()
    for rows, what in ((slice(0, 4), "box"), (slice(4, None), "score")):
        e_gpu = float((yg[:, rows] - y_64[:, rows]).abs().max())
        e_cpu = float((y_cpu[:, rows].double() - y_64[:, rows]).abs().max())
        _log(f"{what} rows: GPU vs fp64 {e_gpu:.3g}, reference-path fp32 CPU vs fp64 {e_cpu:.3g}")
        assert e_gpu <= 2 * e_cpu + 1e-3, (what, e_gpu, e_cpu)


def test_e2e_kept_indices_gpu_vs_oracle(e2e):
    from oracle.nms import non_max_suppression_ref
    from yolosod_amd.utils import ops
    _, _, _, y_gpu, y_cpu, _ = e2e
    yg_all = y_gpu.clone()
    with torch.inference_mode():
        out, counts, index = ops.non_max_suppression_padded(yg_all, 0.25, 0.7, max_det=300)
    yg = y_gpu[ORACLE_IMAGES].cpu().numpy()
    yc = y_cpu.numpy()
    _, idx_cpu = non_max_suppression_ref(yc.copy(), 0.25, 0.7, max_det=300)  # oracle forward -> oracle NMS
    _, idx_gpu_ref = non_max_suppression_ref(yg.copy(), 0.25, 0.7, max_det=300)  # oracle NMS on the GPU output
    exact, stable, kept_exact, report = 0, 0, 0, []
    for k, b in enumerate(ORACLE_IMAGES):
        n = int(counts[b])
        gi = index[b, :n].cpu().numpy().astype(np.int64)
        assert np.array_equal(gi, idx_gpu_ref[k])  # HIP NMS == oracle NMS on the same tensor
        st = nms_stability(yc[k], yg[k])
        assert np.array_equal(st["keep"], idx_cpu[k])  # the margin analysis replays the oracle's greedy NMS
        same = np.array_equal(gi, idx_cpu[k])
        report.append(f"img {b}: kept {n}/{len(idx_cpu[k])} same {same} cand {st['n_cand']} stable {st['stable']} "
                      f"m_conf {st['m_conf']:.2e} m_cls {st['m_cls']:.2e} m_iou {st['m_iou']:.2e} "
                      f"m_order {st['m_order']:.2e} m_out {st['m_out']:.2e} d_score {st['d_score']:.2e} "
                      f"d_iou {st['d_iou']:.2e}")
        stable += st["stable"]
        if same:
            exact += 1
            kept_exact += n
            continue
        # an exception: the indices differ, which is legitimate only at a decision whose margin on the oracle's
        # output is within twice the measured perturbation (never on a decision-stable image); it stays local
        assert not st["stable"], report[-1]
        a, c = set(gi.tolist()), set(idx_cpu[k].tolist())
        assert len(a & c) >= 0.9 * max(len(a | c), 1), report[-1]
    _log(f"{exact}/{len(ORACLE_IMAGES)} images bit-exact ({kept_exact} kept boxes), {stable} decision-stable; "
         + " | ".join(report))
    assert exact >= len(ORACLE_IMAGES) - len(ORACLE_IMAGES) // 4, report  # at most 2 of 8 exceptions
    assert kept_exact >= 100, "too few kept boxes on bit-exact images for the test to mean anything"


def test_e2e_map_through_production_head(e2e):
    """mAP@0.5:0.95 of the full GPU path (fused Detect head + HIP val-mode NMS) vs the full oracle path, same labels."""
    from oracle.nms import non_max_suppression_ref
    from yolosod_amd.engine.validator import VAL_NMS, DetectionEvaluator
    from yolosod_amd.utils.ops import non_max_suppression
    _, _, _, y_gpu, y_cpu, _ = e2e
    nc = y_cpu.shape[1] - 4
    rows_p, _ = non_max_suppression_ref(y_cpu.numpy().copy(), conf_thres=0.25, iou_thres=0.7)
    rng = np.random.default_rng(3)
    labels = []
    for d in rows_p:  # labels: jittered predict-mode oracle detections (60 %) + random boxes
        keep = d[rng.uniform(size=len(d)) < 0.6]
        boxes = keep[:, :4] + rng.normal(0, 3.0, (len(keep), 4)).astype(np.float32)
        m = int(rng.integers(2, 10))
        xy = rng.uniform(0, IMG - 60, (m, 2))
        rnd = np.concatenate([xy, xy + rng.uniform(8, 60, (m, 2))], 1).astype(np.float32)
        labels.append((np.concatenate([keep[:, 5], rng.integers(0, nc, m).astype(np.float32)]),
                       np.concatenate([boxes, rnd]).astype(np.float32)))
    with torch.inference_mode():
        dets_gpu = non_max_suppression(y_gpu[ORACLE_IMAGES].clone(), **VAL_NMS)
    rows_cpu, _ = non_max_suppression_ref(y_cpu.numpy().copy(), **VAL_NMS)
    e_gpu, e_cpu = DetectionEvaluator(nc), DetectionEvaluator(nc)
    e_gpu.update(dets_gpu, labels)
    e_cpu.update([torch.from_numpy(r) for r in rows_cpu], labels)
    m_gpu, m_cpu = e_gpu.get_stats(), e_cpu.get_stats()
    _log(f"mAP50-95 gpu {m_gpu['metrics/mAP50-95(B)']:.6f} cpu {m_cpu['metrics/mAP50-95(B)']:.6f}; "
         f"dets {[len(d) for d in dets_gpu]} vs {[len(r) for r in rows_cpu]}")
    assert m_cpu["metrics/mAP50-95(B)"] > 0.05, m_cpu
    for k in m_cpu:
        assert abs(m_gpu[k] - m_cpu[k]) <= 1e-3, (k, m_gpu[k], m_cpu[k])
