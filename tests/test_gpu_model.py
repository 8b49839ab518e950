"""GPU end-to-end: the seed-0 paper model (backbone on PyTorch-ROCm + HIP hot path) against the reference's fused
fp32 CPU forward (golden and recorded 640x640 checksums) and against the oracle CPU model; the BASELINE batch
(bs=32) against the oracle on a subset of its images.

Tolerances (oplib.pred_close): box rows 1e-3 abs (north star); class-probability rows in logit space,
|dp| <= 1e-4 p (1 - p) (+2 ulp), i.e. 1e-4 relative at random-init scores (~2e-5): a class branch that is off by
more than that, or returns zeros, fails (an absolute 1e-3 over the whole tensor would pass it)."""
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden
from oplib import pred_close, tol_close

pytestmark = pytest.mark.gpu

ATOL = 1e-3


@pytest.fixture(scope="module")
def gpu_model(cuda):
    from yolosod_amd.nn.tasks import build_model
    return build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=cuda)


def test_model_matches_reference_golden(gpu_model, cuda):
    g = torch.Generator().manual_seed(0)
    x = torch.rand(2, 3, 256, 256, generator=g)
    with torch.inference_mode():
        y = gpu_model(x.to(cuda))[0].cpu()
    ok, msg = pred_close(y, torch.from_numpy(golden("model_out_256")["y"]))
    assert ok, msg


@pytest.mark.parametrize("split", [0, 1], ids=["exact_fp32_mfma", "f16_split"])
def test_model_matrix_methods_match_reference_golden(gpu_model, split, cuda):
    """The whole model with the Swin / head / A2 matrix products on exact fp32 MFMA (YOLOSOD_SWIN_X3 = HEAD_X2 =
    A2_X2 = 0) and as fp16 two-term splits (the default), each against the reference golden."""
    from yolosod_amd import _hip
    lib = _hip.load_library()
    g = torch.Generator().manual_seed(0)
    x = torch.rand(2, 3, 256, 256, generator=g)
    hooks = (lib.yolosod_debug_set_swin_x3, lib.yolosod_debug_set_head_x2, lib.yolosod_debug_set_a2_x2)
    for h in hooks:
        h(split)
    try:
        with torch.inference_mode():
            y = gpu_model(x.to(cuda))[0].cpu()
    finally:
        for h in hooks:
            h(1)
    ok, msg = pred_close(y, torch.from_numpy(golden("model_out_256")["y"]))
    assert ok, msg


def test_model_640_matches_oracle(gpu_model, cuda):
    from oracle.model_ref import build_cpu_model
    cpu = build_cpu_model()
    cpu.load_state_dict({k: v.cpu() for k, v in gpu_model.state_dict().items()})
    g = torch.Generator().manual_seed(1)
    x = torch.rand(1, 3, 640, 640, generator=g)
    with torch.inference_mode():
        y = gpu_model(x.to(cuda))[0].cpu()
        ref = cpu(x)[0]
    ok, msg = pred_close(y, ref)
    assert ok, msg


def test_model_640_matches_reference_checksums(gpu_model, cuda):
    """The reference's own fused fp32 forward at 640x640 (seed-0 weights, rand(2,3,640,640) seed 0), recorded by
    make_golden.py as checksums: per-row sums over both images (rows 4.. = sums of 68 000 class probabilities each,
    so a relative error of the class branch shows up 1:1), the total and the max score."""
    man = json.loads((GOLDEN / "model_manifest.json").read_text())["yolov12-sod-fusion-v5-simple"]["out_640"]
    x = torch.rand(2, 3, 640, 640, generator=torch.Generator().manual_seed(0))
    with torch.inference_mode():
        y = gpu_model(x.to(cuda))[0].double().cpu()
    assert list(y.shape) == man["shape"]
    rs = y.sum((0, 2))
    ref = torch.tensor(man["row_sums"], dtype=torch.float64)
    rel = ((rs - ref) / ref).abs()
    assert float(rel[:4].max()) <= 1e-6, rel[:4].tolist()  # 68 000 coordinates per row, each within 1e-3 abs
    assert float(rel[4:].max()) <= 2e-5, rel[4:].tolist()
    assert abs(float(y.sum()) - man["sum"]) <= 1e-6 * man["sum"]
    assert abs(float(y[:, 4:].max()) - man["max_score"]) <= 1e-4 * man["max_score"]


def test_predictor_bs32_vs_oracle(gpu_model, cuda):
    """BASELINE configs[1..2] batch (32 x 640x640): the batched GPU forward against the oracle CPU model on 4 of
    the 32 images (first, last and two inside), and the predictor's padded outputs."""
    from oracle.model_ref import build_cpu_model
    from yolosod_amd.engine.predictor import DetectionPredictor
    cpu = build_cpu_model()
    cpu.load_state_dict({k: v.cpu() for k, v in gpu_model.state_dict().items()})
    pred = DetectionPredictor(gpu_model, conf=0.0005, iou=0.7)
    g = torch.Generator().manual_seed(2)
    x = torch.rand(32, 3, 640, 640, generator=g)
    pick = [0, 9, 17, 31]
    with torch.inference_mode():
        y32 = gpu_model(x.to(cuda))[0].cpu()
        ref = cpu(x[pick])[0]
    ok, msg = pred_close(y32[pick], ref)
    assert ok, msg
    out, counts, index = pred.predict_padded(x.to(cuda))
    assert out.shape == (32, 300, 6) and counts.shape == (32,)
    assert int(counts.min()) >= 0 and int(counts.max()) <= 300


def test_scale_boxes_gpu_matches_reference(cuda):
    """a11: scale_boxes / clip_boxes (ops.py:92-128, 319-338) on GPU tensors, bit-exact on the reference's outputs
    (tests/golden/scale_boxes.npz: same-shape, letterboxed, explicit ratio_pad and xywh cases)."""
    from yolosod_amd.utils import ops
    z = golden("scale_boxes")
    cases = json.loads(str(z["cases"]))
    for i, (s1, s0, rp, pad, xywh) in enumerate(cases):
        b = torch.from_numpy(z["boxes"][i].copy()).to(cuda)
        got = ops.scale_boxes(s1, b, s0, ratio_pad=rp, padding=pad, xywh=xywh).cpu().numpy()
        assert np.array_equal(got, z["out"][i]), (i, np.abs(got - z["out"][i]).max())


def test_fused_head_equals_raw_map_path(gpu_model, cuda):
    """Detect on GPU: the fused head tail + decode kernel vs the reference-shaped path that materialises the raw
    [B, 64+nc, H, W] maps (MIOpen 1x1 convs + HIP bias epilogue + HIP decode)."""
    from yolosod_amd.nn.modules import Detect
    g = torch.Generator().manual_seed(3)
    x = torch.rand(2, 3, 640, 640, generator=g).to(cuda)
    with torch.inference_mode():
        y_fused = gpu_model(x)[0]
        Detect.keep_raw = True
        try:
            y_raw, raw = gpu_model(x)
        finally:
            Detect.keep_raw = False
    assert raw[0].shape == (2, 74, 160, 160)
    ok, msg = pred_close(y_fused.cpu(), y_raw.cpu(), ztol=1e-5)
    assert ok, msg


def test_fused_head_second_output_is_the_reference_raw_maps(gpu_model, cuda):
    """Detect's forward contract (head.py:69-74): the fused path's second output holds the raw [B, 64+nc, Hi, Wi]
    maps (computed from the kept tower features when first read), equal to the unfused path's list."""
    from yolosod_amd.nn.modules import Detect, RawMaps
    x = torch.rand(2, 3, 320, 320, generator=torch.Generator().manual_seed(8)).to(cuda)
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        with torch.inference_mode():
            _, lazy = gpu_model(x)
            Detect.keep_raw = True
            try:
                _, raw = gpu_model(x)
            finally:
                Detect.keep_raw = False
            assert isinstance(lazy, RawMaps) and isinstance(raw, list) and len(lazy) == len(raw) == 4
            maps = list(lazy)
            _, lazy_out = gpu_model(x)
        maps_out = list(lazy_out)  # first read after leaving inference_mode (the features are inference tensors)
    finally:
        torch.backends.cudnn.deterministic = det
    for a, b, c in zip(maps, raw, maps_out):
        assert a.shape == b.shape and a.shape[1] == 74
        assert torch.equal(a, b) and torch.equal(c, b)


def test_m_scale_model_matches_oracle(cuda):
    """yolov12m-sod (the paper YAML with v12's m scale; BASELINE configs[4] in fp32): Swin C=128 on the
    fused kernel, Swin C=512 and A2 C=512 on the GEMM path, Detect c3=128 on the fused head."""
    from oracle.model_ref import build_cpu_model
    from yolosod_amd.nn.tasks import build_model
    gm = build_model("yolov12m-sod.yaml", seed=0, device=cuda)
    cpu = build_cpu_model("yolov12m-sod.yaml")
    cpu.load_state_dict({k: v.cpu() for k, v in gm.state_dict().items()})
    g = torch.Generator().manual_seed(4)
    x = torch.rand(1, 3, 256, 256, generator=g)
    with torch.inference_mode():
        y = gm(x.to(cuda))[0].cpu()
        ref = cpu(x)[0]
    ok, msg = pred_close(y, ref)
    assert ok, msg


def test_model_1280_matches_oracle(gpu_model, cuda):
    """BASELINE configs[3] shape (1280x1280, P2 head at 320x320; Swin L28 on 2116 windows per image)."""
    from oracle.model_ref import build_cpu_model
    cpu = build_cpu_model()
    cpu.load_state_dict({k: v.cpu() for k, v in gpu_model.state_dict().items()})
    g = torch.Generator().manual_seed(5)
    x = torch.rand(1, 3, 1280, 1280, generator=g)
    with torch.inference_mode():
        y = gpu_model(x.to(cuda))[0].cpu()
        ref = cpu(x)[0]
    assert y.shape == (1, 14, 136000)
    ok, msg = pred_close(y, ref)
    assert ok, msg


def test_fusion_v5_model_matches_reference_and_oracle(cuda):
    """yolov12-sod-fusion-v5: the paper graph + MambaBlock (GLU fallback, HIP yolosod_mamba_glu_forward) at P3."""
    from oracle.model_ref import build_cpu_model
    from yolosod_amd.nn.tasks import build_model
    gm = build_model("yolov12-sod-fusion-v5.yaml", seed=0, device=cuda)
    g = torch.Generator().manual_seed(0)
    x = torch.rand(2, 3, 128, 128, generator=g)
    with torch.inference_mode():
        y = gm(x.to(cuda))[0].cpu()
    ok, msg = pred_close(y, torch.from_numpy(golden("model_v5_out_128")["y"]))
    assert ok, f"vs reference golden: {msg}"
    cpu = build_cpu_model("yolov12-sod-fusion-v5.yaml")
    cpu.load_state_dict({k: v.cpu() for k, v in gm.state_dict().items()})
    g = torch.Generator().manual_seed(1)
    x = torch.rand(2, 3, 640, 640, generator=g)
    with torch.inference_mode():
        y = gm(x.to(cuda))[0].cpu()
        ref = cpu(x)[0]
    ok, msg = pred_close(y, ref)
    assert ok, f"vs oracle at 640: {msg}"


def test_executor_streams_and_concat_elision_are_bit_identical(gpu_model, cuda):
    """The GPU executor's side-stream Detect towers (dealt to three side streams, or all on one) and concat elision
    move data and reorder launches only: the output equals the plain one-stream, torch.cat forward bit for bit
    (tasks.py _predict_once_planned).
    MIOpen's split-K conv solvers accumulate with atomics (run-to-run differences ~5e-5 in the backbone), so the
    comparison runs with torch.backends.cudnn.deterministic (every HIP kernel of this library is deterministic)."""
    from yolosod_amd.nn import tasks
    g = torch.Generator().manual_seed(5)
    x = torch.rand(4, 3, 320, 320, generator=g).to(cuda)
    saved, saved_side, saved_gf = tasks.STREAMS, tasks.SIDE_STREAMS, tasks.GATE_FUSE
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        with torch.inference_mode():
            tasks.GATE_FUSE = False  # the fused gate convs change the conv arithmetic (test_gate_fusion_...)
            tasks.STREAMS = 1
            y_streams = gpu_model(x)[0].clone()  # towers dealt to SIDE_STREAMS side streams
            assert gpu_model._last_elided == 6
            tasks.SIDE_STREAMS = 1
            y_side1 = gpu_model(x)[0].clone()
            tasks.STREAMS = 0
            y_one = gpu_model(x)[0].clone()
            gpu_model._fused = False  # plain executor: torch.cat, one stream
            try:
                y_plain = gpu_model(x)[0].clone()
            finally:
                gpu_model._fused = True
    finally:
        tasks.STREAMS, tasks.SIDE_STREAMS, tasks.GATE_FUSE = saved, saved_side, saved_gf
        torch.backends.cudnn.deterministic = det
    torch.cuda.synchronize()
    assert torch.equal(y_streams, y_side1)
    assert torch.equal(y_streams, y_one)
    assert torch.equal(y_one, y_plain)


def test_gate_fusion_matches_the_unfused_model(gpu_model, cuda):
    """SE L1 -> Conv L2 and CBAM L4 -> Conv L5 as gate-only launches + the stride-2 conv that applies the gate while
    staging (tasks.py GATE_FUSE, csrc/conv3x3s2.hip): the op_timer sees the fused operators instead of the SE / CBAM
    apply, and the model output matches the unfused executor (the gate's own apply pass, MIOpen conv) within fp32
    accuracy, at 320 and at 640 (Cout 64 and 128, one and two input chunks)."""
    from yolosod_amd import _hip
    from yolosod_amd.nn import tasks
    saved = tasks.GATE_FUSE
    for S in (320, 640):
        x = torch.rand(2, 3, S, S, generator=torch.Generator().manual_seed(S)).to(cuda)
        try:
            with torch.inference_mode():
                tasks.GATE_FUSE = True
                with _hip.op_timer() as t:
                    y1 = gpu_model(x)[0].clone()
                names = [k[0] for k, _ in t.durations_ms()]
                keys = set(names)
                tasks.GATE_FUSE = False
                y0 = gpu_model(x)[0].clone()
        finally:
            tasks.GATE_FUSE = saved
        assert {"se_gate", "se_conv", "cbam_gate", "cbam_conv"} <= keys, keys
        assert names.count("se") == 1 and names.count("cbam") == 1  # SE L23 and CBAM L18 keep their apply
        ok, e, _ = tol_close(y1.cpu().double(), y0.cpu().double(), 1e-3, 1e-4)
        assert ok, (S, e)


def test_neck_stride2_convs_take_the_kernel(gpu_model, cuda):
    """The neck's 3x3 / stride-2 convs (layers 29 / 33 / 36) run on the stride-2 fp16-split kernel, written into
    their Concat slices, and the model matches the MIOpen path (YOLOSOD_S2_NECK=0) within fp32 accuracy."""
    from yolosod_amd import _hip
    from yolosod_amd.nn import modules as M
    assert [i for i, m in enumerate(gpu_model.model) if getattr(m, "s2", False)] == [29, 33, 36]
    x = torch.rand(2, 3, 640, 640, generator=torch.Generator().manual_seed(7)).to(cuda)
    saved = M.S2_NECK
    try:
        with torch.inference_mode():
            M.S2_NECK = True
            with _hip.op_timer() as t:
                y1 = gpu_model(x)[0].clone()
            plain = [k for k, _ in t.durations_ms() if k[0] == "conv3x3s2" and k[2][1:] == (False, False)]
            M.S2_NECK = False
            y0 = gpu_model(x)[0].clone()
    finally:
        M.S2_NECK = saved
    assert sorted(k[2][0] for k in plain) == [128, 256, 512], plain
    ok, e, _ = tol_close(y1.cpu().double(), y0.cpu().double(), 1e-3, 1e-4)
    assert ok, e
