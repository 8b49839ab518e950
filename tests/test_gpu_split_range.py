"""GPU: range of the fp16 two-term split method (csrc/common.h split4; swin_x3.hip, detect.hip x2, gemm_f32.h X2).

An fp32 operand is split v = h + l with h = fp16(v), l = fp16(v - h). For |v| < 2^-3 the low term falls into
fp16's subnormal range, whose spacing is 2^-24, so the representation error has an absolute floor of 2^-25 per
element instead of fp32's 2^-24 |v| relative error. This test probes that floor where the
kernels split raw activations (everything downstream of a LayerNorm is unit-scale by construction): inputs scaled
by 1e-3, the regime SURVEY App. A.11 measures for random-init activations.

Bar, against the fp64 oracle: max |y - ref| <= 1e-4 max |ref| (the relative tolerance of the unit-scale tests), and
no accuracy lost to the split: the split path's error at most 1.5x that of the same operator on the exact fp32 MFMA
(+1e-7), so a floor that the split adds on top of fp32 rounding would show. The input-dependent part of the output,
max |ref(x) - ref(0)|, is logged beside them (measured: split and exact errors equal to within 10-20 % at every op,
far below the input-dependent signal at Swin, where the LayerNorms make the matrix operands unit-scale).
"""
import os

import pytest
import torch

import recipes
from oplib import build_fixture_module
from oracle import ops_ref as R
from oracle.model_ref import OP_CLASSES
from yolosod_amd import _hip

pytestmark = pytest.mark.gpu

SCALE = 1e-3
RTOL = 1e-4

OPS = {  # name: (op, args, shape, debug switch of the split method)
    "swin_L28": ("SwinBlock", (64, 2, 7), (1, 64, 160, 160), "yolosod_debug_set_swin_x3"),
    "swin_L9": ("SwinBlock", (256, 4, 7), (1, 256, 40, 40), "yolosod_debug_set_swin_x3"),
    "a2_L12": ("A2_Attn", (512, None, 8, 8), (2, 512, 20, 20), "yolosod_debug_set_a2_x2"),
}


def _log(msg):
    log = os.environ.get("YOLOSOD_PARITY_LOG")
    if log:
        with open(log, "a") as f:
            f.write(f"{os.environ.get('PYTEST_CURRENT_TEST', '?')}: {msg}\n")


def _check(err_split, err_exact, ref_max, signal, what):
    _log(f"{what}: split err {err_split:.3g}, exact fp32 err {err_exact:.3g}, max|ref| {ref_max:.3g}, "
         f"input-dependent signal {signal:.3g} (split err / signal {err_split / signal:.3g})")
    assert err_split <= RTOL * ref_max, (err_split, ref_max)
    assert err_split <= 1.5 * err_exact + 1e-7, (err_split, err_exact)


def _run(fn, switch, on):
    lib = _hip.load_library()
    getattr(lib, switch)(on)
    try:
        with torch.inference_mode():
            return fn().cpu().double()
    finally:
        getattr(lib, switch)(1)


@pytest.mark.parametrize("name", list(OPS))
def test_split_small_magnitude_ops(name, cuda, monkeypatch):
    op, args, shape, switch = OPS[name]
    monkeypatch.setitem(recipes.OPS, name, (op, args, shape))
    m, _ = build_fixture_module(name)
    x = recipes.make_input(name, shape) * SCALE
    ref_m, _ = build_fixture_module(name, OP_CLASSES)
    with torch.inference_mode():
        ref = ref_m.double()(x.double())
        ref0 = ref_m.double()(torch.zeros_like(x, dtype=torch.float64))
    signal = float((ref - ref0).abs().max())
    md = m.to(cuda)
    xd = x.to(cuda)
    err_split = float((_run(lambda: md(xd), switch, 1) - ref).abs().max())
    err_exact = float((_run(lambda: md(xd), switch, 0) - ref).abs().max())
    _check(err_split, err_exact, float(ref.abs().max()), signal, f"x*{SCALE}")


def test_split_small_magnitude_detect_head(cuda):
    """The Detect head's fused 1x1 convs split the tower features (raw activations) in registers."""
    g = torch.Generator().manual_seed(9)
    strides, nc, B, img = [4.0, 8.0, 16.0, 32.0], 10, 2, 256
    fb, fc, wb, bb, wc, bc = [], [], [], [], [], []
    for s in strides:
        h = int(img // s)
        fb.append(torch.randn(B, 64, h, h, generator=g) * SCALE)
        fc.append(torch.randn(B, 64, h, h, generator=g) * SCALE)
        wb.append(torch.randn(64, 64, generator=g) * 0.25)
        bb.append(torch.randn(64, generator=g))
        wc.append(torch.randn(nc, 64, generator=g) * 0.2)
        bc.append(torch.randn(nc, generator=g) - 2.0)

    def oracle(scale):
        maps = []
        for i in range(4):
            box = torch.einsum("ok,bkhw->bohw", wb[i].double(), fb[i].double() * scale) + bb[i].double().view(1, -1, 1, 1)
            cls = torch.einsum("ok,bkhw->bohw", wc[i].double(), fc[i].double() * scale) + bc[i].double().view(1, -1, 1, 1)
            maps.append(torch.cat([box, cls], 1))
        return R.decode_ref(maps, strides, nc)

    ref, ref0 = oracle(1.0), oracle(0.0)
    signal = float((ref - ref0).abs().max())
    d = lambda ts: [t.to(cuda) for t in ts]  # noqa: E731
    fn = lambda: _hip.detect_head(d(fb), d(fc), d(wb), d(bb), d(wc), d(bc), strides, nc)  # noqa: E731
    err_split = float((_run(fn, "yolosod_debug_set_head_x2", 1) - ref).abs().max())
    err_exact = float((_run(fn, "yolosod_debug_set_head_x2", 0) - ref).abs().max())
    _check(err_split, err_exact, float(ref.abs().max()), signal, f"features*{SCALE}")


def test_split_is_bitwise_fp16_pair(cuda):
    """common.h split2 (v_cvt_pk_f16_f32 + v_fma_mix{lo,hi}_f16) gives exactly h = fp16(v), l = fp16(v - h): normal,
    subnormal-low-term, tiny (subnormal h), large and overflowing magnitudes, both signs."""
    g = torch.Generator().manual_seed(3)
    mags = [1.0, 1e-3, 1e-5, 3e-8, 1e3, 6e4, 7e4]
    v = torch.cat([torch.randn(4096, generator=g) * m for m in mags] + [torch.tensor([0.0, -0.0, 65504.0, 65520.0,
                                                                                  2.0 ** -24, 2.0 ** -25])])
    v = v[: v.numel() // 2 * 2].contiguous()
    h = torch.empty(v.numel() // 2, dtype=torch.int32, device=cuda)
    lo = torch.empty_like(h)
    vd = v.to(cuda)
    lib = _hip.load_library()
    assert lib.yolosod_debug_split_f16(vd.data_ptr(), h.data_ptr(), lo.data_ptr(), h.numel(), None) == 0
    torch.cuda.synchronize()
    hh = h.cpu().view(torch.float16)
    ll = lo.cpu().view(torch.float16)
    ref_h = v.half()
    ref_l = (v - ref_h.float()).half()  # v - h is exact in fp32 (h finite)
    fin = torch.isfinite(ref_h)
    assert torch.equal(hh.view(torch.int16)[fin], ref_h.view(torch.int16)[fin])
    assert torch.equal(ll.view(torch.int16)[fin], ref_l.view(torch.int16)[fin])


@pytest.mark.parametrize("name", ["swin_L28", "swin_L9", "a2_L12"])
def test_split_range_guard_flags_and_exact_fallback(name, cuda, monkeypatch):
    """Operands beyond fp16's range set the split-range flag (instead of silent inf / NaN), and the exact-fp32 path
    the guard falls back to stays accurate; in-range work leaves it clear."""
    op, args, shape, _ = OPS[name]
    monkeypatch.setitem(recipes.OPS, name, (op, args, shape))
    m, _ = build_fixture_module(name)
    md = m.to(cuda)
    x = recipes.make_input(name, shape)
    _hip.split_range_flag(reset=True)
    with torch.inference_mode():
        md(x.to(cuda))
    assert not _hip.split_range_flag(reset=True)
    big = x * 1e5  # Swin: the residual stream (the pw product's operand) ~1e5; A2: the proj GEMM's input
    with torch.inference_mode():
        md(big.to(cuda))
    assert _hip.split_range_flag(reset=True)
    ref_m, _ = build_fixture_module(name, OP_CLASSES)
    with torch.inference_mode():
        ref = ref_m.double()(big.double())
        with _hip.exact_fp32_matrix():
            y = md(big.to(cuda)).cpu().double()
    assert float((y - ref).abs().max()) <= 1e-4 * float(ref.abs().max())
    if not name.startswith("swin"):
        return
    # weights beyond range (64 W > 65504): flagged by the weight preparation, and again by every later forward on the
    # cached prepared block (the block keeps the preparation's range word)
    with torch.no_grad():
        md.window_attn.mlp[2].weight.mul_(2e4)
    for _ in range(3):
        with torch.inference_mode():
            md(x.to(cuda))
        assert _hip.split_range_flag(reset=True)


@pytest.mark.parametrize("name", ["swin_L28", "swin_L9", "a2_L12"])
def test_split_range_guard_flags_nan(name, cuda, monkeypatch):
    """A NaN operand sets the flag: the running max is the NaN-propagating IEEE maximum (v_maximum3_f32)."""
    op, args, shape, _ = OPS[name]
    monkeypatch.setitem(recipes.OPS, name, (op, args, shape))
    m, _ = build_fixture_module(name)
    md = m.to(cuda)
    x = recipes.make_input(name, shape)
    x[0, 3, 5, 7] = float("nan")
    _hip.split_range_flag(reset=True)
    with torch.inference_mode():
        md(x.to(cuda))
    assert _hip.split_range_flag(reset=True)


def test_exact_fp32_matrix_restores_switches(cuda):
    """exact_fp32_matrix() restores each split switch to its previous state instead of forcing it on."""
    lib = _hip.load_library()
    prev = lib.yolosod_debug_set_head_x2(0)
    try:
        with _hip.exact_fp32_matrix():
            pass
        assert lib.yolosod_debug_set_head_x2(0) == 0  # still off after the context
    finally:
        lib.yolosod_debug_set_head_x2(prev)


def test_split_range_guard_detect_head(cuda):
    g = torch.Generator().manual_seed(4)
    strides, nc, B, img = [4.0, 8.0, 16.0, 32.0], 10, 1, 128
    mk = lambda *s: torch.randn(*s, generator=g).to(cuda)  # noqa: E731
    fb = [mk(B, 64, int(img // s), int(img // s)) for s in strides]
    fc = [mk(B, 64, int(img // s), int(img // s)) for s in strides]
    wb, bb = [mk(64, 64) * 0.1 for _ in strides], [mk(64) for _ in strides]
    wc, bc = [mk(nc, 64) * 0.1 for _ in strides], [mk(nc) for _ in strides]
    _hip.split_range_flag(reset=True)
    _hip.detect_head(fb, fc, wb, bb, wc, bc, strides, nc)
    assert not _hip.split_range_flag(reset=True)
    _hip.detect_head([f * 1e5 for f in fb], fc, wb, bb, wc, bc, strides, nc)
    assert _hip.split_range_flag(reset=True)
    fn = [f.clone() for f in fb]
    fn[1][0, 5, 2, 3] = float("nan")
    _hip.detect_head(fn, fc, wb, bb, wc, bc, strides, nc)
    assert _hip.split_range_flag(reset=True)


def test_sharded_predict_redoes_flagged_shard_on_exact_kernels(cuda):
    """engine.predictor.sharded_predict (the bench's N > 1 step) reads the split-range flag after the rank-local
    predict and redoes a flagged shard on the exact fp32 kernels before the exchange, as DetectionPredictor.__call__
    does: with out-of-range Swin weights (64 W > 65504, flagged by the cached prepared block on every forward) its
    detections equal the exact-fp32 run bit for bit. World size 1 over RCCL (one process, this GPU)."""
    import socket

    import torch.distributed as dist

    from yolosod_amd.engine.predictor import DetectionPredictor, seeded_images, sharded_predict
    from yolosod_amd.nn.tasks import build_model
    m = build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=cuda)
    with torch.no_grad():
        m.model[28].window_attn.mlp[2].weight.mul_(2e4)  # the P2 SwinBlock (C = 64)
    pred = DetectionPredictor(m, conf=0.001, iou=0.7, max_det=300)
    x = seeded_images(0, 2, 256, device=cuda)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=cuda)
    try:
        _hip.split_range_flag(reset=True)
        g_out, g_cnt, g_idx = sharded_predict(pred.predict_padded, 2, lambda lo, hi: x[lo:hi])
        assert not _hip.split_range_flag(reset=True)  # the guard consumed (and cleared) the flag
        with _hip.exact_fp32_matrix():
            r_out, r_cnt, r_idx = pred.predict_padded(x)
        _hip.split_range_flag(reset=True)
    finally:
        dist.destroy_process_group()
        torch.backends.cudnn.deterministic = det
    assert torch.isfinite(g_out).all()
    assert torch.equal(g_cnt, r_cnt) and torch.equal(g_idx, r_idx)
    assert torch.equal(g_out, r_out)


def test_split_range_cached_a2_block_rereports_long_sequence(cuda):
    """A2 with L = areas * W > 160 (the n1280 shape class) skips the fused attention kernel; the proj / pool kernel
    re-raises the cached prepared block's range word, so out-of-range proj weights flag every forward, not only the
    one that prepared the block."""
    from yolosod_amd.nn.modules import A2_Attn
    torch.manual_seed(3)
    m = A2_Attn(64, None, 8, 1).eval().to(cuda)
    x = torch.randn(1, 64, 40, 40, device=cuda)
    _hip.split_range_flag(reset=True)
    with torch.inference_mode():
        m(x)
    assert not _hip.split_range_flag(reset=True)
    with torch.no_grad():
        m.proj.conv.weight.mul_(4e4)  # 64 W beyond 65504
    for _ in range(3):
        with torch.inference_mode():
            m(x)
        assert _hip.split_range_flag(reset=True)


def _conv_target(m, which):
    """The first fused Conv of the model that the executor routes to an fp16-split conv kernel of kind ``which``:
    a Detect tower 3x3 (conv3x3), a neck C2f Bottleneck 3x3 (conv3x3, s1), a neck stride-2 3x3 (conv3x3s2, s2), a
    neck wide 1x1 (conv1x1x2, n1), or the SE / CBAM gate's consumer (gate-fused conv3x3s2)."""
    from yolosod_amd.nn import modules as M
    if which == "gate":
        plan = m._gate_consumers()
        return plan[min(plan)]
    return next(c for c in m.modules() if isinstance(c, M.Conv) and getattr(c, which))


@pytest.mark.parametrize("which", ["tower", "s1", "s2", "n1", "gate"])
def test_predictor_guard_recovers_out_of_range_conv_weights(which, cuda):
    """the fp16-split conv kernels report into the split-range flag, and the predictor's fallback
    (exact_fp32_matrix) must route them away too - to MIOpen + the exact epilogues - or the redone batch would run the
    same kernels and return inf / NaN. Weights of one conv scaled past fp16's range (64 W > 65504, flagged by the
    cached weight preparation on every forward): the guarded predict is finite and equals the exact run bit for bit."""
    from yolosod_amd.engine.predictor import DetectionPredictor, seeded_images
    from yolosod_amd.nn.tasks import build_model
    m = build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=cuda)
    pred = DetectionPredictor(m, conf=0.001, iou=0.7, max_det=300)
    conv = _conv_target(pred.model, which)
    with torch.no_grad():
        conv.conv.weight.mul_(4e4)
    x = seeded_images(0, 2, 256, device=cuda)
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        _hip.split_range_flag(reset=True)
        with torch.inference_mode():
            pred.predict_padded(x)
        assert _hip.split_range_flag(reset=True), which  # the split conv kernel saw its weights out of range
        with torch.inference_mode():
            g_out, g_cnt, g_idx = pred.predict_padded_guarded(x)
        assert not _hip.split_range_flag(reset=True)  # the guard consumed (and cleared) the flag
        with torch.inference_mode(), _hip.exact_fp32_matrix():
            r_out, r_cnt, r_idx = pred.predict_padded(x)
        assert not _hip.split_range_flag(reset=True), which  # nothing on the exact path splits
    finally:
        torch.backends.cudnn.deterministic = det
    assert torch.isfinite(g_out).all()
    assert torch.equal(g_cnt, r_cnt) and torch.equal(g_idx, r_idx) and torch.equal(g_out, r_out)
