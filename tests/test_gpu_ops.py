"""GPU parity of the HIP MAFN operators and Detect decode.

Every HIP output is compared with (a) the golden output of the reference module on the same inputs / parameters
(tests/golden, produced by the reference in fp32 on CPU) and (b) the oracle restatement evaluated in float64 on
the CPU. Tolerance: BASELINE.json north star, |y - ref| <= 1e-3 absolute (fp32), plus a relative 1e-4 check
against the fp64 oracle that keeps the test meaningful where outputs are large.
"""
import numpy as np
import pytest
import torch

import recipes
from conftest import golden
from oplib import build_fixture_module, tol_close
from yolosod_amd import _hip
from oracle import ops_ref as R
from oracle.model_ref import OP_CLASSES

pytestmark = pytest.mark.gpu

ATOL = 1e-3  # north-star fp32 tolerance


def _oracle64(name, x):
    m, _ = build_fixture_module(name, OP_CLASSES)
    with torch.inference_mode():
        return m.double()(x.double())


@pytest.mark.parametrize("name", list(recipes.OPS))
def test_op_matches_reference_fixture(name, cuda):
    z = golden(f"ops_{name}")
    m, sha = build_fixture_module(name)
    assert sha == str(z["params_sha256_unfused"])
    x = torch.from_numpy(z["x"])
    with torch.inference_mode():
        y = m.to(cuda)(x.to(cuda)).cpu()
    ok, err, _ = tol_close(y, torch.from_numpy(z["y"]), ATOL, 0.0)
    assert ok, f"{name}: max abs err vs reference {err:.3g}"
    y64 = _oracle64(name, x)
    ok, err, ratio = tol_close(y, y64, 5e-5, 1e-4)
    assert ok, f"{name}: vs fp64 oracle max abs err {err:.3g} (ratio {ratio:.2f})"


@pytest.mark.parametrize("x3", [0, 1], ids=["fp32_mfma", "f16x2_mfma"])
@pytest.mark.parametrize("name", [n for n in recipes.OPS if n.startswith("swin_c64") or n.startswith("swin_c256")])
def test_swin_kernels_match_reference_fixture(name, x3, cuda):
    """Both kinds of fused Swin kernel: the default ones (C = 64 and C = 256) that run every matrix product as fp16
    two-term splits on the fp16 matrix cores (csrc/swin_x3.hip: three exact products per fp32 product) and the
    exact-fp32-MFMA ones (csrc/swin_fused.hip, csrc/swin_wide.hip; YOLOSOD_SWIN_X3=0), all held to the fp32
    tolerances."""
    lib = _hip.load_library()
    z = golden(f"ops_{name}")
    m, _ = build_fixture_module(name)
    x = torch.from_numpy(z["x"])
    lib.yolosod_debug_set_swin_x3(x3)
    try:
        with torch.inference_mode():
            y = m.to(cuda)(x.to(cuda)).cpu()
    finally:
        lib.yolosod_debug_set_swin_x3(1)
    ok, err, _ = tol_close(y, torch.from_numpy(z["y"]), ATOL, 0.0)
    assert ok, f"{name}: max abs err vs reference {err:.3g}"
    ok, err, ratio = tol_close(y, _oracle64(name, x), 5e-5, 1e-4)
    assert ok, f"{name}: vs fp64 oracle max abs err {err:.3g} (ratio {ratio:.2f})"


# real-model shapes (one image; the batch dimension is exercised by the model tests)
REAL = {
    "se_L1": ("SE_Block", (64,), (1, 32, 320, 320)),
    "cbam_L4": ("CBAM_Block", (64, 128, 16), (1, 64, 160, 160)),
    "swin_L9": ("SwinBlock", (256, 4, 7), (1, 256, 40, 40)),
    "a2_L12": ("A2_Attn", (512, None, 8, 8), (2, 512, 20, 20)),
    "cbam_L18": ("CBAM_Block", (256, 512, 16), (1, 256, 40, 40)),
    "se_L23": ("SE_Block", (256,), (2, 128, 80, 80)),
    "swin_L28": ("SwinBlock", (64, 2, 7), (1, 64, 160, 160)),
    "ca_L32": ("CA_Block", (128, 256, 32), (2, 128, 80, 80)),
    "swin_L28_1280": ("SwinBlock", (64, 2, 7), (1, 64, 320, 320)),
    "a2_L12_1280": ("A2_Attn", (512, None, 8, 8), (1, 512, 40, 40)),
    "swin_L9_1280": ("SwinBlock", (256, 4, 7), (1, 256, 80, 80)),
    "swin_wide_pad_20x13": ("SwinBlock", (256, 4, 7), (2, 256, 20, 13)),  # bottom + right zero pad, fused wide
    "mamba_L7": ("MambaBlock", (128, 256, 2), (1, 128, 80, 80)),          # yolov12-sod-fusion-v5 L7
}


@pytest.mark.parametrize("name", list(REAL))
def test_op_real_shapes_vs_oracle(name, cuda, monkeypatch):
    monkeypatch.setitem(recipes.OPS, name, REAL[name])
    m, _ = build_fixture_module(name)
    x = recipes.make_input(name, REAL[name][2])
    with torch.inference_mode():
        y = m.to(cuda)(x.to(cuda)).cpu()
    ref = _oracle64(name, x)
    ok, err, ratio = tol_close(y, ref, ATOL, 0.0)
    assert ok, f"{name}: max abs err {err:.3g}"
    ok, err, ratio = tol_close(y, ref, 5e-5, 1e-4)
    assert ok, f"{name}: rel check max abs err {err:.3g} ratio {ratio:.2f}"


@pytest.mark.parametrize("name", ["swin_L28", "swin_L28_1280", "swin_L9", "swin_wide_pad_20x13"])
def test_swin_exact_fp32_kernels_real_shapes(name, cuda, monkeypatch):
    """The exact-fp32-MFMA Swin kernels (swin_fused.hip, swin_wide.hip; YOLOSOD_SWIN_X3=0) at the real shapes (the
    default fp16-split kernels run them in test_op_real_shapes_vs_oracle)."""
    lib = _hip.load_library()
    monkeypatch.setitem(recipes.OPS, name, REAL[name])
    m, _ = build_fixture_module(name)
    x = recipes.make_input(name, REAL[name][2])
    lib.yolosod_debug_set_swin_x3(0)
    try:
        with torch.inference_mode():
            y = m.to(cuda)(x.to(cuda)).cpu()
    finally:
        lib.yolosod_debug_set_swin_x3(1)
    ok, err, ratio = tol_close(y, _oracle64(name, x), 5e-5, 1e-4)
    assert ok, f"{name}: max abs err {err:.3g} ratio {ratio:.2f}"


C64_SHAPES = {  # C = 64 SwinBlocks through the fp16-split kernel (swin_x3_kernel<64, 2>)
    "swin_c64_h20": None, "swin_c64_h14": None, "swin_c64_h16x12": None,
    "swin_L28": REAL["swin_L28"],
    "swin_c64_b3_20x13": ("SwinBlock", (64, 2, 7), (3, 64, 20, 13)),  # cropped windows, several images
    "swin_c64_b5_9x7": ("SwinBlock", (64, 2, 7), (5, 64, 9, 7)),
}


@pytest.mark.parametrize("name", list(C64_SHAPES))
def test_swin_c64_fp16_split_kernel_shapes(name, cuda, monkeypatch):
    """The C = 64 fp16-split kernel against the fp64 oracle at the fp32 tolerances; shapes with cropped windows
    (20 x 13, 9 x 7), several images and the real L28 shape."""
    if C64_SHAPES[name] is not None:
        monkeypatch.setitem(recipes.OPS, name, C64_SHAPES[name])
    m, _ = build_fixture_module(name)
    x = recipes.make_input(name, recipes.OPS[name][2])
    with torch.inference_mode():
        y = m.to(cuda)(x.to(cuda)).cpu()
    ok, err, ratio = tol_close(y, _oracle64(name, x), 5e-5, 1e-4)
    assert ok, f"{name}: vs fp64 oracle max abs err {err:.3g} (ratio {ratio:.2f})"


A2_FUSED_SHAPES = {  # A2_Attn through both forms of its fp16-split path
    "a2_c512_h20": None, "a2_c128_h16": None,
    "a2_L12": REAL["a2_L12"],
    "a2_b3_c256_12x8": ("A2_Attn", (256, None, 8, 4), (3, 256, 12, 8)),   # L = 64, 96 pixels, 4 heads
    "a2_b2_c192_10x20": ("A2_Attn", (192, None, 4, 3), (2, 192, 10, 20)),  # 4 areas of 3 rows, overlapping bins
    "a2_L12_1280": REAL["a2_L12_1280"],  # L = 320: the decomposed path in both forms
}


@pytest.mark.parametrize("fused", [0, 1], ids=["decomposed", "fused"])
@pytest.mark.parametrize("name", list(A2_FUSED_SHAPES))
def test_a2_fused_and_decomposed_forms(name, fused, cuda, monkeypatch):
    """A2_Attn's split path as the fused kernels (a2_fused.hip: proj + SiLU + row pooling, then LN + QKV + attention
    per (image, head); the default) and as the decomposed GEMM path (yolosod_debug_set_a2_fused(0)), both with the
    token GEMM + upsample tail, against the fp64 oracle."""
    lib = _hip.load_library()
    if A2_FUSED_SHAPES[name] is not None:
        monkeypatch.setitem(recipes.OPS, name, A2_FUSED_SHAPES[name])
    m, _ = build_fixture_module(name)
    x = recipes.make_input(name, recipes.OPS[name][2])
    prev = lib.yolosod_debug_set_a2_fused(fused)
    try:
        with torch.inference_mode():
            y = m.to(cuda)(x.to(cuda)).cpu()
    finally:
        lib.yolosod_debug_set_a2_fused(prev)
    ok, err, ratio = tol_close(y, _oracle64(name, x), 5e-5, 1e-4)
    assert ok, f"{name} fused={fused}: vs fp64 oracle max abs err {err:.3g} (ratio {ratio:.2f})"


@pytest.mark.parametrize("name", ["a2_c512_h20", "a2_L12", "a2_b3_c256_12x8", "a2_b2_c192_10x20", "a2_L12_1280"])
def test_a2_proj_pool_area_groups_bit_identical(name, cuda, monkeypatch):
    """The proj + SiLU + pooling kernel over one tile per image (cap 400 pixels) and split into area groups (cap 208:
    two groups of 10 rows at 20x20; cap 100: four groups), and the wide kernel (128 / 256 output channels per
    workgroup, the default) compute every pixel with the same k order and MFMA operand layout, so the outputs are
    bit-identical. At 40x40 (n1280, L = 320: the decomposed attention after the fused proj / pool)
    the caps give 4 / 8 / 4 groups."""
    lib = _hip.load_library()
    if A2_FUSED_SHAPES[name] is not None:
        monkeypatch.setitem(recipes.OPS, name, A2_FUSED_SHAPES[name])
    m, _ = build_fixture_module(name)
    m = m.to(cuda)
    x = recipes.make_input(name, recipes.OPS[name][2]).to(cuda)
    prev = lib.yolosod_debug_set_a2_pool_px(400)
    prev_w = lib.yolosod_debug_set_a2_pool_wide(0)
    try:
        with torch.inference_mode():
            ys = [m(x).cpu()]
            for cap in (208, 100):
                lib.yolosod_debug_set_a2_pool_px(cap)
                ys.append(m(x).cpu())
            lib.yolosod_debug_set_a2_pool_wide(1)  # 128 / 256 channels per workgroup, its own area groups
            ys.append(m(x).cpu())
    finally:
        lib.yolosod_debug_set_a2_pool_px(prev)
        lib.yolosod_debug_set_a2_pool_wide(prev_w)
    for cap, y in zip((208, 100, "wide"), ys[1:]):
        assert torch.equal(ys[0], y), f"{name} cap {cap}: max|d| {float((ys[0] - y).abs().max()):.3g}"


@pytest.mark.parametrize("name,shape", [("se_c32_r64", (9, 32, 64, 64)), ("se_c64_r4_odd", (5, 64, 9, 7)),
                                        ("cbam_c64", (9, 64, 48, 40)), ("cbam_c32_odd", (5, 32, 13, 11)),
                                        ("ca_c128", (9, 128, 24, 20)), ("ca_c64_odd", (5, 64, 9, 7))])
def test_channel_ops_batch_invariant(name, shape, cuda):
    """Partial-reduction plans depend on the plane shape only, so a batch, its Infinity-Cache chunks and any
    shard of it give bitwise identical results."""
    m, _ = build_fixture_module(name)
    m = m.to(cuda)
    x = torch.randn(*shape, device=cuda)
    with torch.inference_mode():
        a = m(x)
        b = torch.cat([m(x[i:i + 1]) for i in range(shape[0])])
    assert torch.equal(a, b)


@pytest.mark.parametrize("M_,N,K,bkc", [(300, 192, 64, True), (1000, 64, 128, True), (129, 768, 256, True),
                                         (512, 400, 512, False), (64, 1600, 64, False), (130, 13, 32, True),
                                         (70, 150, 32, False)])
@pytest.mark.parametrize("x2", [0, 1], ids=["fp32_mfma", "f16x2_mfma"])
def test_gemm_f32(M_, N, K, bkc, x2, cuda):
    """Generic fp32 GEMM with the fused epilogue, on exact fp32 MFMA and as fp16 two-term split products."""
    from yolosod_amd import _hip
    g = torch.Generator().manual_seed(M_ * 7 + N)
    A = torch.randn(M_, K, generator=g)
    B = torch.randn(N, K, generator=g) if bkc else torch.randn(K, N, generator=g)
    bias = torch.randn(N, generator=g)
    res = torch.randn(M_, N, generator=g)
    ref = (A.double() @ (B.double().t() if bkc else B.double())) + bias.double()
    ref = torch.nn.functional.silu(ref) + res.double()
    lib = _hip.load_library()
    lib.yolosod_debug_set_gemm_x2(x2)
    try:
        C = _hip.gemm_f32(A.to(cuda), B.to(cuda), bkc, bias=bias.to(cuda), bias_mode=2, act=1,
                          res=res.to(cuda)).cpu()
    finally:
        lib.yolosod_debug_set_gemm_x2(0)
    ok, err, _ = tol_close(C, ref, 1e-4, 1e-5)
    assert ok, err


@pytest.mark.parametrize("L,C,heads", [(49, 64, 2), (49, 256, 4), (36, 64, 2), (160, 512, 8), (160, 64, 8),
                                        (320, 512, 8), (35, 64, 4), (7, 128, 1), (100, 256, 2)])
def test_attention(L, C, heads, cuda):
    from yolosod_amd import _hip
    nseq = 5
    g = torch.Generator().manual_seed(L * 31 + C)
    qkv = torch.randn(nseq * L, 3 * C, generator=g)
    q, k, v = qkv.double().view(nseq, L, 3, heads, C // heads).permute(2, 0, 3, 1, 4)
    p = torch.softmax(q @ k.transpose(-1, -2) / (C // heads) ** 0.5, -1)
    ref = (p @ v).transpose(1, 2).reshape(nseq * L, C)
    out = _hip.attention(qkv.to(cuda), nseq, L, C, heads).cpu()
    ok, err, _ = tol_close(out, ref, 1e-5, 1e-4)
    assert ok, err


@pytest.mark.parametrize("C", [64, 256, 512, 1000])
def test_layernorm(C, cuda):
    from yolosod_amd import _hip
    x = torch.randn(333, C) * 3 + 1
    w, b = torch.randn(C), torch.randn(C)
    ref = torch.nn.functional.layer_norm(x.double(), (C,), w.double(), b.double(), 1e-5)
    y = _hip.layernorm(x.to(cuda), w.to(cuda), b.to(cuda), 1e-5).cpu()
    ok, err, _ = tol_close(y, ref, 1e-5, 1e-5)
    assert ok, err


def test_decode_matches_reference_fixture(cuda):
    from yolosod_amd import _hip
    z = golden("decode_128")
    maps = [torch.from_numpy(z[f"map{i}"]).to(cuda) for i in range(4)]
    y = _hip.detect_decode(maps, recipes.DECODE["strides"], recipes.DECODE["nc"]).cpu()
    ok, err, _ = tol_close(y, torch.from_numpy(z["y"]), ATOL, 0.0)
    assert ok, err
    # the reference's own fp32 decode is 1.2e-4 from fp64 here (x2 - x1 cancellation); allow 2x that
    y64 = R.decode_ref([m.cpu().double() for m in maps], recipes.DECODE["strides"], recipes.DECODE["nc"])
    ok, err, _ = tol_close(y, y64, 2.5e-4, 0.0)
    assert ok, err


def test_decode_real_shapes(cuda):
    from yolosod_amd import _hip
    g = torch.Generator().manual_seed(5)
    maps = [torch.randn(2, 74, s, s, generator=g) * 3 for s in (160, 80, 40, 20)]
    y = _hip.detect_decode([m.to(cuda) for m in maps], [4.0, 8.0, 16.0, 32.0], 10).cpu()
    ref = R.decode_ref([m.double() for m in maps], [4.0, 8.0, 16.0, 32.0], 10)
    assert y.shape == (2, 14, 34000)
    ok, err, _ = tol_close(y, ref, ATOL, 0.0)
    assert ok, err


@pytest.mark.parametrize("B,Cin,Cout,H,W,act,res", [(2, 64, 64, 40, 40, 1, True), (3, 96, 256, 20, 20, 1, False),
                                                     (2, 1024, 512, 20, 20, 1, False), (1, 64, 10, 16, 16, 0, False),
                                                     (2, 128, 32, 80, 80, 1, True)])
def test_conv1x1_epilogue(B, Cin, Cout, H, W, act, res, cuda):
    """Backbone 1x1 conv as fused GEMM: act(conv(x) + b) (+ res), written into a channel slice."""
    from yolosod_amd import _hip
    g = torch.Generator().manual_seed(Cin + Cout)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, generator=g) / Cin ** 0.5
    b = torch.randn(Cout, generator=g)
    r = torch.randn(B, Cout, H, W, generator=g) if res else None
    ref = torch.nn.functional.conv2d(x.double(), w.double().view(Cout, Cin, 1, 1), b.double())
    ref = torch.nn.functional.silu(ref) if act else ref
    if res:
        ref = ref + r.double()
    buf = torch.zeros(B, Cout + 8, H, W, device=cuda)  # write into a channel slice of a concat buffer
    out = _hip.conv1x1(x.to(cuda), w.to(cuda), b.to(cuda), act, out=buf[:, 4:4 + Cout],
                       res=None if r is None else r.to(cuda))
    ok, err, _ = tol_close(out.cpu(), ref, 1e-4, 1e-5)
    assert ok, err
    assert float(buf[:, :4].abs().max()) == 0.0 and float(buf[:, 4 + Cout:].abs().max()) == 0.0


def test_bias_act_slice(cuda):
    from yolosod_amd import _hip
    y = torch.randn(2, 16, 12, 12)
    b = torch.randn(16)
    r = torch.randn(2, 16, 12, 12)
    buf = torch.zeros(2, 40, 12, 12, device=cuda)
    out = _hip.bias_act(y.to(cuda), b.to(cuda), 1, out=buf[:, 8:24], res=r.to(cuda))
    ref = torch.nn.functional.silu(y.double() + b.double().view(1, -1, 1, 1)) + r.double()
    ok, err, _ = tol_close(out.cpu(), ref, 1e-5, 1e-6)
    assert ok, err


@pytest.mark.parametrize("B,Cin,Cout,H,W,res,dual", [(2, 96, 64, 32, 40, False, False), (3, 256, 128, 16, 16, True, False),
                                                     (2, 64, 64, 8, 24, True, True), (1, 192, 128, 40, 40, False, True),
                                                     (2, 128, 64, 80, 80, False, False)])
def test_conv1x1_thin(B, Cin, Cout, H, W, res, dual, cuda):
    """yolosod_conv1x1_thin: SiLU(conv1x1(x) + b) (+ res) vs fp64, from / into channel slices, dual store."""
    from yolosod_amd import _hip
    g = torch.Generator().manual_seed(Cin * 7 + Cout + H)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, generator=g) / Cin ** 0.5
    b = torch.randn(Cout, generator=g)
    r = torch.randn(B, Cout, H, W, generator=g) if res else None
    ref = torch.nn.functional.silu(torch.nn.functional.conv2d(x.double(), w.double().view(Cout, Cin, 1, 1), b.double()))
    if res:
        ref = ref + r.double()
    xin = torch.zeros(B, Cin + 4, H, W, device=cuda)
    xin[:, 4:] = x.to(cuda)
    buf = torch.zeros(B, Cout + 8, H, W, device=cuda)
    c2lo = Cout // 2
    out2 = torch.full((B, Cout - c2lo, H, W), float("nan"), device=cuda) if dual else None
    out = _hip.conv1x1_thin(xin[:, 4:], w.to(cuda), b.to(cuda), out=buf[:, 4:4 + Cout],
                            res=None if r is None else r.to(cuda), out2=out2, c2lo=c2lo)
    ok, err, _ = tol_close(out.cpu(), ref, 1e-4, 1e-5)
    assert ok, err
    assert float(buf[:, :4].abs().max()) == 0.0 and float(buf[:, 4 + Cout:].abs().max()) == 0.0
    if dual:
        assert torch.equal(out2, out[:, c2lo:])


@pytest.mark.parametrize("c2lo,res", [(8, False), (0, True), (15, True)])
def test_bias_act_dual_store(c2lo, res, cuda):
    """yolosod_bias_act_dual: the slice store equals yolosod_bias_act bit for bit and out2 holds channels
    [c2lo, C) of it packed (C2f's Bottleneck inputs)."""
    from yolosod_amd import _hip
    g = torch.Generator().manual_seed(c2lo)
    y = torch.randn(3, 16, 10, 12, generator=g).to(cuda)
    b = torch.randn(16, generator=g).to(cuda)
    r = torch.randn(3, 16, 10, 12, generator=g).to(cuda) if res else None
    buf = torch.zeros(3, 40, 10, 12, device=cuda)
    out2 = torch.full((3, 16 - c2lo, 10, 12), float("nan"), device=cuda)
    out = _hip.bias_act(y, b, 1, out=buf[:, 8:24], res=r, out2=out2, c2lo=c2lo)
    ref = _hip.bias_act(y, b, 1, out=torch.empty_like(y), res=r)
    assert torch.equal(out, ref)
    assert torch.equal(out2, ref[:, c2lo:])
    assert float(buf[:, :8].abs().max()) == 0.0 and float(buf[:, 24:].abs().max()) == 0.0


@pytest.mark.parametrize("x2", [1, 0], ids=["f16x2_mfma", "fp32_mfma"])
@pytest.mark.parametrize("c3,img", [(64, 256), (128, 192), (64, 200)])
def test_detect_head_fused_vs_oracle(c3, img, x2, cuda):
    """Fused last 1x1 convs + decode vs the fp64 oracle (1x1 convs then decode_ref, head.py:70,100-131), with the
    convs as fp16 two-term splits on the fp16 matrix cores (default) and on the exact fp32 MFMA."""
    g = torch.Generator().manual_seed(c3 + img)
    strides, nc, B = [4.0, 8.0, 16.0, 32.0], 10, 2
    fb, fc, wb, bb, wc, bc, maps = [], [], [], [], [], [], []
    for s in strides:
        h = w = int(img // s)
        fb.append(torch.randn(B, 64, h, w, generator=g))
        fc.append(torch.randn(B, c3, h, w, generator=g))
        wb.append(torch.randn(64, 64, generator=g) * 0.25)
        bb.append(torch.randn(64, generator=g))
        wc.append(torch.randn(nc, c3, generator=g) * 0.2)
        bc.append(torch.randn(nc, generator=g) - 2.0)
        box = torch.einsum("ok,bkhw->bohw", wb[-1].double(), fb[-1].double()) + bb[-1].double().view(1, -1, 1, 1)
        cls = torch.einsum("ok,bkhw->bohw", wc[-1].double(), fc[-1].double()) + bc[-1].double().view(1, -1, 1, 1)
        maps.append(torch.cat([box, cls], 1))
    ref = R.decode_ref(maps, strides, nc)
    d = lambda ts: [t.to(cuda) for t in ts]  # noqa: E731
    lib = _hip.load_library()
    lib.yolosod_debug_set_head_x2(x2)
    try:
        y = _hip.detect_head(d(fb), d(fc), d(wb), d(bb), d(wc), d(bc), strides, nc).cpu()
    finally:
        lib.yolosod_debug_set_head_x2(1)
    ok, err, _ = tol_close(y, ref, 5e-4, 1e-5)
    assert ok, f"max abs err {err:.3g}"


@pytest.mark.parametrize("bf16", [False, True], ids=["fp32", "bf16"])
def test_detect_head_level_ranges_bit_identical(bf16, cuda):
    """detect_head_into (levels [l0, l1) into y laid out for all levels, the executor's split head) over a partition
    of the levels equals the one-launch head bit for bit, and leaves the other levels' slices of y untouched."""
    g = torch.Generator().manual_seed(11)
    strides, nc, B = [4.0, 8.0, 16.0, 32.0], 10, 2
    dt = torch.bfloat16 if bf16 else torch.float32
    fb = [torch.randn(B, 64, int(256 // s), int(256 // s), generator=g).to(cuda, dt) for s in strides]
    fc = [torch.randn(B, 64, int(256 // s), int(256 // s), generator=g).to(cuda, dt) for s in strides]
    wb = [(torch.randn(64, 64, generator=g) * 0.25).to(cuda) for _ in strides]
    bb = [torch.randn(64, generator=g).to(cuda) for _ in strides]
    wc = [(torch.randn(nc, 64, generator=g) * 0.2).to(cuda) for _ in strides]
    bc = [(torch.randn(nc, generator=g) - 2.0).to(cuda) for _ in strides]
    args = (fb, fc, wb, bb, wc, bc, strides, nc)
    y1 = _hip.detect_head(*args)
    offs = [0]
    for t in fb:
        offs.append(offs[-1] + t.shape[2] * t.shape[3])
    for parts in ([(0, 3), (3, 4)], [(0, 1), (1, 2), (2, 4)]):
        y = torch.full_like(y1, float("nan"))
        for l0, l1 in parts[:-1]:
            _hip.detect_head_into(y, l0, l1, *args)
        assert torch.isnan(y[..., offs[parts[-1][0]]:]).all()  # the last range not written yet
        _hip.detect_head_into(y, *parts[-1], *args)
        assert torch.equal(y, y1), parts


@pytest.mark.parametrize("name", [n for n in recipes.OPS if n.startswith("a2_")])
def test_a2_exact_fp32_gemms_match_reference_fixture(name, cuda):
    """A2_Attn with its GEMMs on exact fp32 MFMA (YOLOSOD_A2_X2=0); the default fp16-split GEMMs run the same
    fixtures in test_op_matches_reference_fixture."""
    lib = _hip.load_library()
    z = golden(f"ops_{name}")
    m, _ = build_fixture_module(name)
    x = torch.from_numpy(z["x"])
    lib.yolosod_debug_set_a2_x2(0)
    try:
        with torch.inference_mode():
            y = m.to(cuda)(x.to(cuda)).cpu()
    finally:
        lib.yolosod_debug_set_a2_x2(1)
    ok, err, _ = tol_close(y, torch.from_numpy(z["y"]), ATOL, 0.0)
    assert ok, f"{name}: max abs err vs reference {err:.3g}"
    ok, err, ratio = tol_close(y, _oracle64(name, x), 5e-5, 1e-4)
    assert ok, f"{name}: vs fp64 oracle max abs err {err:.3g} (ratio {ratio:.2f})"


@pytest.mark.parametrize("name", [n for n in recipes.OPS if n.startswith("a2_")])
def test_a2_premultiplied_out_projection_matches_two_gemm_form(name, cuda):
    """A2_Attn folds the MHA out-projection into the output conv (Wconv @ Wmha, one token GEMM); the C-ABI's
    two-GEMM form (attention.out_proj passed separately) must give the same output and both match the reference."""
    from yolosod_amd.nn.modules import conv_weight_bias
    z = golden(f"ops_{name}")
    m, _ = build_fixture_module(name)
    m = m.to(cuda).eval()
    x = torch.from_numpy(z["x"]).to(cuda)
    at = m.attention
    with torch.inference_mode():
        y1 = m(x)
        pw, pb = conv_weight_bias(m.proj)
        ow, ob = conv_weight_bias(m.out_proj)
        y2 = _hip.a2_forward(x, m.num_areas, m.num_heads, pw, pb, m.layer_norm.weight, m.layer_norm.bias,
                             m.layer_norm.eps, at.in_proj_weight, at.in_proj_bias, at.out_proj.weight,
                             at.out_proj.bias, ow, ob)
    ok, err, _ = tol_close(y1.cpu(), y2.cpu(), 1e-5, 1e-5)
    assert ok, f"premultiplied vs two-GEMM: {err:.3g}"
    for y in (y1, y2):
        ok, err, _ = tol_close(y.cpu(), torch.from_numpy(z["y"]), ATOL, 0.0)
        assert ok, f"{name}: max abs err vs reference {err:.3g}"


@pytest.mark.parametrize("shape,res", [((2, 128, 80, 80), False), ((3, 64, 20, 16), True), ((2, 32, 13, 12), False),
                                       ((1, 16, 200, 48), True)])
def test_producer_epilogue_pool_feeds_ca(shape, res, cuda):
    """bias_act(stats="capool") writes the same output as bias_act plus CA's row / column means, and CA_Block run on
    it (gate + apply only) equals the self-contained CA (up to summation order)."""
    from yolosod_amd.nn import modules as M
    g = torch.Generator().manual_seed(11)
    y = torch.randn(shape, generator=g).to(cuda)
    bias = torch.randn(shape[1], generator=g).to(cuda)
    r = torch.randn(shape, generator=g).to(cuda) if res else None
    plain = _hip.bias_act(y.clone(), bias, 1, res=r)
    pooled = _hip.bias_act(y.clone(), bias, 1, res=r, stats="capool")
    assert torch.equal(plain, pooled) and pooled._ys_ca_pool is not None
    yin = pooled._ys_ca_pool[0].cpu().double()
    ref = torch.cat([plain.double().mean(3), plain.double().mean(2)], 2).cpu()
    ok, err, _ = tol_close(yin, ref, 1e-5, 1e-5)
    assert ok, f"pooled means: {err:.3g}"
    m = M.CA_Block(shape[1], None, 32)
    recipes.perturb_(m, 5)
    m.to(cuda).eval()
    with torch.inference_mode():
        a = m(plain)
        b = m(pooled)
    ok, err, _ = tol_close(b.cpu(), a.cpu(), 1e-6, 1e-5)
    assert ok, f"CA with producer pooling vs self-contained: {err:.3g}"


@pytest.mark.parametrize("shape", [(2, 32, 40, 40), (3, 64, 96, 120), (2, 128, 20, 20)])
def test_producer_epilogue_stats_feed_se_and_cbam(shape, cuda):
    """bias_act(stats=...) writes the same output as bias_act and per-plane partials that make SE / CBAM skip
    their statistics pass; results equal the self-contained path (up to summation order)."""
    from yolosod_amd import _hip
    from yolosod_amd.nn import modules as M
    g = torch.Generator().manual_seed(7)
    y = torch.randn(shape, generator=g).to(cuda)
    bias = torch.randn(shape[1], generator=g).to(cuda)
    plain = _hip.bias_act(y.clone(), bias, 1)
    with_stats = _hip.bias_act(y.clone(), bias, 1, stats="summax")
    assert torch.equal(plain, with_stats) and with_stats._ys_plane_stats is not None
    se = M.SE_Block(4)
    se._maybe_build(shape[1], None)
    cb = M.CBAM_Block(shape[1], None, 4)
    for m in (se, cb):
        recipes.perturb_(m, 3)
        m.to(cuda).eval()
        with torch.inference_mode():
            a = m(plain)            # statistics pass over x
            b = m(with_stats)       # partials from the producer
        ok, err, _ = tol_close(b.cpu(), a.cpu(), 1e-6, 1e-5)
        assert ok, (type(m).__name__, err)


@pytest.mark.parametrize("B,Cin,H,W,stats", [(2, 96, 40, 40, "summax"), (3, 64, 16, 24, "sum"), (2, 256, 8, 8, "summax")])
def test_conv1x1_thin_stats_feed_se_and_cbam(B, Cin, H, W, stats, cuda):
    """yolosod_conv1x1_thin_stats: same output as yolosod_conv1x1_thin and plane statistics that SE / CBAM take
    instead of their own statistics pass (equal up to summation order)."""
    from yolosod_amd import _hip
    from yolosod_amd.nn import modules as M
    g = torch.Generator().manual_seed(Cin + H)
    x = torch.randn(B, Cin, H, W, generator=g).to(cuda)
    w = (torch.randn(64, Cin, generator=g) / Cin ** 0.5).to(cuda)
    b = torch.randn(64, generator=g).to(cuda)
    plain = _hip.conv1x1_thin(x, w, b)
    with_stats = _hip.conv1x1_thin(x, w, b, stats=stats)
    assert torch.equal(plain, with_stats) and with_stats._ys_plane_stats is not None
    mods = [M.CBAM_Block(64, None, 4)] if stats == "summax" else []
    if stats == "sum":
        se = M.SE_Block(16)
        se._maybe_build(64, None)
        mods.append(se)
    for m in mods:
        recipes.perturb_(m, 3)
        m.to(cuda).eval()
        with torch.inference_mode():
            a = m(plain)
            c = m(with_stats)
        ok, err, _ = tol_close(c.cpu(), a.cpu(), 1e-6, 1e-5)
        assert ok, (type(m).__name__, err)


@pytest.mark.parametrize("name", ["swin_L28", "swin_L9"])
def test_swin_prepared_parameters_cached_and_refreshed(name, cuda, monkeypatch):
    """SwinBlock caches the fp16-split kernels' weight split across calls (swin_prep / swin_fwd_prepared): the
    prepared call is bitwise the per-call-prepared one (same kernels), it is made once, and an in-place parameter
    update (version bump) rebuilds it."""
    from yolosod_amd import _hip
    monkeypatch.setitem(recipes.OPS, name, REAL[name])
    m, _ = build_fixture_module(name)
    m = m.to(cuda)
    x = recipes.make_input(name, REAL[name][2]).to(cuda)
    wa = m.window_attn
    with torch.inference_mode():
        y1 = m(x)
        prep1 = m._ys_cache["x3prep"][1]
        y2 = m(x)
        assert m._ys_cache["x3prep"][1] is prep1  # cached, not rebuilt
        ref = _hip.swin_forward(  # unprepared entry point: the split done inside the call
            x, wa.attn.num_heads, wa.window_size, m.dw.weight, wa.norm1.weight, wa.norm1.bias, wa.norm1.eps,
            wa.attn.in_proj_weight, wa.attn.in_proj_bias, wa.attn.out_proj.weight, wa.attn.out_proj.bias,
            wa.norm2.weight, wa.norm2.bias, wa.norm2.eps, wa.mlp[0].weight, wa.mlp[0].bias, wa.mlp[2].weight,
            wa.mlp[2].bias, m.pw.weight, m.bn.weight, m.bn.bias, m.bn.running_mean, m.bn.running_var, m.bn.eps)
    assert torch.equal(y1, y2) and torch.equal(y1, ref)
    with torch.no_grad():
        wa.mlp[2].weight.mul_(1.5)
    with torch.inference_mode():
        y3 = m(x)
        assert m._ys_cache["x3prep"][1] is not prep1
        ref3 = _hip.swin_forward(
            x, wa.attn.num_heads, wa.window_size, m.dw.weight, wa.norm1.weight, wa.norm1.bias, wa.norm1.eps,
            wa.attn.in_proj_weight, wa.attn.in_proj_bias, wa.attn.out_proj.weight, wa.attn.out_proj.bias,
            wa.norm2.weight, wa.norm2.bias, wa.norm2.eps, wa.mlp[0].weight, wa.mlp[0].bias, wa.mlp[2].weight,
            wa.mlp[2].bias, m.pw.weight, m.bn.weight, m.bn.bias, m.bn.running_mean, m.bn.running_var, m.bn.eps)
    assert torch.equal(y3, ref3) and not torch.equal(y3, y1)


@pytest.mark.parametrize("shape", [(2, 16, 20, 20), (1, 8, 7, 13), (3, 4, 40, 40), (1, 2, 1, 5), (2, 3, 64, 64)])
def test_sppf_pool_matches_chained_max_pools(shape, cuda):
    """yolosod_sppf_pool = three chained F.max_pool2d(5, 1, 2) (block.py SPPF) bit for bit, into a batch-strided
    concat buffer; channels [0, C) untouched."""
    import torch.nn.functional as F
    B, C, H, W = shape
    g = torch.Generator().manual_seed(B * 1000 + C * 10 + H)
    big = torch.randn(B, 4 * C + 3, H, W, generator=g).to(cuda)
    z = big[:, 3:]
    y0 = z[:, :C].clone()
    _hip.sppf_pool(z, C)
    p1 = F.max_pool2d(y0, 5, 1, 2)
    p2 = F.max_pool2d(p1, 5, 1, 2)
    p3 = F.max_pool2d(p2, 5, 1, 2)
    assert torch.equal(z[:, :C], y0)
    assert torch.equal(z[:, C:2 * C], p1) and torch.equal(z[:, 2 * C:3 * C], p2) and torch.equal(z[:, 3 * C:], p3)


def test_sppf_pool_propagates_nan(cuda):
    """A NaN activation reaches every pooled output whose window holds it, as in the chained F.max_pool2d (ADVICE r05:
    fmaxf would mask it)."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(7)
    z = torch.randn(2, 4 * 5, 20, 20, generator=g)
    z[0, 1, 3, 4] = float("nan")
    z[1, 4, 19, 0] = float("nan")
    z[1, 2, 10, 10] = float("inf")
    z = z.to(cuda)
    y0 = z[:, :5].clone()
    _hip.sppf_pool(z, 5)
    p1 = F.max_pool2d(y0, 5, 1, 2)
    p2 = F.max_pool2d(p1, 5, 1, 2)
    p3 = F.max_pool2d(p2, 5, 1, 2)
    for k, p in enumerate((p1, p2, p3), 1):
        out = z[:, k * 5:(k + 1) * 5]
        assert torch.equal(torch.isnan(out), torch.isnan(p)) and bool(torch.isnan(p).any())
        assert torch.equal(torch.nan_to_num(out, nan=0.0), torch.nan_to_num(p, nan=0.0))
