"""Analytic cost model of the hot-path operators: algorithmic HBM bytes and FLOPs per call.

Bytes count compulsory traffic only - each activation tensor read once and written once, weights once; FLOPs
count multiply-adds as 2. These are the numerators of ``roofline.achieved`` in bench.py.
"""
from __future__ import annotations

import os

F32 = 4

# MI355X peaks (MI355X_MICROARCH.md "Chip-level parameters" / "Matrix cores"): dense, no sparsity
PEAK_HBM_GBS = 8000.0
PEAK_FP32_MFMA_TFLOPS = 157.3
PEAK_BF16_MFMA_TFLOPS = 2516.6  # 16x the f32 MFMA rate per clock (256 CUs x 4 SIMDs x 1024 flop/clk x 2.4 GHz)


def elem_size(key) -> int:
    """Bytes per activation element of a recorded launch: keys of bf16 launches carry a 4th element 2."""
    return key[3] if len(key) > 3 else F32


def peak_tflops(key) -> float:
    """Matrix-core peak of the arithmetic the launch runs: bf16 MFMA for bf16 activations, fp32 MFMA otherwise."""
    return PEAK_BF16_MFMA_TFLOPS if elem_size(key) == 2 else PEAK_FP32_MFMA_TFLOPS


def _on(name: str) -> bool:
    return os.environ.get(name, "1") != "0"


def method_peak_tflops(key) -> float:
    """Matrix-core ceiling of the METHOD an fp32 launch runs its matrix products with: the fp32 Swin (C 64 / 256),
    A2 and head kernels compute each fp32 product as 3 fp16 MFMA products of two-term splits (csrc/swin_x3.hip,
    gemm_f32.h X2, detect_head_x2_kernel), so their ceiling is the fp16 peak / 3; everything else keeps
    peak_tflops. bench.py quotes every roofline fraction against this ceiling (the roof the kernel actually runs
    on); the fraction of the dtype's peak is reported beside it as a secondary field."""
    if elem_size(key) == 4:
        op = key[0]
        split = ((op == "swin" and key[1][1] in (64, 256) and _on("YOLOSOD_SWIN_X3"))
                 or (op == "a2" and _on("YOLOSOD_A2_X2")) or (op == "head" and _on("YOLOSOD_HEAD_X2")))
        if split:
            return PEAK_BF16_MFMA_TFLOPS / 3
    return peak_tflops(key)


# operators of the SURVEY 8(a) path (rooflined); other keys the op_timer records are backbone conv kernels
PATH_OPS = frozenset({"se", "cbam", "ca", "a2", "swin", "mamba", "decode", "head", "nms"})


def swin_geom(H, W, ws=7):
    if H <= ws and W <= ws:
        return H, W, H, W
    wh, ww = min(ws, H), min(ws, W)
    return wh, ww, H + (wh - H % wh) % wh, W + (ww - W % ww) % ww


def op_cost(key):
    """key = (op, shape, extra[, elem bytes]) as recorded by yolosod_amd._hip.op_timer -> (bytes, flops).
    Activations count at the launch's element size (2 for the bf16 config), parameters at 4 bytes."""
    b, f = _op_cost(key[:3], elem_size(key))
    return b, f


def _op_cost(key, E):
    op, shape, extra = key
    if op in ("se", "cbam", "ca"):
        B, C, H, W = shape
        hid = extra
        act = 2 * B * C * H * W * E
        w = (2 * C * hid + C + hid) * F32
        flops = B * C * H * W * (2 if op == "se" else 6)
        return act + w, flops
    if op == "a2":
        B, C, H, W = shape
        A, heads = extra
        L = A * W
        act = 2 * B * C * H * W * E
        w = (2 * (C * C + C) + 4 * C * C + 4 * C + 2 * C) * F32
        conv = 2 * 2 * C * C * H * W  # proj + out_proj (1x1 convs on the full map)
        mha = 2 * L * C * 3 * C + 2 * L * C * C + 2 * 2 * L * L * C
        return act + w, B * (conv + mha)
    if op == "swin":
        B, C, H, W = shape
        heads, ws, hid = extra
        wh, ww, Hp, Wp = swin_geom(H, W, ws)
        L = wh * ww
        tok_p = Hp * Wp
        act = 2 * B * C * H * W * E
        w = (9 * C + 4 * C * C + 3 * C + C + 2 * C * hid + hid + C + C * C + 6 * C) * F32
        dense = tok_p * (2 * C * 3 * C + 2 * C * C + 2 * 2 * C * hid) + H * W * 2 * C * C
        attn = tok_p * 2 * 2 * L * C
        dw = H * W * 2 * 9 * C
        return act + w, B * (dense + attn + dw)
    if op == "mamba":  # GLU fallback: in_proj at full res, pool, pw1 (2x GLU width), dw, pw2, out_proj reduced
        B, C, H, W = shape
        ch, r = extra
        hd = 2 * ch
        hw, hwh = H * W, (H // r) * (W // r)
        act = 2 * B * C * hw * E
        w = (ch * C + 2 * hd * ch + 9 * hd + ch * hd + C * ch + 4 * (ch + hd + C)) * F32
        flops = 2 * ch * C * hw + hwh * (2 * 2 * hd * ch + 2 * 9 * hd + 2 * ch * hd + 2 * C * ch)
        return act + w, B * flops
    if op == "decode":
        B, A = shape
        nc = extra
        return B * A * ((64 + nc) + (4 + nc)) * F32, B * A * (64 * 4 + nc * 4)
    if op == "head":  # fused last 1x1 convs of both towers + decode: reads the tower features, writes y
        B, A = shape
        nc, c2, c3 = extra
        return (B * A * ((c2 + c3) * E + (4 + nc) * F32) + (64 * c2 + nc * c3 + 64 + nc) * F32,
                B * A * (2 * (64 * c2 + nc * c3) + 64 * 4 + nc * 4))
    if op == "nms":
        B, nc, A = shape
        return B * A * (4 + nc) * F32, 0
    raise KeyError(op)


def bound_of(key, method: bool = True) -> str:
    """The roof that bounds a launch: whichever of its HBM time and matrix-core time (at the ceiling of the method
    the launch computes with, or at the dtype peak with method=False) is longer."""
    nbytes, flops = op_cost(key)
    peak = method_peak_tflops(key) if method else peak_tflops(key)
    return "mfma" if flops / (peak * 1e12) > nbytes / (PEAK_HBM_GBS * 1e9) else "hbm"


def t_min_ms(key, method: bool = False) -> float:
    """max(HBM time, matrix time) at the dtype peak, or (method=True) at the method ceiling method_peak_tflops."""
    nbytes, flops = op_cost(key)
    peak = method_peak_tflops(key) if method else peak_tflops(key)
    return max(nbytes / (PEAK_HBM_GBS * 1e9), flops / (peak * 1e12)) * 1e3
