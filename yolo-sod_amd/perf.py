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
                 or (op == "a2" and _on("YOLOSOD_A2_X2")) or (op == "head" and _on("YOLOSOD_HEAD_X2"))
                 or op in FUSED_CONV)
        if split:
            return PEAK_BF16_MFMA_TFLOPS / 3
    return peak_tflops(key)


# gate operators whose apply their consumer conv does (nn/tasks.py GATE_FUSE): the fused operator "<gate>_conv" =
# the gate's own launches ("<gate>_gate", billed to it) + the stride-2 conv that applies the gate while staging its
# input (csrc/conv3x3s2.hip, fp16 two-term splits); its roofline counts its real I/O (x read once, the conv output
# written once) and the conv's FLOPs
FUSED_CONV = {"se_conv": "se", "cbam_conv": "cbam"}
GATE_ONLY = {"se_gate": "se_conv", "cbam_gate": "cbam_conv"}
# operators of the SURVEY 8(a) path (rooflined); other keys the op_timer records are backbone conv kernels
PATH_OPS = frozenset({"se", "cbam", "ca", "a2", "swin", "mamba", "decode", "head", "nms", *FUSED_CONV})


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
    if op in FUSED_CONV:  # gate (statistics from the producer, MLP, CBAM's spatial map) + gated stride-2 conv
        B, C, H, W = shape
        cout, hid = extra
        Ho, Wo = (H + 1) // 2, (W + 1) // 2
        act = B * C * H * W * E + B * cout * Ho * Wo * E + (B * H * W * F32 if op == "cbam_conv" else 0)
        w = (cout * C * 9 + cout + 2 * C * hid + C + hid + (98 if op == "cbam_conv" else 0)) * F32
        flops = 2 * B * Ho * Wo * cout * C * 9 + B * C * H * W * (1 if op == "se_conv" else 2)
        return act + w, flops
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


# ---- hot-path summary of one timed region (bench.py, scripts/roofline_from_csv.py) --------------------------------

# statistics a producing conv epilogue emits for the gate that consumes its output (nn/tasks.py): the gate's own
# kernels then read x once; the producer's extra time over its plain variant is billed to the gate
PRODUCER_GATE = {"sum": "se", "summax": "cbam", "capool": "ca"}


def _numel(shape) -> int:
    n = 1
    for d in shape:
        n *= d
    return n


def producer_of(key):
    """For a launch key of a producing epilogue that emitted a gate's statistics: (gate op, gate input shape, key of
    the plain variant of the same shape, HBM bytes of the plain pass); None for any other key."""
    op, shape, extra = key[:3]
    tail, E = tuple(key[3:]), elem_size(key)
    if op == "bias_act" and isinstance(extra, str) and extra.split("+")[0] in PRODUCER_GATE:
        st, res = extra.split("+")[0], extra.endswith("+res")
        plain = ("bias_act", tuple(shape), "res" if res else None) + tail
        return PRODUCER_GATE[st], tuple(shape), plain, _numel(shape) * E * (3 if res else 2)
    if op == "conv1x1_thin" and isinstance(extra, tuple) and len(extra) == 2 and extra[1] in ("sum", "summax"):
        B, cin, H, W = shape
        cout = extra[0]
        plain = ("conv1x1_thin", tuple(shape), (cout, False, False)) + tail
        return PRODUCER_GATE[extra[1]], (B, cout, H, W), plain, B * H * W * (cin + cout) * E
    return None


class PathSelect:
    """``op_timer`` filter for bench.py's timed region: the hot-path operators, their gate-only launches, the producing
    epilogues that emit a gate's statistics and the plain variants those are billed against (collected while the
    filter sees the producers: run one untimed-region step through it first); everything else - the backbone's,
    the neck's and the Detect towers' convolutions and epilogues - runs without HIP events."""

    def __init__(self):
        self.plain = set()

    def __call__(self, key):
        if key[0] in PATH_OPS or key[0] in GATE_ONLY:
            return True
        p = producer_of(key)
        if p is not None:
            self.plain.add(p[2])
            return True
        return key in self.plain


def aggregate(calls):
    """[(key, ms), ...] per launch -> {key: [total ms, launches]} in first-seen order."""
    agg = {}
    for key, ms in calls:
        a = agg.setdefault(key, [0.0, 0])
        a[0] += ms
        a[1] += 1
    return agg


def producer_billing(agg):
    """{(gate op, gate shape): (extra ms per launch, description)} from the SAME timed region: the producer's mean
    in-model time minus the mean in-model time of its plain variant of the same shape (same element type, same
    residual input). When the model runs no plain variant of that shape, the plain pass is priced at the HBM roof
    (plain bytes / 8 TB/s), which bills the gate an upper bound of the producer's extra time."""
    out = {}
    for key, (tot, n) in agg.items():
        p = producer_of(key)
        if p is None:
            continue
        gate, gshape, plain, pbytes = p
        t_st = tot / n
        if plain in agg:
            t_pl = agg[plain][0] / agg[plain][1]
            basis = f"its in-model plain variant, {agg[plain][1]} launches"
        else:
            t_pl = pbytes / (PEAK_HBM_GBS * 1e9) * 1e3
            basis = "plain pass at the HBM roof (no plain variant of this shape in the model)"
        out[(gate, gshape)] = (max(0.0, t_st - t_pl),
                               f"{key[0]}{tuple(key[1])} {key[2]}: {t_st:.4f} ms in-model vs {t_pl:.4f} ms ({basis})")
    return out


def summarize(calls, steps):
    """Per-operator summary of one timed region's launches: (ops, backbone ops, path_roofline). ``ops`` carry the
    cost-model fields (bytes, flops, key) beside the reported ones; avg_ms = the operator's own launch sequence + the
    billed producer extra; path_roofline = sum_k t_k^min / sum_k t_k^meas."""
    agg = aggregate(calls)
    billed = producer_billing(agg)
    # gate-only launches: billed (per launch of the fused operator) to the fused operator of the same gate shape
    gate_ms = {}
    for key, (tot, n) in agg.items():
        if key[0] in GATE_ONLY:
            k2 = (GATE_ONLY[key[0]], tuple(key[1]))
            gate_ms[k2] = gate_ms.get(k2, 0.0) + tot
    ops, backbone = [], []
    for key, (tot, n) in agg.items():
        if key[0] in GATE_ONLY:
            continue
        if key[0] not in PATH_OPS:  # backbone conv kernels of this library: outside the path roofline
            backbone.append({"op": key[0], "shape": list(key[1]), "extra": str(key[2]), "launches": n,
                             "total_ms_per_step": round(tot / steps, 4)})
            continue
        nbytes, flops = op_cost(key)
        kern = tot / n + gate_ms.get((key[0], tuple(key[1])), 0.0) / n
        ext, src = billed.get((FUSED_CONV.get(key[0], key[0]), tuple(key[1])), (0.0, None))
        avg = kern + ext
        bound = bound_of(key)
        tm, tm_d = t_min_ms(key, method=True), t_min_ms(key)
        o = {"op": key[0], "shape": list(key[1]), "dtype": "bf16" if elem_size(key) == 2 else "f32",
             "launches": n, "avg_ms": round(avg, 4), "kernels_ms": round(kern, 4),
             "total_ms_per_step": round(avg * n / steps, 4),
             "GBps": round(nbytes / (avg * 1e-3) / 1e9, 1), "TFLOPs": round(flops / (avg * 1e-3) / 1e12, 2),
             "bound": bound, "peak": method_peak_tflops(key) if bound == "mfma" else PEAK_HBM_GBS,
             "t_min_ms": round(tm, 4), "frac": round(tm / avg, 3), "frac_vs_dtype_peak": round(tm_d / avg, 3),
             "bytes": nbytes, "flops": flops, "key": key}
        if src:
            o["producer_extra_ms"] = round(ext, 4)
            o["producer"] = src
        ops.append(o)
    ops.sort(key=lambda o: -o["total_ms_per_step"])
    t_meas = sum(o["total_ms_per_step"] for o in ops)
    t_min = sum(t_min_ms(o["key"], method=True) * o["launches"] / steps for o in ops)
    t_min_d = sum(t_min_ms(o["key"]) * o["launches"] / steps for o in ops)
    path = {"t_min_ms": round(t_min, 4), "t_meas_ms": round(t_meas, 4),
            "frac": round(t_min / t_meas, 4) if t_meas else None,
            "definition": "sum over hot-path ops of max(bytes / 8 TB/s, flops / matrix ceiling of the method the op "
                          "computes with: fp16 peak / 3 = 838.9 TF/s for the fp32 ops on fp16 two-term splits, 2516.6 "
                          "for bf16, 157.3 for exact fp32 MFMA) / measured; a producing epilogue's extra time for a "
                          "gate's statistics (in-model producer minus its in-model plain variant of the same shape) is "
                          "billed to the gate",
            "frac_vs_dtype_peak": round(t_min_d / t_meas, 4) if t_meas else None}
    path["mafn"] = mafn_path(ops, steps)
    return ops, sorted(backbone, key=lambda o: -o["total_ms_per_step"]), path


# ---- the MAFN + decode + NMS path exactly as SURVEY 8(d) defines it -------------------------------------------------

def _split_fused(key):
    """A gate-fused operator (se_conv / cbam_conv) -> (8(d) key of its gate instance, the consumer conv's own t_min in
    ms): the conv reads the gated input once and writes its output once, its FLOPs at the fp16-split ceiling."""
    op, shape, extra = key[:3]
    B, C, H, W = shape
    cout, hid = extra
    E = elem_size(key)
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    conv_b = (B * C * H * W + B * cout * Ho * Wo) * E + (cout * C * 9 + cout) * F32
    conv_f = 2 * B * Ho * Wo * cout * C * 9
    t_conv = max(conv_b / (PEAK_HBM_GBS * 1e9), conv_f / (PEAK_BF16_MFMA_TFLOPS / 3 * 1e12)) * 1e3
    return (FUSED_CONV[op], tuple(shape), hid) + tuple(key[3:]), t_conv


def mafn_path(ops, steps):
    """SURVEY 8(d)'s path, a fixed definition: the MAFN instances (SE / CBAM / CA / A2 / Swin / Mamba: input read once,
    output written once, weights once), the decode (A (74 + 14) floats per image: the fused Detect head is billed at the
    decode's bytes, its measured time includes the towers' last 1x1 convs) and the NMS scan (A 14 floats per image).
    t_min per instance = max(bytes / 8 TB/s, FLOPs / the matrix ceiling of the method it computes with); t_meas = its
    measured time. SE L1 / CBAM L4 run inside their consumer stride-2 conv (gate fusion): the instance is billed at its
    8(d) bytes, its measured time = the fused operator's time minus the conv's own t_min (so an upper bound on the
    gate's time) and the conv's FLOPs are not counted. ``frac_vs_hbm_floor`` = the 8(d) HBM floor (all bytes at 8 TB/s;
    0.352 ms for n640 bs 32) / t_meas."""
    t_min = t_meas = 0.0
    nbytes = 0
    parts = []
    for o in ops:
        key, n = o["key"], o["launches"]
        if key[0] in FUSED_CONV:
            k8, t_conv = _split_fused(key)
            meas = max(o["avg_ms"] - t_conv, 0.0)
        elif key[0] == "head":
            B, A = key[1]
            nc = key[2][0]
            k8, meas = ("decode", (B, A), nc) + tuple(key[3:]), o["avg_ms"]
        else:
            k8, meas = key, o["avg_ms"]
        b, _ = op_cost(k8)
        tm = t_min_ms(k8, method=True)
        nbytes += b * n / steps
        t_min += tm * n / steps
        t_meas += meas * n / steps
        parts.append(f"{k8[0]}{tuple(k8[1])}: {meas:.4f} ms")
    floor = nbytes / (PEAK_HBM_GBS * 1e9) * 1e3
    return {"bytes_per_step": int(nbytes), "t_hbm_floor_ms": round(floor, 4), "t_min_ms": round(t_min, 4),
            "t_meas_ms": round(t_meas, 4), "frac": round(t_min / t_meas, 4) if t_meas else None,
            "frac_vs_hbm_floor": round(floor / t_meas, 4) if t_meas else None,
            "definition": "SURVEY 8(d): MAFN instances + decode + NMS scan; gate-fused SE/CBAM billed without their "
                          "consumer conv (its t_min subtracted, its FLOPs excluded)", "instances": parts}


# ---- per-launch CSV (bench.py --ops-csv): one row per timed C-ABI launch sequence ---------------------------------

CSV_FIELDS = ("config", "steps", "seq", "op", "shape", "extra", "esize", "ms")


def calls_to_rows(config, steps, calls):
    return [{"config": config, "steps": steps, "seq": i, "op": k[0], "shape": "x".join(map(str, k[1])),
             "extra": repr(k[2]), "esize": k[3] if len(k) > 3 else "", "ms": f"{ms:.6f}"}
            for i, (k, ms) in enumerate(calls)]


def rows_to_calls(rows):
    """CSV rows of one config -> [(key, ms)] exactly as the op_timer recorded them."""
    import ast
    out = []
    for r in rows:
        key = (r["op"], tuple(int(d) for d in r["shape"].split("x")), ast.literal_eval(r["extra"]))
        if r["esize"] != "":
            key = key + (int(r["esize"]),)
        out.append((key, float(r["ms"])))
    return out
