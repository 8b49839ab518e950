"""Micro-benchmark of individual HIP operators at the bs=32 640x640 shapes (GPU only; for rocprof A/B work)."""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import yolosod_import  # noqa: E402,F401
import recipes  # noqa: E402
from yolosod_amd import _hip, perf  # noqa: E402
from yolosod_amd.nn import modules as M  # noqa: E402

CASES = {
    "swin_L28": ("SwinBlock", (64, 2, 7), (32, 64, 160, 160)),
    "swin_L9": ("SwinBlock", (256, 4, 7), (32, 256, 40, 40)),
    "a2_L12": ("A2_Attn", (512, None, 8, 8), (32, 512, 20, 20)),
    "a2_L12_1280": ("A2_Attn", (512, None, 8, 8), (8, 512, 40, 40)),  # configs[3] (n1280, bs 8)
    "swin_L28_1280": ("SwinBlock", (64, 2, 7), (8, 64, 320, 320)),
    "swin_L9_1280": ("SwinBlock", (256, 4, 7), (8, 256, 80, 80)),
    "se_L1": ("SE_Block", (64,), (32, 32, 320, 320)),
    "cbam_L4": ("CBAM_Block", (64, 128, 16), (32, 64, 160, 160)),
    "ca_L32": ("CA_Block", (128, 256, 32), (32, 128, 80, 80)),
    "cbam_L18": ("CBAM_Block", (256, 512, 16), (32, 256, 40, 40)),
    "se_L23": ("SE_Block", (256,), (32, 128, 80, 80)),
    "mamba_L7": ("MambaBlock", (128, 256, 2), (32, 128, 80, 80)),  # yolov12-sod-fusion-v5 only
    "head": ("detect_head", (64, 64, 10), (32, 0, 640, 640)),  # fused Detect tail + decode, 4 levels P2..P5
    # bf16 m-scale config (bs=64): run with --bf16
    "swin_L28_m": ("SwinBlock", (128, 2, 7), (64, 128, 160, 160)),
    "swin_L9_m": ("SwinBlock", (512, 4, 7), (64, 512, 40, 40)),
    "a2_L12_m": ("A2_Attn", (512, None, 8, 8), (64, 512, 20, 20)),
    "cbam_L4_m": ("CBAM_Block", (128, 128, 16), (64, 128, 160, 160)),
    "ca_L32_m": ("CA_Block", (256, 256, 32), (64, 256, 80, 80)),
    # the gate-fused operators as the model runs them (GATE_FUSE): the gate kernels, then the consumer stride-2 conv
    # applying it while staging its input (se_conv: SE L1 -> Conv L2; cbam_conv: CBAM L4 -> Conv L5)
    "se_conv_L1": ("gated_se", (64, 64), (32, 32, 320, 320)),
    "cbam_conv_L4": ("gated_cbam", (64, 128, 16), (32, 64, 160, 160)),
    # NMS (predict mode) on [32, 14, 34000] with 0 / 30k candidates per image (synthetic, bench.loaded_predictions)
    "nms_empty": ("nms", (0,), (32, 14, 34000)),
    "nms_30k": ("nms", (30000,), (32, 14, 34000)),
}


def head_case(dev, c2, c3, nc, B, S):
    g = torch.Generator(device="cpu").manual_seed(0)
    sizes = [S // s for s in (4, 8, 16, 32)]
    fb = [torch.randn(B, c2, h, h, generator=g).to(dev) for h in sizes]
    fc = [torch.randn(B, c3, h, h, generator=g).to(dev) for h in sizes]
    bw = [(torch.randn(64, c2, generator=g) * 0.1).to(dev) for _ in sizes]
    bb = [torch.zeros(64).to(dev) for _ in sizes]
    cw = [(torch.randn(nc, c3, generator=g) * 0.1).to(dev) for _ in sizes]
    cb = [torch.zeros(nc).to(dev) for _ in sizes]
    return lambda: _hip.detect_head(fb, fc, bw, bb, cw, cb, [4.0, 8.0, 16.0, 32.0], nc)


def gated_case(dev, op, args, shape):
    """gate + gated consumer conv (Conv.forward_gated) on x that carries its producer's statistics"""
    from yolosod_amd.nn.tasks import _fuse_conv_and_bn
    B, C, H, W = shape
    se = op == "gated_se"
    gate = M.SE_Block(args[0]) if se else M.CBAM_Block(C, None, args[2])
    if se:
        gate._maybe_build(C, None)
    cout = args[1]
    cons = M.Conv(C, cout, 3, 2)
    recipes.perturb_(gate, 1)
    recipes.perturb_(cons, 1)
    cons.conv = _fuse_conv_and_bn(cons.conv, cons.bn)
    delattr(cons, "bn")
    gate, cons = gate.to(dev).eval(), cons.to(dev).eval()
    x = torch.randn(shape, device=dev)
    x = _hip.bias_act(x, torch.zeros(C, device=dev), 0, out=torch.empty_like(x), stats="sum" if se else "summax")
    if se:
        key = ("se_conv", tuple(x.shape), (cout, gate.fc1.out_channels))
    else:
        key = ("cbam_conv", tuple(x.shape), (cout, gate.channel_attention.fc[0].out_channels))

    def fn():
        gc, gp = (gate.gate(x), None) if se else gate.gates(x)
        return cons.forward_gated(x, gc, gp, key)
    return fn, key


def nms_case(dev, n_cand, shape):
    from bench import loaded_predictions
    from yolosod_amd.utils.ops import non_max_suppression_padded
    B, no, A = shape
    pred = loaded_predictions(B, A, no - 4, n_cand, 50, 0.25, 0, dev)
    # in place: the repeated xywh -> xyxy rewrite changes the boxes, not the candidate set or the traffic
    return lambda: non_max_suppression_padded(pred, 0.25, 0.7, max_det=300)


def main():
    args = sys.argv[1:]
    bf16 = "--bf16" in args
    names = [a for a in args if not a.startswith("--")] or list(CASES)
    dev = torch.device("cuda")
    dt = torch.bfloat16 if bf16 else torch.float32
    for name in names:
        op, args, shape = CASES[name]
        if op == "detect_head":
            fn = head_case(dev, *args, shape[0], shape[2])
            m, x = (lambda _x: fn()), None
        elif op in ("gated_se", "gated_cbam"):
            fn, fused_key = gated_case(dev, op, args, shape)
            m, x = (lambda _x: fn()), None
        elif op == "nms":
            fn = nms_case(dev, args[0], shape)
            m, x = (lambda _x: fn()), None
        else:
            m = getattr(M, op)(*args)
            if op == "SE_Block":
                m._maybe_build(shape[1], None)
            recipes.perturb_(m, 1)
            if bf16:  # as build_model(dtype=bf16): fold the Conv+BN pairs in fp32, then cast
                from yolosod_amd.nn.tasks import _fuse_conv_and_bn
                for sub in m.modules():
                    if isinstance(sub, M.Conv) and hasattr(sub, "bn"):
                        sub.conv = _fuse_conv_and_bn(sub.conv, sub.bn)
                        delattr(sub, "bn")
                        sub.forward = sub.forward_fuse
            m = m.to(dev).to(dt).eval()
            x = torch.randn(shape, device=dev).to(dt)
            # SE / CBAM / CA as the model runs them: x comes from a conv epilogue that also emitted the gate's
            # statistics (bias_act stats=...), so the timed call takes the *_pre path (no statistics pass over x)
            mode = {"SE_Block": "sum", "CBAM_Block": "summax", "CA_Block": "capool"}.get(op)
            if mode:
                x = _hip.bias_act(x, torch.zeros(shape[1], device=dev), 0, out=torch.empty_like(x), stats=mode)
        with torch.inference_mode():
            for _ in range(3):
                m(x)
            torch.cuda.synchronize()
            with _hip.op_timer() as t:
                for _ in range(10):
                    m(x)
            d = t.durations_ms()
        key = d[0][0]
        ms = sum(v for _, v in d) / len(d)
        if op in ("gated_se", "gated_cbam"):  # the gate and the conv are separate timed launches: both per call
            key, ms = fused_key, sum(v for _, v in d) / 10
        b, f = perf.op_cost(key)
        print(f"{name:10s} {ms:8.3f} ms  {b / ms / 1e6:8.1f} GB/s  {f / ms / 1e9:7.2f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
