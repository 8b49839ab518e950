"""Micro-benchmark: the gate-consumer stride-2 convs at the n640 / m640 shapes on the fused kernel (gate applied at
staging) vs what it replaces: the gate's apply pass + MIOpen conv (no bias) + the HIP bias / SiLU epilogue. GPU only."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import yolosod_import  # noqa: E402,F401
from yolosod_amd import _hip  # noqa: E402

dev = torch.device("cuda", 0)
# (input shape, Cout, gates): SE L1 -> L2 and CBAM L4 -> L5 (n640, n1280), SE L1 -> L2 (m640 shape)
SHAPES = [((32, 32, 320, 320), 64, "c"), ((32, 64, 160, 160), 128, "cp"), ((8, 32, 640, 640), 64, "c"),
          ((8, 64, 320, 320), 128, "cp"), ((64, 64, 320, 320), 128, "c")]


def timed(fn, reps=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


ABL = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else []
if ABL:  # timing ablations at the SE L1 -> L2 shape (wrong results): yolosod_debug_set_conv3x3s2_abl
    lib = _hip.load_library()
    (B, cin, H, W), cout, _ = SHAPES[0]
    x = torch.randn(B, cin, H, W, device=dev)
    w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
    b = torch.randn(cout, device=dev) * 0.1
    gc = torch.sigmoid(torch.randn(B, cin, device=dev))
    prep = _hip.conv3x3s2_prepare(w)
    for a in ABL:
        lib.yolosod_debug_set_conv3x3s2_abl(a)
        t = timed(lambda: _hip.conv3x3s2_silu(x, b, lambda: prep, cout, gc))
        print(f"abl {a:2d} {t:7.3f} ms", flush=True)
    lib.yolosod_debug_set_conv3x3s2_abl(0)
    sys.exit(0)

for shape, cout, gates in SHAPES:
    B, cin, H, W = shape
    x = torch.randn(shape, device=dev)
    w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
    b = torch.randn(cout, device=dev) * 0.1
    gc = torch.sigmoid(torch.randn(B, cin, device=dev))
    gp = torch.sigmoid(torch.randn(B, H, W, device=dev)) if "p" in gates else None
    prep = _hip.conv3x3s2_prepare(w)
    t_f = timed(lambda: _hip.conv3x3s2_silu(x, b, lambda: prep, cout, gc, gp))
    t_n = timed(lambda: _hip.conv3x3s2_silu(x, b, lambda: prep, cout))

    def unfused():
        xg = x * gc[:, :, None, None]
        if gp is not None:
            xg = xg * gp[:, None]
        return _hip.bias_act(F.conv2d(xg, w, None, stride=2, padding=1), b, 1)

    t_u = timed(unfused)
    t_c = timed(lambda: _hip.bias_act(F.conv2d(x, w, None, stride=2, padding=1), b, 1))
    gf = 2 * B * ((H + 1) // 2) * ((W + 1) // 2) * cout * cin * 9 / 1e9
    gb = (x.numel() + B * cout * ((H + 1) // 2) * ((W + 1) // 2)) * 4 / 1e9
    print(f"{str(shape):22s} Cout {cout:3d} gates {gates:2s}  fused {t_f:7.3f} ms ({gf / t_f:6.1f} TF/s, "
          f"{gb / t_f:5.2f} TB/s)  no-gate {t_n:7.3f}  |  torch apply + MIOpen + epilogue {t_u:7.3f} "
          f"(MIOpen + epilogue alone {t_c:7.3f})", flush=True)
