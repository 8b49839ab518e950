"""Micro-benchmark: the Detect tower 3x3 convs at the n640 shapes (bs 32) on the fp16-split kernel vs MIOpen
(F.conv2d without bias + the HIP bias / SiLU epilogue, as the executor runs it). GPU only."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import yolosod_import  # noqa: E402,F401
from yolosod_amd import _hip  # noqa: E402

dev = torch.device("cuda", 0)
SHAPES = [(32, 64, 160, 160), (32, 128, 80, 80), (32, 64, 80, 80), (32, 256, 40, 40), (32, 64, 40, 40),
          (32, 512, 20, 20), (32, 64, 20, 20)]


def timed(fn, reps=50):
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
if ABL:  # timing ablations of the kernel (wrong results): see yolosod_debug_set_conv3x3_abl
    lib = _hip.load_library()
    for shape in SHAPES[:2]:
        B, cin, H, W = shape
        x = torch.randn(shape, device=dev)
        w = torch.randn(64, cin, 3, 3, device=dev) * 0.05
        b = torch.randn(64, device=dev) * 0.1
        prep = _hip.conv3x3_prepare(w)
        gf = 2 * B * H * W * 64 * cin * 9 / 1e9
        lib.yolosod_debug_set_conv3x3_abl(0)
        y0 = _hip.conv3x3_silu(x, b, lambda: prep)
        for a in ABL:
            lib.yolosod_debug_set_conv3x3_abl(a)
            t_k = timed(lambda: _hip.conv3x3_silu(x, b, lambda: prep))
            d = (_hip.conv3x3_silu(x, b, lambda: prep) - y0).abs().max().item()  # 0 for the exact variants
            print(f"{str(shape):22s} abl {a:2d} {t_k:7.3f} ms ({gf / t_k:6.1f} TF/s)  max|y - y_abl0| {d:.3g}",
                  flush=True)
        lib.yolosod_debug_set_conv3x3_abl(0)
    sys.exit(0)

for shape in SHAPES:
    B, cin, H, W = shape
    x = torch.randn(shape, device=dev)
    w = torch.randn(64, cin, 3, 3, device=dev) * 0.05
    b = torch.randn(64, device=dev) * 0.1
    prep = _hip.conv3x3_prepare(w)
    t_k = timed(lambda: _hip.conv3x3_silu(x, b, lambda: prep))
    t_m = timed(lambda: _hip.bias_act(F.conv2d(x, w, None, padding=1), b, 1))
    gf = 2 * B * H * W * 64 * cin * 9 / 1e9
    print(f"{str(shape):22s} kernel {t_k:7.3f} ms ({gf / t_k:6.1f} TF/s)   MIOpen+epilogue {t_m:7.3f} ms "
          f"({gf / t_m:6.1f} TF/s)", flush=True)
