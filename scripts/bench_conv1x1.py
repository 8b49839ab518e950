"""A/B of the backbone's 1x1 convs at bs=32 640x640: MIOpen conv + HIP bias/act pass vs the library's fused
fp32 MFMA GEMM (yolosod_conv1x1). GPU only; prints one line per distinct shape."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import yolosod_import  # noqa: E402,F401
from yolosod_amd import _hip  # noqa: E402
from yolosod_amd.nn import modules as M  # noqa: E402
from yolosod_amd.nn.tasks import build_model  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    dev = torch.device("cuda")
    model = build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=dev)
    shapes = {}

    def hook(mod, inp):
        c = mod.conv
        if c.kernel_size == (1, 1) and c.stride == (1, 1) and c.groups == 1:
            x = inp[0]
            shapes[(tuple(x.shape), c.out_channels)] = (c.weight.detach().reshape(c.out_channels, -1),
                                                      c.bias.detach())

    hs = [m.register_forward_pre_hook(hook) for m in model.modules() if isinstance(m, M.Conv)]
    with torch.inference_mode():
        model(torch.rand(bs, 3, 640, 640, device=dev))
    for h in hs:
        h.remove()
    tot_a = tot_b = 0.0
    with torch.inference_mode():
        for (shape, cout), (w, b) in sorted(shapes.items(), key=lambda kv: -kv[0][0][2]):
            x = torch.randn(shape, device=dev)
            w4 = w.view(cout, -1, 1, 1)
            ta = timeit(lambda: _hip.bias_act(F.conv2d(x, w4), b, 1))
            ok = shape[1] % 32 == 0 and (shape[2] * shape[3]) % 4 == 0
            tb = timeit(lambda: _hip.conv1x1(x, w, b, 1)) if ok else float("nan")
            okt = _hip.conv1x1_thin_ok(x, cout)
            tt = timeit(lambda: _hip.conv1x1_thin(x, w, b)) if okt else float("nan")
            print(f"   thin {tt:7.3f} ms", flush=True)
            flops = 2.0 * shape[0] * shape[2] * shape[3] * shape[1] * cout
            print(f"{str(shape):24s} -> {cout:5d}  miopen+epi {ta:7.3f} ms  gemm {tb:7.3f} ms  "
                  f"({flops / tb / 1e9 if ok else 0:6.1f} TF/s gemm)", flush=True)
            tot_a += ta
            tot_b += tb if ok else ta
    print(f"total 1x1: miopen+epi {tot_a:.3f} ms  gemm {tot_b:.3f} ms")


if __name__ == "__main__":
    main()
