"""Times the fp16-split 1x1 kernel (yolosod_conv1x1x2_silu) on the neck's n1 conv shapes of the n640 model at bs=32
(MIOpen conv + HIP bias/SiLU beside it). GPU only; one line per distinct (shape, Cout)."""
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


def timeit(fn, iters=30):
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
        if mod.n1:
            c = mod.conv
            shapes[(tuple(inp[0].shape), c.out_channels)] = (c.weight.detach(), c.bias.detach())

    hs = [m.register_forward_pre_hook(hook) for m in model.modules() if isinstance(m, M.Conv)]
    with torch.inference_mode():
        model(torch.rand(bs, 3, 640, 640, device=dev))
    for h in hs:
        h.remove()
    tot_a = tot_b = 0.0
    with torch.inference_mode():
        for (shape, cout), (w, b) in sorted(shapes.items(), key=lambda kv: -kv[0][0][2]):
            x = torch.randn(shape, device=dev)
            blk = _hip.conv1x1x2_prepare(w)
            out = torch.empty((shape[0], cout, shape[2], shape[3]), device=dev)
            out2 = torch.empty((shape[0], cout // 2, shape[2], shape[3]), device=dev)
            ta = timeit(lambda: _hip.bias_act(F.conv2d(x, w), b, 1))
            tb = timeit(lambda: _hip.conv1x1x2_silu(x, b, lambda: blk, cout, out=out))
            td = timeit(lambda: _hip.conv1x1x2_silu(x, b, lambda: blk, cout, out=out, out2=out2, c2lo=cout // 2))
            flops = 2.0 * shape[0] * shape[2] * shape[3] * shape[1] * cout
            byt = 4.0 * shape[0] * shape[2] * shape[3] * (shape[1] + cout)
            print(f"{str(shape):24s} -> {cout:5d}  miopen+epi {ta:7.3f} ms  x2 {tb:7.3f} ms "
                  f"({flops / tb / 1e9:6.1f} TF/s, {byt / tb / 1e6:6.0f} GB/s)  dual {td:7.3f} ms", flush=True)
            tot_a += ta
            tot_b += tb
    print(f"total n1 shapes: miopen+epi {tot_a:.3f} ms  x2 {tot_b:.3f} ms")


if __name__ == "__main__":
    main()
