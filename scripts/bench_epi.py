"""Conv-epilogue micro-benchmark at the n640 backbone shapes (GPU only): bias_act (+ residual, dual store), the
statistics and CA-pool variants. python scripts/bench_epi.py; YOLOSOD_LIB_AB=<lib> for A/B builds."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import yolosod_import  # noqa: E402,F401
from yolosod_amd import _hip  # noqa: E402

CASES = [  # (B, C, H, W, residual, stats)
    (32, 64, 160, 160, False, None), (32, 64, 80, 80, False, None), (32, 128, 80, 80, False, None),
    (32, 32, 160, 160, False, None), (32, 256, 40, 40, False, None), (32, 32, 320, 320, False, None),
    (32, 64, 160, 160, True, None), (32, 32, 320, 320, False, "sum"), (32, 128, 80, 80, False, "capool"),
]


def main():
    dev = torch.device("cuda")
    bf16 = "--bf16" in sys.argv
    dt = torch.bfloat16 if bf16 else torch.float32
    for B, C, H, W, res, stats in CASES:
        if bf16:
            B *= 2  # the m640 config's batch of 64
        y = torch.randn(B, C, H, W, device=dev).to(dt)
        out = torch.empty_like(y)
        r = torch.randn_like(y) if res else None
        bias = torch.randn(C, device=dev)
        fn = lambda: _hip.bias_act(y, bias, 1, out=out, res=r, stats=stats)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        nbytes = y.numel() * y.element_size() * (3 if res else 2)
        print(f"bias_act {B}x{C}x{H}x{W} res={int(res)} stats={stats}: {ms * 1e3:7.1f} us  {nbytes / ms / 1e9:6.2f} TB/s",
              flush=True)


if __name__ == "__main__":
    main()
