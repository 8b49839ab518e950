"""Micro-benchmark of the fp32 MFMA GEMM (C-ABI test hook) at the Swin-L9 / A2 shapes; --bf16: the bf16 GEMM at the
m-scale bf16 config's Swin-L9 / A2 shapes (tokens x N x K)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import yolosod_import  # noqa: E402,F401
from yolosod_amd import _hip  # noqa: E402

SHAPES_BF16 = [(112896, 1536, 512), (112896, 512, 512), (112896, 1024, 512), (112896, 512, 1024), (10240, 1536, 512),
               (8192, 8192, 8192)]
SHAPES = [(56448, 768, 256), (56448, 512, 256), (56448, 256, 512), (56448, 256, 256), (5120, 1536, 512),
          (829472, 192, 64), (4096, 4096, 4096)]


def main():
    dev = torch.device("cuda")
    bf16 = "--bf16" in sys.argv
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:] if not a.startswith("--")] or (
        SHAPES_BF16 if bf16 else SHAPES)
    torch_ref = "--no-torch" not in sys.argv
    shapes = [s for s in shapes if len(s) == 3]
    for (M, N, K) in shapes:
        dt = torch.bfloat16 if bf16 else torch.float32
        A = torch.randn(M, K, device=dev).to(dt)
        B = torch.randn(N, K, device=dev).to(dt)
        bias = torch.randn(N, device=dev)
        gemm = _hip.gemm_bf16 if bf16 else _hip.gemm_f32
        for _ in range(3):
            gemm(A, B, True, bias=bias, bias_mode=2)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 10
        e0.record()
        for _ in range(n):
            gemm(A, B, True, bias=bias, bias_mode=2)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        tf = 2 * M * N * K / ms / 1e9
        if not torch_ref:
            print(f"M={M:7d} N={N:5d} K={K:5d}  {ms:8.3f} ms  {tf:7.1f} TFLOP/s", flush=True)
            continue
        Bt = B.t()
        for _ in range(3):
            torch.mm(A, Bt)
        e0.record()
        for _ in range(n):
            torch.mm(A, Bt)
        e1.record()
        torch.cuda.synchronize()
        ms_t = e0.elapsed_time(e1) / n
        print(f"M={M:7d} N={N:5d} K={K:5d}  {ms:8.3f} ms  {tf:7.1f} TFLOP/s   (torch.mm {ms_t:7.3f} ms "
              f"{2 * M * N * K / ms_t / 1e9:6.1f} TFLOP/s)", flush=True)


if __name__ == "__main__":
    main()
