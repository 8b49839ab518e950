"""A few launches of the P2 Detect tower conv (32 x 64 x 160 x 160 -> 64) on the stride-1 fp16-split kernel, for
rocprofv3 --pmc passes. GPU only."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import yolosod_import  # noqa: E402,F401
from yolosod_amd import _hip  # noqa: E402

dev = torch.device("cuda", 0)
B, cin, H, W, cout = 32, 64, 160, 160, 64
x = torch.randn(B, cin, H, W, device=dev)
w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
b = torch.randn(cout, device=dev) * 0.1
prep = _hip.conv3x3_prepare(w)
for _ in range(5):
    _hip.conv3x3_silu(x, b, lambda: prep, cout)
torch.cuda.synchronize()
print("ok")
