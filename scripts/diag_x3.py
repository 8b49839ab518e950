"""Read the swin_x3 (C = 64) stage stamps of a diag build (scripts/diag_x3.sh):
YOLOSOD_LIB_AB=ablib/lib_diag.so python scripts/diag_x3.py"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import yolosod_import  # noqa: E402,F401
import recipes  # noqa: E402
from yolosod_amd import _hip  # noqa: E402
from yolosod_amd.nn import modules as M  # noqa: E402

NAMES = ["halo load -> halo store", "dw conv", "LN1 + Q chunk0 store", "Q gemm chunk0", "Q chunk1 store",
         "Q chunk1 + K/V gemms", "K/V planes store", "attention", "O planes store", "out-proj + T", "LN2",
         "MLP1 x2 + GELU, hidden0 store wait", "hidden0 store", "MLP2 half0, wait", "hidden1 store", "MLP2 half1 + ",
         "final T planes", "pw gemm + store"]

dev = torch.device("cuda")
m = M.SwinBlock(64, 2, 7)
recipes.perturb_(m, 1)
m = m.to(dev).eval()
x = torch.randn(32, 64, 160, 160, device=dev)
with torch.inference_mode():
    for _ in range(3):
        m(x)
    torch.cuda.synchronize()
lib = _hip.load_library()
buf = (ctypes.c_ulonglong * (256 * 32))()
assert lib.yolosod_diag_x3_stamps(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 32).astype(np.int64)
d = np.diff(a[:, :19], axis=1)
tot = a[:, 18] - a[:, 0]
print(f"window total (median over 256 windows): {np.median(tot):.0f} ticks; first-window start spread "
      f"{np.ptp(a[:, 0]):.0f}")
for i in range(18):
    print(f"  {i:2d} {NAMES[i]:38s} {np.median(d[:, i]):9.0f}  ({np.median(d[:, i]) / np.median(tot) * 100:5.1f} %)")
