"""Read the swin_wx stage stamps of a diag build (scripts/diag_wx.sh): YOLOSOD_LIB_AB=diag/lib_diag.so python ..."""
import ctypes
import os
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

NAMES = {0: "start", 1: "halo+dw", 2: "LN1", 23: "pw gemm", 22: "final T planes", 24: "pw store", 15: "T+=O, LN2"}
for hp in range(2):
    for k, n in enumerate(["Q gemm", "KV gemm", "bar", "KV store", "attention", "O store+outproj"]):
        NAMES[3 + 6 * hp + k] = f"hp{hp} {n}"
for ck in range(2):
    for k, n in enumerate(["MLP1", "hidden store", "MLP2"]):
        NAMES[16 + 3 * ck + k] = f"ck{ck} {n}"

dev = torch.device("cuda")
m = M.SwinBlock(256, 4, 7)
recipes.perturb_(m, 1)
m = m.to(dev).eval()
x = torch.randn(32, 256, 40, 40, device=dev)
with torch.inference_mode():
    for _ in range(3):
        m(x)
    torch.cuda.synchronize()
lib = _hip.load_library()
buf = (ctypes.c_ulonglong * (256 * 32))()
assert lib.yolosod_diag_wx_stamps(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 32).astype(np.int64)
keys = sorted(NAMES)
order = [0, 1, 2] + [3 + 6 * hp + k for hp in range(2) for k in range(6)] + [15] + \
        [16 + 3 * ck + k for ck in range(2) for k in range(3)] + [22, 23, 24]
d = np.diff(a[:, order], axis=1)
tot = a[:, 24] - a[:, 0]
print(f"window total (median over 256 windows): {np.median(tot):.0f} ticks")
for i, k in enumerate(order[1:]):
    print(f"  {NAMES[k]:22s} {np.median(d[:, i]):9.0f}  ({np.median(d[:, i]) / np.median(tot) * 100:5.1f} %)")
