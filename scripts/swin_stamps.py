"""Diagnostic: per-stage cycle shares of the fused Swin kernel (YOLOSOD_SWIN_STAMPS=1 build path)."""
import ctypes
import os
import sys
from pathlib import Path

os.environ["YOLOSOD_SWIN_STAMPS"] = "1"
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import torch  # noqa: E402
import yolosod_import  # noqa: E402,F401
import recipes  # noqa: E402
from yolosod_amd import _hip  # noqa: E402
from yolosod_amd.nn import modules as M  # noqa: E402

NAMES = {1: "patch", 2: "dwconv", 3: "ln1stats", 4: "qkv", 5: "attn", 6: "outproj", 7: "ln2stats", 8: "mlp1", 9: "mlp2", 15: "pw+store"}
m = M.SwinBlock(64, 2, 7)
recipes.perturb_(m, 1)
m = m.cuda().eval()
x = torch.randn(32, 64, 160, 160, device="cuda")
lib = _hip.load_library()
lib.yolosod_debug_swin_stage_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
with torch.inference_mode():
    for _ in range(3):
        m(x)
    torch.cuda.synchronize()
out = (ctypes.c_double * 16)()
assert lib.yolosod_debug_swin_stage_cycles(out, 16) == 0
tot = sum(out[1:16])
for k in range(1, 16):
    if out[k]:
        print(f"{k:2d} {NAMES.get(k, '?'):10s} {out[k]:10.0f} cycles {100 * out[k] / tot:5.1f}%")
print("total per window", tot)
