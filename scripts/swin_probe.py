"""Diagnostic: fused Swin (L28 shape) timing under load ablations (YOLOSOD_SWIN_ABL) and per-stage cycle shares.

abl bits: 1 skip halo loads, 2 skip weight loads, 4 skip residual loads (results are wrong; timing only)."""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import torch  # noqa: E402
import yolosod_import  # noqa: E402,F401
import recipes  # noqa: E402
from yolosod_amd import _hip  # noqa: E402
from yolosod_amd.nn import modules as M  # noqa: E402

C = int(os.environ.get("PROBE_C", "64"))
NH = int(os.environ.get("PROBE_NH", "2"))
S = int(os.environ.get("PROBE_S", "160"))
m = M.SwinBlock(C, NH, 7)
recipes.perturb_(m, 1)
m = m.cuda().eval()
x = torch.randn(32, C, S, S, device="cuda")
flops = None


def timeit(n=20):
    with torch.inference_mode():
        for _ in range(3):
            m(x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            m(x)
        e1.record()
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for abl in (0, 1, 2, 4, 7):
    os.environ["YOLOSOD_SWIN_ABL"] = str(abl)
    print(f"abl={abl}: {timeit():.4f} ms", flush=True)
os.environ["YOLOSOD_SWIN_ABL"] = "0"

NAMES = {1: "patch", 2: "dwconv", 3: "ln1stats", 4: "qkv", 5: "attn", 6: "outproj", 7: "ln2stats", 8: "mlp1",
         9: "mlp2", 15: "pw+store"}
os.environ["YOLOSOD_SWIN_STAMPS"] = "1"
lib = _hip.load_library()
lib.yolosod_debug_swin_stage_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
with torch.inference_mode():
    m(x)
    torch.cuda.synchronize()
out = (ctypes.c_double * 16)()
assert lib.yolosod_debug_swin_stage_cycles(out, 16) == 0
tot = sum(out[1:16])
for k in range(1, 16):
    if out[k]:
        print(f"{k:2d} {NAMES.get(k, '?'):10s} {out[k]:10.0f} cycles {100 * out[k] / tot:5.1f}%")
print("total per window", tot)
