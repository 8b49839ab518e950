"""Per-phase cycle breakdown of the NMS image kernel (diagnostic build path: YOLOSOD_NMS_STAMPS=1).
Phases: compaction, radix sort, greedy, tail; median over the 32 images of one call. GPU only."""
import ctypes
import os
import sys
from pathlib import Path

os.environ["YOLOSOD_NMS_STAMPS"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))
import yolosod_import  # noqa: E402,F401
from bench_nms import make_pred  # noqa: E402
from yolosod_amd import _hip  # noqa: E402
from yolosod_amd.utils.ops import non_max_suppression_padded  # noqa: E402

lib = _hip.load_library()
lib.yolosod_debug_nms_stage_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
dev = torch.device("cuda")
B = 32
print(f"{'mode':8s} {'cand':>6s} {'K':>5s}  {'compact':>9s} {'select':>9s} {'greedy':>9s} {'fallback':>9s}   (kcycles, median image)")
for mode, conf, kw in (("predict", 0.25, {}), ("val", 0.001, dict(multi_label=True))):
    for n_cand in (0, 1000, 10000, 30000):
        pred = make_pred(B, 34000, 10, max(n_cand, 1), 50, conf, 0, dev)
        if n_cand == 0:
            pred[:, 4:] = 0.0
        for _ in range(2):
            non_max_suppression_padded(pred.clone(), conf_thres=conf, iou_thres=0.7, max_det=300, **kw)
        torch.cuda.synchronize()
        out = (ctypes.c_double * (B * 6))()
        assert lib.yolosod_debug_nms_stage_cycles(out, B) == 0
        a = np.array(out[:]).reshape(B, 6)
        med = np.median(a, 0)
        print(f"{mode:8s} {int(med[4]):6d} {int(med[5]):5d}  {med[0] / 1e3:9.1f} {med[1] / 1e3:9.1f} "
              f"{med[2] / 1e3:9.1f} {med[3] / 1e3:9.1f}", flush=True)
