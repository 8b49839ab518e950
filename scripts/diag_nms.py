"""Read the NMS phase stamps of a diag build (scripts/diag_nms.sh), median over the 32 images, per load:
YOLOSOD_LIB_AB=ab_nms/lib_nms_diag.so python scripts/diag_nms.py [loads...]"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import yolosod_import  # noqa: E402,F401
from yolosod_amd import _hip  # noqa: E402
from yolosod_amd.utils.ops import non_max_suppression_padded  # noqa: E402
from bench import loaded_predictions  # noqa: E402

SEL = ["count scan", "to key loads", "radix select (regs)", "compaction + pos gather", "sort prefix", "prefix boxes"]
RES = ["prefix greedy", "rows out + fallback + pad"]


CLUSTERS = 50


def main():
    global CLUSTERS
    if "--clusters" in sys.argv:
        k = sys.argv.index("--clusters")
        CLUSTERS = int(sys.argv[k + 1])
        del sys.argv[k:k + 2]
    dev = torch.device("cuda")
    lib = _hip.load_library()
    buf = (ctypes.c_ulonglong * (32 * 24))()
    for n in [int(a) for a in sys.argv[1:]] or [1000, 10000, 30000]:
        pred = loaded_predictions(32, 34000, 10, n, CLUSTERS, 0.25, 0, dev)
        for _ in range(3):
            non_max_suppression_padded(pred.clone(), 0.25, 0.7, max_det=300)
        torch.cuda.synchronize()
        assert lib.yolosod_diag_nms_stamps(buf) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(32, 24).astype(np.int64)
        out = [f"n={n}:"]
        for i, name in enumerate(SEL):
            d = a[:, i + 1] - a[:, i]
            out.append(f"{name} {np.median(d) / 1e3:.1f}k")
        out.append(f"| select total {np.median(a[:, 6] - a[:, 0]) / 1e3:.1f}k")
        for i, name in enumerate(RES):
            d = a[:, 9 + i] - a[:, 8 + i]
            out.append(f"| {name} {np.median(d) / 1e3:.1f}k")
        ps = [f"{np.median(a[:, 16 + d] - a[:, 2]) / 1e3:.1f}k" for d in (2, 1, 0) if np.median(a[:, 16 + d]) > 0]
        out.append(f"| pass ends after key loads (digit 23:16, 15:8, 7:0): {' '.join(ps)}")
        out.append(f"| fallback rem {np.median(a[:, 19]):.0f} chunks {np.median(a[:, 23]):.0f}: kept-test "
                   f"{np.median(a[:, 20]) / 1e3:.1f}k, chunk mask {np.median(a[:, 21]) / 1e3:.1f}k, greedy "
                   f"{np.median(a[:, 22]) / 1e3:.1f}k")
        out.append(f"| image 0: n {a[0, 11]} m {a[0, 12]} K {a[0, 13]} T {a[0, 14]:#x}")
        print(" ".join(out), "(kcycles of s_memtime)", flush=True)


if __name__ == "__main__":
    main()
