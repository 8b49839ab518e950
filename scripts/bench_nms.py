"""NMS at controlled candidate loads: at random init nothing clears conf 0.25, so the bench's NMS
line is an empty workload. Here (B=32, 4+nc=14, A=34000) predictions get exactly N candidates per image above
conf_thres, scattered over A, boxes drawn around `clusters` centres (heavy overlap, as trained heads produce).
Predict mode (conf 0.25, single label, max_det 300) and val mode (conf 0.001, multi-label, max_det 300).
GPU only; parity at these sizes is tests/test_gpu_nms.py::test_nms_full_size_vs_oracle.
usage: python scripts/bench_nms.py [--clusters C] [N ...]   (N given: predict mode, C clusters (default 50), those
candidate counts only; 0 = empty NMS; for per-kernel rocprofv3 summaries of one load)"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import yolosod_import  # noqa: E402,F401
from yolosod_amd.utils.ops import non_max_suppression_padded  # noqa: E402
from bench import loaded_predictions as make_pred  # noqa: E402


def main():
    dev = torch.device("cuda")
    B, A, nc = 32, 34000, 10
    print(f"{'mode':8s} {'cand/img':>9s} {'clusters':>8s} {'ms/call':>8s} {'kept/img':>9s}")
    args = sys.argv[1:]
    ncl = 50
    if "--clusters" in args:
        k = args.index("--clusters")
        ncl = int(args[k + 1])
        del args[k:k + 2]
    only = [int(a) for a in args]
    modes = (("predict", 0.25, {}),) if only else (("predict", 0.25, {}), ("val", 0.001, dict(multi_label=True)))
    for mode, conf, kw in modes:
        for n_cand in (only or (1000, 10000, 30000)):
            for clusters in ((ncl,) if only else (50, 1000)):
                pred = make_pred(B, A, nc, n_cand, clusters, conf, 0, dev)
                work = [pred.clone() for _ in range(13)]  # in-place xywh->xyxy rewrite: fresh copy per call
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for i in range(3):
                    non_max_suppression_padded(work[i], conf_thres=conf, iou_thres=0.7, max_det=300, **kw)
                e0.record()
                for i in range(3, 13):
                    _, counts, _ = non_max_suppression_padded(work[i], conf_thres=conf, iou_thres=0.7, max_det=300,
                                                              **kw)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 10
                print(f"{mode:8s} {n_cand:9d} {clusters:8d} {ms:8.3f} {counts.float().mean().item():9.1f}",
                      flush=True)


if __name__ == "__main__":
    main()
