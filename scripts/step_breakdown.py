"""Per-step kernel-time breakdown from a rocprofv3 --kernel-trace CSV of bench.py.

Steps are delimited by one marker kernel that runs once per step (default: the fused Swin kernel); the last
``--steps`` complete steps are averaged, so warm-up work (MIOpen's first-use search, allocator growth) is excluded.

    python scripts/step_breakdown.py gpurun_out/prof20/run_kernel_trace.csv --steps 3 > profiles/r01_step_breakdown.txt
"""
import argparse
import csv
from collections import defaultdict


def category(name):
    if name.startswith("miopenSp3AsmConv"):
        return "MIOpen Winograd " + "_".join(name.split("_")[-2:])
    if name.startswith("igemm_fwd"):
        return "MIOpen implicit GEMM (NHWC)"
    if name.startswith("Cijk"):
        return "hipBLASLt GEMM (MIOpen 1x1 convs)"
    if "batched_transpose" in name:
        return "MIOpen NCHW<->NHWC transposes"
    if "CatArrayBatchedCopy" in name:
        return "torch cat"
    if name.startswith(("ys::", "void ys::")) or "fold_bn_kernel" in name:
        return "HIP  " + name.split("(")[0].replace("void ", "")
    return "torch " + name.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="swin_fused_kernel")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"need {a.steps + 1} marker kernels, found {len(marks)}")
    lo, hi = marks[-a.steps - 1], marks[-1]
    seg = rows[lo:hi]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # noqa: E731
    wall = (int(rows[hi]["Start_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e6 / a.steps
    busy = sum(dur(r) for r in seg) / a.steps
    t, n = defaultdict(float), defaultdict(int)
    for r in seg:
        k = category(r["Kernel_Name"])
        t[k] += dur(r) / a.steps
        n[k] += 1
    hip = sum(v for k, v in t.items() if k.startswith("HIP"))
    print(f"# per step (mean of last {a.steps}): wall {wall:.3f} ms, kernels busy {busy:.3f} ms, "
          f"{len(seg) / a.steps:.0f} kernels; HIP library kernels {hip:.3f} ms")
    print(f"{'kernel / category':78s} {'calls':>6s} {'ms/step':>8s} {'%':>6s}")
    for k, v in sorted(t.items(), key=lambda kv: -kv[1]):
        print(f"{k[:78]:78s} {n[k] / a.steps:6.0f} {v:8.3f} {100 * v / busy:6.1f}")


if __name__ == "__main__":
    main()
