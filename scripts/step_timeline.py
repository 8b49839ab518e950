"""Per-step GPU occupancy from a rocprofv3 --kernel-trace CSV of bench.py: how much of a step's wall time has at least
one kernel running (the union of kernel intervals), how much kernel time overlaps, each stream's busy time, and the
longest whole-GPU idle gaps with the kernel that ended before each.

    python scripts/step_timeline.py gpurun_out/TAG/prof/.../run_kernel_trace.csv --steps 5
"""
import argparse
import csv
from collections import defaultdict


def short(name):
    return name.replace("void ", "").split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="swin_x3_kernel")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--gaps", type=int, default=12)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"need {a.steps + 1} marker kernels, found {len(marks)}")
    t0 = int(rows[marks[-a.steps - 1]]["Start_Timestamp"])
    t1 = int(rows[marks[-1]]["Start_Timestamp"])
    seg = [r for r in rows if t0 <= int(r["Start_Timestamp"]) < t1]
    sid = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    iv = sorted((int(r["Start_Timestamp"]), min(int(r["End_Timestamp"]), t1), r) for r in seg)
    union, gaps, cur_s, cur_e, last = 0, [], None, None, None
    for s, e, r in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
                gaps.append((s - cur_e, last))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= cur_e:
            last = r
    union += cur_e - cur_s
    wall = t1 - t0
    ksum = sum(e - s for s, e, _ in iv)
    per = defaultdict(int)
    for s, e, r in iv:
        per[r.get(sid, "?")] += e - s
    n = a.steps
    print(f"# per step (mean of {n}): wall {wall / n / 1e6:.3f} ms, GPU busy (union) {union / n / 1e6:.3f} ms "
          f"({100 * union / wall:.1f} %), kernel time {ksum / n / 1e6:.3f} ms (overlap x{ksum / max(union, 1):.2f}), "
          f"{len(seg) / n:.0f} kernels")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"  {sid} {k}: busy {v / n / 1e6:.3f} ms")
    print(f"# idle gaps: {len(gaps) / n:.0f} per step, {sum(g for g, _ in gaps) / n / 1e6:.3f} ms per step; longest:")
    for g, r in sorted(gaps, key=lambda x: -x[0])[:a.gaps]:
        print(f"  {g / 1e3:8.1f} us after {short(r['Kernel_Name']) if r else '?'}")


if __name__ == "__main__":
    main()
