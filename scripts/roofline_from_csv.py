"""Recompute bench.py's hip_ops (avg_ms, kernels_ms, producer_extra_ms), roofline and path_roofline from the per-launch
CSV that `bench.py --ops-csv` wrote, and check them against the JSON line of the same run. CPU only.

    python scripts/roofline_from_csv.py profiles/r04_bench/ops_calls.csv profiles/r04_bench/bench.json
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import yolosod_import  # noqa: E402,F401
from yolosod_amd import perf  # noqa: E402

FIELDS = ("avg_ms", "kernels_ms", "total_ms_per_step", "frac", "producer_extra_ms", "launches")


def recompute(csv_path):
    by_cfg = defaultdict(list)
    with open(csv_path, newline="") as f:
        for r in csv.DictReader(f):
            by_cfg[r["config"]].append(r)
    out = {}
    for cfg, rows in by_cfg.items():
        steps = int(rows[0]["steps"])
        ops, _, path = perf.summarize(perf.rows_to_calls(rows), steps)
        out[cfg] = (ops, path)
    return out


def check(line, ops, path, label):
    bad = 0
    got = {(o["op"], tuple(o["shape"])): o for o in ops}
    for o in line["hip_ops"]:
        r = got.get((o["op"], tuple(o["shape"])))
        if r is None:
            print(f"{label}: {o['op']}{o['shape']} missing from the CSV")
            bad += 1
            continue
        for k in FIELDS:
            if k in o and abs(float(o[k]) - float(r.get(k, 0.0))) > 1.5e-4 * max(1.0, abs(float(o[k]))):
                print(f"{label}: {o['op']}{o['shape']} {k}: line {o[k]} vs CSV {r.get(k)}")
                bad += 1
    for k in ("t_min_ms", "t_meas_ms", "frac"):
        if abs(line["path_roofline"][k] - path[k]) > 2e-4:
            print(f"{label}: path_roofline.{k}: line {line['path_roofline'][k]} vs CSV {path[k]}")
            bad += 1
    mp = line["path_roofline"].get("mafn")
    if mp is not None:
        for k in ("t_min_ms", "t_meas_ms", "frac", "t_hbm_floor_ms"):
            if abs(mp[k] - path["mafn"][k]) > 2e-4:
                print(f"{label}: mafn_path.{k}: line {mp[k]} vs CSV {path['mafn'][k]}")
                bad += 1
    return bad


def main():
    res = recompute(sys.argv[1])
    for cfg, (ops, path) in res.items():
        print(f"{cfg}: path_roofline {path['frac']} (t_min {path['t_min_ms']} / t_meas {path['t_meas_ms']} ms)")
        mp = path["mafn"]
        print(f"{cfg}: mafn_path {mp['frac']} (t_min {mp['t_min_ms']} / t_meas {mp['t_meas_ms']} ms), HBM floor "
              f"{mp['t_hbm_floor_ms']} ms -> {mp['frac_vs_hbm_floor']}; {'; '.join(mp['instances'])}")
        for o in ops:
            ex = f"  producer_extra {o['producer_extra_ms']:.4f}  [{o['producer']}]" if "producer_extra_ms" in o else ""
            print(f"  {o['op']:5s} {str(o['shape']):22s} x{o['launches']:3d} avg {o['avg_ms']:.4f} ms "
                  f"(kernels {o['kernels_ms']:.4f}) frac {o['frac']:.3f}{ex}")
    if len(sys.argv) > 2:
        txt = Path(sys.argv[2]).read_text().strip().splitlines()
        line = json.loads(txt[-1])
        bad = 0
        for cfg, (ops, path) in res.items():
            sub = line if line["config"].get("name") == cfg else line.get("configs", {}).get(cfg)
            if sub is None:
                print(f"{cfg}: not in the JSON line")
                bad += 1
                continue
            bad += check(sub, ops, path, cfg)
        print("MATCH" if bad == 0 else f"{bad} MISMATCHES")
        sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
