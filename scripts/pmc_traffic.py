"""HBM traffic per operator call from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE), gfx950-corrected.

Collected on the GPU box as separate passes, one operator per process, with scripts/bench_ops.py (13 calls:
3 warm-up + 10 timed):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/<case>_f -o f -- python scripts/bench_ops.py <case>
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/<case>_w -o w -- python scripts/bench_ops.py <case>

then here:  python scripts/pmc_traffic.py gpurun_out/pmc > profiles/traffic.json

Correction (MI355X_MICROARCH.md, HBM section): both counters are in KiB; FETCH_SIZE reports half the bytes of a
16-B-per-lane streaming read, so reads are counted as 2 x FETCH_SIZE. Only the library's own kernels (ys::*,
fold_bn_kernel) are summed; the total over the process is divided by the number of operator calls.
"""
import csv
import glob
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from bench_ops import CASES  # noqa: E402

OPKEY = {"SwinBlock": "swin", "A2_Attn": "a2", "SE_Block": "se", "CBAM_Block": "cbam", "CA_Block": "ca",
         "MambaBlock": "mamba", "detect_head": "head", "gated_se": "se_conv", "gated_cbam": "cbam_conv", "nms": "nms"}
CALLS = 13


def counter_total(d, counter):
    files = glob.glob(str(Path(d) / "**" / "*counter_collection.csv"), recursive=True)
    if not files:
        return None
    tot = 0.0
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if r.get("Counter_Name") != counter:
                continue
            # the operator's own kernels; bias_act* is the producer epilogue bench_ops.py runs once to attach the
            # gate statistics to x (as in the model) and is not part of the operator call
            if ("ys::" in name or "fold_bn_kernel" in name) and "bias_act" not in name:
                tot += float(r["Counter_Value"])
    return tot


def main():
    root = Path(sys.argv[1])
    out = {}
    for case, (cls, _, shape) in CASES.items():
        f = counter_total(root / f"{case}_f", "FETCH_SIZE")
        w = counter_total(root / f"{case}_w", "WRITE_SIZE")
        if f is None or w is None:
            continue
        per_call = (2.0 * f + w) * 1024.0 / CALLS
        key_shape = shape if cls != "detect_head" else (shape[0], 34000 * (shape[2] // 640) ** 2)
        if cls == "nms":  # key shape (B, nc, A); the bench's NMS (random init) is the empty one
            key_shape = (shape[0], shape[1] - 4, shape[2])
        if cls != "nms" or case == "nms_empty":
            out[f"{OPKEY[cls]}:{'x'.join(map(str, key_shape))}"] = round(per_call)
        out[f"_detail:{case}"] = {"read_bytes_per_call": round(2.0 * f * 1024.0 / CALLS),
                                  "write_bytes_per_call": round(w * 1024.0 / CALLS)}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
