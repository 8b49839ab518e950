"""Static instruction mix of a kernel in a hipcc -S listing, split at s_barrier (one row per LDS stage).

usage: python scripts/isa_mix.py file.s kernel_substring [--top N]
Build the listing with: hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S -Iyolo-sod_amd/csrc -o /tmp/k.s <src>.hip
Static counts equal dynamic counts per wave for fully unrolled straight-line stages (loops are counted once).
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, key = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    text = open(path).read()
    names = [m.group(1) for m in re.finditer(r"^(\S+):\s*;\s*@", text, re.M) if key in m.group(1)]
    for name in names:
        start = text.index(f"\n{name}:") + 1
        body = text[start:text.index("s_endpgm", start)].splitlines()[1:]
        ops = [ln.strip().split()[0] for ln in body
               if ln.strip() and not ln.strip().startswith((".", ";")) and not ln.strip().endswith(":")]
        total = Counter(classify(o) for o in ops)
        print(name, dict(total))
        seg, i = Counter(), 0
        for o in ops + ["s_barrier"]:
            if o == "s_barrier":
                print(f"  stage {i:2d}: " + " ".join(f"{k}={v}" for k, v in sorted(seg.items())))
                seg, i = Counter(), i + 1
            else:
                seg[classify(o)] += 1
        vc = Counter(o for o in ops if classify(o) == "valu")
        print("  top VALU:", vc.most_common(top))
        sp = re.search(rf"{re.escape(name)}\.num_vgpr, (\d+)", text)
        print("  vgpr:", sp.group(1) if sp else "?")


if __name__ == "__main__":
    main()
