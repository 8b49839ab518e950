"""Static scan of hipcc -S listings for loads that wait for everything in flight.

usage: python scripts/isa_waits.py file.s [file.s ...]
Build a listing with: hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S -Iyolo-sod_amd/csrc -o /tmp/k.s <src>.hip

Two patterns, per kernel:
  phi   a global / buffer load followed within two instructions by `s_waitcnt vmcnt(0)` and a branch join: a load
        under a per-lane predicate whose result merges into a phi (the copy needs the data, so every such load waits
        for all loads in flight - and, on gfx950, for earlier stores too, which share the counter);
  full  kernels where full waits are frequent relative to loads (vmcnt(0) count >= loads / 3): a hint, not a proof.
"""
import re
import sys


def scan(fn):
    lines = open(fn).read().split("\n")
    cur, stats = None, {}
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            cur = m.group(1)
            stats[cur] = {"loads": 0, "vmcnt0": 0, "phi": 0}
            continue
        if cur is None:
            continue
        t = l.strip()
        if t.startswith(("global_load", "buffer_load")):
            stats[cur]["loads"] += 1
        elif re.match(r"s_waitcnt vmcnt\(0\)", t):
            stats[cur]["vmcnt0"] += 1
            prev = [lines[k].strip() for k in range(max(0, i - 2), i)]
            nxt = [lines[k].strip() for k in range(i + 1, min(i + 5, len(lines)))]
            if any(p.startswith(("global_load", "buffer_load")) for p in prev) and any(n.startswith(".LBB") for n in nxt):
                stats[cur]["phi"] += 1
        elif t.startswith("s_endpgm"):
            cur = None
    return stats


def main():
    for fn in sys.argv[1:]:
        for k, st in scan(fn).items():
            flags = []
            if st["phi"]:
                flags.append(f"phi {st['phi']}")
            if st["loads"] >= 4 and st["vmcnt0"] * 3 >= st["loads"]:
                flags.append(f"full {st['vmcnt0']}/{st['loads']}")
            if flags:
                print(f"{fn.split('/')[-1]:24s} {', '.join(flags):16s} {k[:100]}")


if __name__ == "__main__":
    main()
