#!/bin/bash
# PMC HBM-traffic passes per operator (one counter group per run, as the MI355X guide prescribes):
#   bash scripts/pmc_run.sh OUTDIR case [case ...]     (cases: scripts/bench_ops.py CASES)
# then here: python scripts/pmc_traffic.py OUTDIR > profiles/traffic.json
set -o pipefail
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for c in "$@"; do
  bf=""; case "$c" in *_m) bf="--bf16";; esac  # the bf16 config's cases
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/${c}_f" -o f -- python3 scripts/bench_ops.py "$c" $bf \
    > "$OUT/${c}_f.txt" 2>&1 || { echo "FETCH pass failed for $c"; tail -5 "$OUT/${c}_f.txt"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/${c}_w" -o w -- python3 scripts/bench_ops.py "$c" $bf \
    > "$OUT/${c}_w.txt" 2>&1 || { echo "WRITE pass failed for $c"; tail -5 "$OUT/${c}_w.txt"; exit 1; }
  grep -h "ms " "$OUT/${c}_f.txt" | tail -1
done
echo done
