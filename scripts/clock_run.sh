#!/bin/bash
# Effective shader clock per kernel (MI355X_MICROARCH.md, DVFS): one rocprofv3 pass of GRBM_GUI_ACTIVE (summed over
# the 8 XCDs) with the kernel trace; then python scripts/clock_summary.py OUTDIR.
#   bash scripts/clock_run.sh OUTDIR case [case ...]   (scripts/bench_ops.py cases; CLK_ARGS=--bf16 for bf16 cases)
set -o pipefail
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for c in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE,GRBM_COUNT --kernel-trace --output-format csv -d "$OUT/${c}_clk" -o clk \
    -- python3 scripts/bench_ops.py $CLK_ARGS "$c" > "$OUT/${c}_clk.txt" 2>&1 || { echo "clock pass failed for $c"; tail -5 "$OUT/${c}_clk.txt"; exit 1; }
  grep -h "ms " "$OUT/${c}_clk.txt" | tail -1
done
echo done
