#!/bin/bash
# round 4: full GPU suite + the profiled bench with its per-launch CSV (hip_ops recomputable from it)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04o}; mkdir -p $O
export YOLOSOD_PARITY_LOG=$O/parity_margins.txt
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o bench -- python3 -u bench.py --no-cpu-baseline \
  --ops-csv $O/ops_calls.csv > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
python3 scripts/roofline_from_csv.py $O/ops_calls.csv $O/bench.json > $O/recompute.txt 2>&1; echo "recompute rc=$?"
cat $O/recompute.txt | head -60
