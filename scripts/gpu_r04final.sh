#!/bin/bash
# round 4 final: full GPU suite, smoke, the profiled bench with its per-launch CSV (recomputed), fresh PMC traffic of
# the A2 block, then the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04final}; mkdir -p $O
export YOLOSOD_PARITY_LOG=$O/parity_margins.txt
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o bench -- python3 -u bench.py --no-cpu-baseline \
  --ops-csv $O/ops_calls.csv > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
python3 scripts/roofline_from_csv.py $O/ops_calls.csv $O/bench_prof.json > $O/recompute.txt 2>&1; echo "recompute rc=$?"
head -14 $O/recompute.txt
bash scripts/pmc_run.sh $O/pmc a2_L12 swin_L28 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['path_roofline']['frac'], d['cpu_baseline'])
for k, c in d.get('configs', {}).items(): print(k, c['value'], c['path_roofline']['frac'])
"
