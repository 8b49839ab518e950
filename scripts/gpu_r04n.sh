#!/bin/bash
# round 4: full GPU suite (parity log) + default bench line + rocprof kernel summary of the same bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04n}; mkdir -p $O
export YOLOSOD_PARITY_LOG=$O/parity_margins.txt
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -30; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['path_roofline']['frac'], d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)
for o in d['hip_ops']: print(o['op'], o['shape'], o['avg_ms'], o['frac'])
for k, c in d.get('configs', {}).items(): print(k, c['value'], c['path_roofline']['frac'])
"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o bench -- python3 -u bench.py --no-cpu-baseline --no-nms-load --no-extra-configs > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
echo done
