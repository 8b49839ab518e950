#!/bin/bash
# round 4: fused A2 (LN -> QKV -> attention) parity + A/B + kernel trace, then the full GPU suite and the bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04h; mkdir -p $O
export YOLOSOD_PARITY_LOG=$O/parity_margins.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "a2" tests/test_gpu_split_range.py tests/test_gpu_e2e.py > $O/pytest_a2.log 2>&1 || { tail -30 $O/pytest_a2.log; exit 1; }
tail -2 $O/pytest_a2.log
for i in 1 2; do for f in 0 1; do
  YOLOSOD_A2_FUSED=$f timeout -k 10 120 python -u scripts/bench_ops.py a2_L12 > $O/ops_f${f}_$i.txt 2>&1 || exit 1
  echo "fused=$f: $(grep ' ms ' $O/ops_f${f}_$i.txt)"
done; done
bash scripts/prof_ops.sh r04h/prof a2_L12 || exit 1
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -30; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['path_roofline'])
for o in d['hip_ops']: print(o['op'], o['shape'], o['avg_ms'], o['frac'])
for k, c in d.get('configs', {}).items(): print(k, c['value'], c['path_roofline']['frac'])
"
exit $rc
