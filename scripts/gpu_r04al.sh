#!/bin/bash
# round 4: CA gate with its output biases staged in LDS; Detect head paired line loads: CA tests, same-box A/B (isolated op and kernel trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04al}; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/yolo-sod_amd/lib_ab/libyolosod_hip_base.so
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_bf16.py -k "ca" > $O/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  echo "base rep $rep"; YOLOSOD_LIB_AB=$BASE timeout -k 10 120 python3 scripts/bench_ops.py ca_L32 2>&1 | grep " ms "
  echo "new rep $rep"; timeout -k 10 120 python3 scripts/bench_ops.py ca_L32 2>&1 | grep " ms "
done
for lib in base new; do
  if [ $lib = base ]; then export YOLOSOD_LIB_AB=$BASE; else unset YOLOSOD_LIB_AB; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$lib -o kt -- python3 scripts/bench_ops.py ca_L32 > $O/kt_$lib.log 2>&1 || { tail -5 $O/kt_$lib.log; exit 1; }
  f=$(find $O/kt_$lib -name "kt_kernel_stats.csv" | head -1); python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'ca_' in r['Name'] or 'capool' in r['Name']: print('$lib', r['Name'][:40], r['Calls'], r['AverageNs'])"
done
# Detect head: the two 64-byte halves of each line loaded together (YOLOSOD_HEAD_PAIR=1) vs one group ahead
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_model.py -k "head" > $O/pytest_head.log 2>&1 \
  && YOLOSOD_HEAD_PAIR=1 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_model.py -k "head" >> $O/pytest_head.log 2>&1 \
  || { grep -E "FAILED|Error" $O/pytest_head.log | head -20; exit 1; }
grep passed $O/pytest_head.log
for rep in 1 2; do
  for v in 0 1; do echo "pair $v"; YOLOSOD_HEAD_PAIR=$v timeout -k 10 120 python3 scripts/bench_ops.py head 2>&1 | grep " ms "; done
done
