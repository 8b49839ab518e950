#!/bin/bash
# round 4: bf16 GEMM with two tiles of register lookahead: bf16 tests, same-box A/B, kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04ak}; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/yolo-sod_amd/lib_ab/libyolosod_hip_base.so
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf16.py > $O/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  echo "base rep $rep"; YOLOSOD_LIB_AB=$BASE timeout -k 10 120 python3 scripts/bench_ops.py --bf16 swin_L9_m a2_L12_m 2>&1 | grep " ms "
  echo "new rep $rep"; timeout -k 10 120 python3 scripts/bench_ops.py --bf16 swin_L9_m a2_L12_m 2>&1 | grep " ms "
done
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $O/kt -o kt -- python3 scripts/bench_ops.py --bf16 swin_L9_m > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 - <<PY
import csv, glob
rows=list(csv.DictReader(open(glob.glob('$O/kt/**/kt_kernel_trace.csv', recursive=True)[0])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
for r in [r for r in rows if 'gemm_bf16' in r['Kernel_Name']][-5:]:
    print(round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000,1), r['Grid_Size_X'], r['Kernel_Name'][:50])
PY
