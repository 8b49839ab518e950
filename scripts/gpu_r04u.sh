#!/bin/bash
# round 4: Swin C=64 swizzled planes: tests, same-box bench_ops A/B, SQ counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04u}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_split_range.py \
  -k "swin" > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for z in 0 1; do
    echo "swz=$z rep $rep"; YOLOSOD_X3_SWZ=$z timeout -k 10 120 python3 scripts/bench_ops.py swin_L28 swin_L28_1280 2>&1 | grep " ms "
  done
done
YOLOSOD_X3_SWZ=1 bash scripts/sq_run.sh $O/sq1 swin_L28 > /dev/null && YOLOSOD_X3_SWZ=0 bash scripts/sq_run.sh $O/sq0 swin_L28 > /dev/null && \
  python3 scripts/sq_summary.py $O/sq1 | grep -A2 "swin_x3_kernel" && python3 scripts/sq_summary.py $O/sq0 | grep -A2 "swin_x3_kernel"
