#!/bin/bash
# round 4: fused A2 kernels - parity + same-box A/B + kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04i}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "a2" tests/test_gpu_split_range.py > $O/pytest_a2.log 2>&1 || { tail -30 $O/pytest_a2.log; exit 1; }
tail -1 $O/pytest_a2.log
for i in 1 2; do for f in 0 1; do
  YOLOSOD_A2_FUSED=$f timeout -k 10 120 python -u scripts/bench_ops.py a2_L12 > $O/ops_f${f}_$i.txt 2>&1 || exit 1
  echo "fused=$f: $(grep ' ms ' $O/ops_f${f}_$i.txt)"
done; done
bash scripts/prof_ops.sh ${TAG:-r04i}/prof a2_L12 | grep " us " | head -8
