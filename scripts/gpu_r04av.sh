#!/bin/bash
# round 4: fp32 GEMM with 64x64 tiles (YOLOSOD_GEMM_TILE=4) vs the default choice: A2 tests under the forced tile, A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04av}; mkdir -p $O
YOLOSOD_GEMM_TILE=4 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "a2" > $O/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in 0 4; do echo "tile $t"; YOLOSOD_GEMM_TILE=$t timeout -k 10 120 python3 scripts/bench_ops.py a2_L12 a2_L12_1280 2>&1 | grep " ms "; done
done
