#!/bin/bash
# bf16 epilogue change: full GPU tests + bench (all configs); then n640 step time with the fast SiLU also for fp32
# storage (ab_push/lib_fastsilu.so) against the in-tree build, twice each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_round.sh r03x n640 || exit 1
for r in 1 2; do
  for lib in "" ab_push/lib_fastsilu.so; do
    YOLOSOD_LIB_AB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-nms-load --no-extra-configs \
      > gpurun_out/r03x/silu_$r_$(basename ${lib:-tree}).json 2>/dev/null || exit 1
    echo "${lib:-tree}: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03x/silu_$r_$(basename ${lib:-tree}).json | head -1)"
  done
done
