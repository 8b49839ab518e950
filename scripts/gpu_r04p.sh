#!/bin/bash
# round 4: per-op timings (bench_ops, fp32 + bf16 cases), fresh PMC traffic passes for the n640 hot-path ops
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04p}; mkdir -p $O
timeout -k 10 300 python3 -u scripts/bench_ops.py swin_L28 swin_L9 a2_L12 se_L1 cbam_L4 ca_L32 cbam_L18 se_L23 head \
  a2_L12_1280 > $O/ops_f32.txt 2>&1 || { tail -5 $O/ops_f32.txt; exit 1; }
cat $O/ops_f32.txt | grep " ms "
timeout -k 10 300 python3 -u scripts/bench_ops.py --bf16 swin_L28_m swin_L9_m a2_L12_m cbam_L4_m ca_L32_m \
  > $O/ops_bf16.txt 2>&1 || { tail -5 $O/ops_bf16.txt; exit 1; }
cat $O/ops_bf16.txt | grep " ms "
timeout -k 10 900 bash scripts/pmc_run.sh $O/pmc swin_L28 swin_L9 a2_L12 se_L1 cbam_L4 ca_L32 cbam_L18 se_L23 head \
  > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 scripts/pmc_traffic.py $O/pmc > $O/traffic.json && echo traffic ok
