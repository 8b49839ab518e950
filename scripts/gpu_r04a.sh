#!/bin/bash
# round 4: Swin C=64 split at the attention residual - parity + same-box A/B + kernel trace
set -o pipefail
cd /root/repo
O=gpurun_out/r04a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "swin" tests/test_gpu_split_range.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for i in 1 2; do
  for s in 0 1; do
    YOLOSOD_SWIN_SPLIT=$s timeout -k 10 120 python -u scripts/bench_ops.py swin_L28 swin_L28_1280 > $O/ops_s${s}_$i.txt 2>&1 || exit 1
    echo "split=$s run $i"; cat $O/ops_s${s}_$i.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d /root/repo/$O/prof -o run -- python3 /root/repo/scripts/bench_ops.py swin_L28 > /root/repo/$O/prof.log 2>&1 || exit 1
find /root/repo/$O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} /root/repo/$O/kernel_stats.csv
head -12 /root/repo/$O/kernel_stats.csv | cut -c1-220
