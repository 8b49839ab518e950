#!/bin/bash
# bf16 GEMM tile-shape A/B at the L9_m shapes: 128x128 (2), 256x128 (3), 128x256 (4)
set -o pipefail
mkdir -p gpurun_out/tile
for t in 2 3 4 2 3 4; do
  echo "== tile $t"
  YOLOSOD_GEMMB_TILE=$t timeout -k 10 120 python3 -u scripts/bench_gemm.py --bf16 --no-torch 112896,1536,512 \
    112896,512,512 112896,1024,512 112896,512,1024 10240,1536,512 || exit 1
done > gpurun_out/tile/ab.txt 2>&1
