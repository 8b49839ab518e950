#!/bin/bash
# Fresh PMC HBM traffic for every hot-path operator (the MAFN ops, the gate-fused consumer convs, the
# Detect head + decode, NMS; fp32 n640 shapes, A2 at n1280, the bf16 m-scale shapes): bash scripts/pmc_all.sh OUTDIR
# then here: python scripts/pmc_traffic.py OUTDIR > profiles/traffic.json
set -o pipefail
OUT=${1:?outdir}
bash scripts/pmc_run.sh "$OUT" swin_L28 swin_L9 a2_L12 a2_L12_1280 se_L1 cbam_L4 ca_L32 cbam_L18 se_L23 head \
  se_conv_L1 cbam_conv_L4 nms_empty nms_30k swin_L28_m swin_L9_m a2_L12_m cbam_L4_m ca_L32_m
