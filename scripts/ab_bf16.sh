#!/bin/bash
# Same-box A/B of bf16 cases: bash scripts/ab_bf16.sh LIB_A case [case ...]
set -o pipefail
A=${1:?lib}; shift
for r in 1 2; do
  echo "-- A ($A)"; YOLOSOD_LIB_AB=$A timeout -k 10 120 python -u scripts/bench_ops.py --bf16 "$@" 2>&1 | grep " ms " || exit 1
  echo "-- B (current)"; timeout -k 10 120 python -u scripts/bench_ops.py --bf16 "$@" 2>&1 | grep " ms " || exit 1
done
