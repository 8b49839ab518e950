#!/bin/bash
# SQ (shader-sequencer) counter passes per operator, one 8-counter group per run:
#   bash scripts/sq_run.sh OUTDIR case [case ...]      (cases: scripts/bench_ops.py CASES; SQ_ARGS=--bf16 for the
#   bf16 cases)
# then here: python scripts/sq_summary.py OUTDIR
set -o pipefail
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
A=SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_ANY,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU
B=SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_SALU,SQ_VALU_MFMA_COEXEC_CYCLES,SQ_INSTS_VMEM
for c in "$@"; do
  for p in A B; do
    timeout -s KILL 90 rocprofv3 --pmc ${!p} --output-format csv -d "$OUT/${c}_$p" -o $p -- python3 scripts/bench_ops.py $SQ_ARGS "$c" \
      > "$OUT/${c}_$p.txt" 2>&1 || { echo "pass $p failed for $c"; tail -5 "$OUT/${c}_$p.txt"; exit 1; }
  done
  grep -h "ms " "$OUT/${c}_A.txt" | tail -1
done
echo done
