#!/bin/bash
# One GPU-box pass: parity tests, the default bench line (with cpu_baseline), and a rocprofv3 kernel summary of
# the same bench command. Usage (from the repo root, via gpurun): bash scripts/gpu_check.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-run}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  "${KARG[@]}" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed: $?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 -u bench.py --no-cpu-baseline \
  > "$OUT/bench_rocprof.json" 2> "$OUT/bench_rocprof.err" || { echo "rocprof failed"; tail -20 "$OUT/bench_rocprof.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$OUT/kernel_stats.csv"
echo done
