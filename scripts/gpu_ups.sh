#!/bin/bash
# upsample-into-Concat HIP pass: its GPU test and the model tests, then a same-box n640 A/B against PyTorch's copy
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/ups; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_upsample.py tests/test_gpu_model.py tests/test_gpu_e2e.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    YOLOSOD_UPSAMPLE_HIP=$v timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-nms-load --no-extra-configs \
      --steps 30 --warmup 10 > $OUT/b$v$r.json 2> $OUT/b$v$r.err || { echo "bench fail $v$r"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b$v$r.json'));print('hip=$v', d['value'], d['ms_per_step'])"
  done
done
