#!/bin/bash
# 64-bit payload CSC transposes: sparse GPU tests, SVC whole fit (idle-before / refit diagnostics)
set -o pipefail
mkdir -p gpurun_out/r3i
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_glm_sparse_gpu.py \
  tests/test_batch_csc.py > gpurun_out/r3i/sparse_tests.log 2>&1 || { tail -30 gpurun_out/r3i/sparse_tests.log; exit 1; }
tail -2 gpurun_out/r3i/sparse_tests.log
for v in 0 50 500; do
  BENCH_REFIT=1 BENCH_PRESLEEP_MS=$v timeout -k 10 200 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 \
    > gpurun_out/r3i/svc_sl$v.jsonl 2> gpurun_out/r3i/svc_sl$v.err || { tail -20 gpurun_out/r3i/svc_sl$v.err; exit 1; }
  echo "sleep=$v $(grep -o '"totalTimeMs": [0-9.]*' gpurun_out/r3i/svc_sl$v.jsonl) $(grep second gpurun_out/r3i/svc_sl$v.err)"
done
