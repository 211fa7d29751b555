#!/bin/bash
# Round-4 session 8: bucket-local second pass of the column-major copy (rows, values and column
# pointers in one pass, no sorted keys) — exactness, SVC whole fits (10 samples) + kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$(pwd)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_radix_gpu.py tests/test_glm_sparse_gpu.py tests/test_batch_csc.py -x -v \
  --timeout 150 --timeout-method thread -m gpu > gpurun_out/r4_s8_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4_s8_tests.log; [ $rc -eq 0 ] || exit $rc
BENCH_FIT_SAMPLES=10 timeout -k 10 300 python scripts/bench_north.py --config svc_sparse --scale 0.125 > gpurun_out/r4_svc_shard_e.jsonl 2>&1 || exit $?
grep -o '"whole_fit_samples_ms[^]]*]' gpurun_out/r4_svc_shard_e.jsonl
FMLX_CSC_BUCKET=0 BENCH_FIT_SAMPLES=10 timeout -k 10 300 python scripts/bench_north.py --config svc_sparse --scale 0.125 > gpurun_out/r4_svc_shard_e0.jsonl 2>&1 || exit $?
grep -o '"whole_fit_samples_ms[^]]*]' gpurun_out/r4_svc_shard_e0.jsonl
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/r4_svc_ktrace8" -o run --output-format csv \
  -- python3 "$root/scripts/bench_north.py" --config svc_sparse --scale 0.125 --steady-rounds 20) > gpurun_out/r4_svc_ktrace8.log 2>&1 || exit $?
