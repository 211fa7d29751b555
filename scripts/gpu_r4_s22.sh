#!/bin/bash
# Round-4 session 22: packed payload (low column bits beside the row) — exactness, transpose timing, SVC fits.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_glm_sparse_gpu.py tests/test_radix_gpu.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/r4_s22_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4_s22_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/debug_csc_bucket.py > gpurun_out/r4_dbg_bucket2.log 2>&1 || exit $?
grep -c "mismatches 0" gpurun_out/r4_dbg_bucket2.log
timeout -k 10 200 python scripts/bench_csc_transpose.py 2>&1 | grep "csc transpose"
BENCH_FIT_SAMPLES=10 timeout -k 10 300 python scripts/bench_north.py --config svc_sparse --scale 0.125 > gpurun_out/r4_svc_shard_g.jsonl 2>&1 || exit $?
grep -o '"whole_fit_samples_ms[^]]*]' gpurun_out/r4_svc_shard_g.jsonl
