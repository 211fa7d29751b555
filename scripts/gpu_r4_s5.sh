#!/bin/bash
# Round-4 session 5: LDS-staged radix scatter — exactness, SVC whole fit (samples + kernel trace), KMeans split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$(pwd)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_radix_gpu.py tests/test_glm_sparse_gpu.py tests/test_kmeans.py \
  tests/test_batch_csc.py -x -v --timeout 150 --timeout-method thread -m gpu > gpurun_out/r4_s5_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4_s5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_north.py --config svc_sparse --scale 0.125 > gpurun_out/r4_svc_shard_b.jsonl 2>&1 || exit $?
grep -o '"totalTimeMs[^}]*steady_samples_per_s": [0-9.]*' gpurun_out/r4_svc_shard_b.jsonl
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/r4_svc_ktrace" -o run --output-format csv \
  -- python3 "$root/scripts/bench_north.py" --config svc_sparse --scale 0.125 --steady-rounds 20) > gpurun_out/r4_svc_ktrace.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_north.py --config kmeans --scale 0.125 > gpurun_out/r4_kmeans_shard_c.jsonl 2>&1 || exit $?
grep -o '"totalTimeMs[^}]*tflops_per_s": [0-9.]*' gpurun_out/r4_kmeans_shard_c.jsonl
