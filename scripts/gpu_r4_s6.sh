#!/bin/bash
# Round-4 session 6: radix segments preloaded into registers, vectorised colptr — exactness, SVC whole fit (samples + kernel trace), KMeans split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$(pwd)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_radix_gpu.py tests/test_glm_sparse_gpu.py tests/test_kmeans.py \
  tests/test_batch_csc.py -x -v --timeout 150 --timeout-method thread -m gpu > gpurun_out/r4_s6_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4_s6_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_north.py --config svc_sparse --scale 0.125 > gpurun_out/r4_svc_shard_c.jsonl 2>&1 || exit $?
grep -o '"totalTimeMs[^}]*steady_samples_per_s": [0-9.]*' gpurun_out/r4_svc_shard_c.jsonl
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/r4_svc_ktrace6" -o run --output-format csv \
  -- python3 "$root/scripts/bench_north.py" --config svc_sparse --scale 0.125 --steady-rounds 20) > gpurun_out/r4_svc_ktrace6.log 2>&1 || exit $?
# the first-launch-after-idle stall: runtime-setting A/B, 10 whole fits each
for cfg in "X=0" "HSA_ENABLE_INTERRUPT=0" "HIP_FORCE_DEV_KERNARG=0" "GPU_MAX_HW_QUEUES=1"; do
  env $cfg BENCH_FIT_SAMPLES=10 timeout -k 10 300 python scripts/bench_north.py --config svc_sparse --scale 0.125 \
    --steady-rounds 20 > gpurun_out/r4_svc_stall_ab.tmp 2>&1 || exit $?
  echo "{\"env\": \"$cfg\", \"samples\": $(grep -o '"whole_fit_samples_ms": \[[^]]*\]' gpurun_out/r4_svc_stall_ab.tmp | cut -d: -f2)}" >> gpurun_out/r4_svc_stall_ab.jsonl
  tail -1 gpurun_out/r4_svc_stall_ab.jsonl
done
