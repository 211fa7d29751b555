#!/bin/bash
# Round-4 session 2: segmented radix sort exactness + sparse/KMeans users, LR loop A/B + bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_radix_gpu.py tests/test_glm_sparse_gpu.py tests/test_kmeans.py tests/test_batch_csc.py -x -v \
  --timeout 120 --timeout-method thread -m gpu > gpurun_out/r4_s2_tests.log 2>&1
rc=$?; tail -8 gpurun_out/r4_s2_tests.log; [ $rc -eq 0 ] || exit $rc
for sp in 4 1; do
  FMLX_KMEANS_SPLIT=$sp timeout -k 10 300 python scripts/bench_north.py --config kmeans --scale 0.125 >> gpurun_out/r4_kmeans_split_shard.jsonl 2>&1 || exit $?
done
tail -2 gpurun_out/r4_kmeans_split_shard.jsonl
AB_TAG=r4_ahead2_ab AB_CONFIGS="u=2,b=224;u=2,b=256;u=2,b=240;u=1,b=512;u=4,b=224" bash scripts/gpu_r4_dma.sh
