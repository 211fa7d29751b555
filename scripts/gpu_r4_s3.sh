#!/bin/bash
# Round-4 session 3: everything of session 2 plus the deferred xGMI round at 2 / 4 ranks on one GPU
# and the 2-rank flagship rehearsal (deferred vs ticketed exchange).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_radix_gpu.py tests/test_glm_sparse_gpu.py tests/test_kmeans.py \
  tests/test_batch_csc.py tests/test_xgmi_gpu.py -x -v --timeout 150 --timeout-method thread -m gpu \
  > gpurun_out/r4_s3_tests.log 2>&1
rc=$?; grep -c PASSED gpurun_out/r4_s3_tests.log; tail -6 gpurun_out/r4_s3_tests.log; [ $rc -eq 0 ] || exit $rc
for dx in 1 0; do
  FMLX_GLM_DEFER_XGMI=$dx FMLX_BACKEND=gloo FMLX_XGMI=force FMLX_DEVICE=cuda:0 timeout -k 10 300 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29517 + dx)) \
    bench.py --gpus 2 --rows 2000000 --steps 50 --warmup 10 > gpurun_out/r4_bench_2rank_defer$dx.log 2>&1 || exit $?
  grep metric gpurun_out/r4_bench_2rank_defer$dx.log | cut -c1-300
done
for sp in 4 1; do
  FMLX_KMEANS_SPLIT=$sp timeout -k 10 300 python scripts/bench_north.py --config kmeans --scale 0.125 >> gpurun_out/r4_kmeans_split_shard.jsonl 2>&1 || exit $?
done
tail -2 gpurun_out/r4_kmeans_split_shard.jsonl | cut -c1-400
timeout -k 10 400 python scripts/bench_north.py --config svc_sparse --scale 0.125 > gpurun_out/r4_svc_shard.jsonl 2>&1 || exit $?
tail -1 gpurun_out/r4_svc_shard.jsonl | cut -c1-700
AB_TAG=r4_ahead2_ab AB_CONFIGS="u=2,b=224;u=2,b=256;u=2,b=240;u=1,b=512;u=4,b=224" bash scripts/gpu_r4_dma.sh
