#!/bin/bash
# Round-4 session 11: full xGMI suite after the fence change + 2/4-rank LR and 2-rank KMeans rehearsals.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for w in 2 4; do
  FMLX_BACKEND=gloo FMLX_XGMI=force FMLX_DEVICE=cuda:0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $w --master-addr 127.0.0.1 --master-port 2954$w bench.py --gpus $w --rows 2000000 --steps 50 --warmup 10 \
    > gpurun_out/r4_bench_${w}rank.log 2>&1 || exit $?
  grep -o '"ms_per_step": [0-9.]*, "kernel_us_per_step": [0-9.]*' gpurun_out/r4_bench_${w}rank.log
done
FMLX_BACKEND=gloo FMLX_XGMI=force FMLX_DEVICE=cuda:0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 scripts/bench_north.py --config kmeans --scale 0.02 \
  > gpurun_out/r4_kmeans_2rank.log 2>&1 || exit $?
grep -o '"totalTimeMs[^}]*tflops_per_s": [0-9.]*' gpurun_out/r4_kmeans_2rank.log
