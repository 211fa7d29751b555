#!/bin/bash
# Round-3 multi-rank rehearsals on the one GPU (ranks share cuda:0; gloo host group, xGMI exchange
# forced): flagship bench at 2 ranks (one-graph default), KMeans shard at 2 ranks (512 KB payload
# through the two-shot), sparse SVC at 2 ranks (4 MB feedback through the two-shot).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r3mr
mkdir -p $O
FMLX_BACKEND=gloo FMLX_XGMI=force FMLX_DEVICE=cuda:0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --rows 2000000 --steps 50 --warmup 10 \
  > $O/bench_2rank.log 2>&1 || { echo "bench 2rank failed"; tail -30 $O/bench_2rank.log; exit 1; }
grep metric $O/bench_2rank.log | cut -c1-400
FMLX_BACKEND=gloo FMLX_XGMI=force FMLX_DEVICE=cuda:0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29518 scripts/bench_north.py --config kmeans --scale 0.02 \
  > $O/kmeans_2rank.log 2>&1 || { echo "kmeans 2rank failed"; tail -30 $O/kmeans_2rank.log; exit 1; }
grep metric $O/kmeans_2rank.log | cut -c1-500
FMLX_BACKEND=gloo FMLX_XGMI=force FMLX_DEVICE=cuda:0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29519 scripts/bench_north.py --config svc_sparse --scale 0.02 --steady-rounds 50 \
  > $O/svc_2rank.log 2>&1 || { echo "svc 2rank failed"; tail -30 $O/svc_2rank.log; exit 1; }
grep metric $O/svc_2rank.log | cut -c1-500
