#!/bin/bash
# Round-4 session 10: the multi-rank sparse SVC round split (ranks share the one GPU: gloo host
# group, xGMI exchange forced) — 1 rank, 2 ranks, 2 ranks with the RCCL-free gloo all-reduce.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r4_svc_mr.jsonl
: > $O
FMLX_DEVICE=cuda:0 timeout -k 10 200 python scripts/svc_multirank_breakdown.py >> $O 2> gpurun_out/r4_svc_mr1.err || exit $?
FMLX_BACKEND=gloo FMLX_XGMI=force FMLX_DEVICE=cuda:0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 scripts/svc_multirank_breakdown.py >> $O 2> gpurun_out/r4_svc_mr2.err || exit $?
FMLX_BACKEND=gloo FMLX_XGMI=0 FMLX_DEVICE=cuda:0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 scripts/svc_multirank_breakdown.py >> $O 2> gpurun_out/r4_svc_mr3.err || exit $?
cat $O
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py -x -q --timeout 150 --timeout-method thread -m gpu -k "two_ranks or twoshot or two_shot or oneshot or allreduce or exchange" > gpurun_out/r4_s10_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_s10_tests.log; exit $rc
