set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
# 4 ranks sharing the one GPU: gloo for the host collectives, the in-kernel xGMI exchange forced on
FMLX_BACKEND=gloo FMLX_XGMI=force timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --rows 2000000 --steps 50 --warmup 10 \
  > gpurun_out/bench_4rank.log 2>&1; rc=$?; echo "4rank rc=$rc"; grep -E "metric|Error|error" gpurun_out/bench_4rank.log | cut -c1-600; exit $rc
