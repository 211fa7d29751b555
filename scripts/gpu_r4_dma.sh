#!/bin/bash
# Round-4: LDS-DMA row ring of the fused LR round — exactness first, then interleaved A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "covers_every_row or flagship_shape or shipped_default" > gpurun_out/r4_dma_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r4_dma_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_glm_kernel.py --rows 10000000 --rounds 200 --reps 3 \
  --configs "${AB_CONFIGS:-u=2,b=224;u=2,b=256;u=2,b=192;u=4,b=224;u=2,b=224,dma=3;u=1,b=512}" \
  > gpurun_out/${AB_TAG:-r4_dma_ab}.jsonl 2>&1
rc=$?; cat gpurun_out/${AB_TAG:-r4_dma_ab}.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_bench_b.log 2>&1; rc=$?; cat gpurun_out/r4_bench_b.log; exit $rc
