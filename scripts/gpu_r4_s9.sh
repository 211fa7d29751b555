#!/bin/bash
# Round-4 session 9: overlapped deferred LR rounds (two streams, in-kernel arrival hand-off):
# exactness, kernel A/B, bench.py both ways.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_glm_overlap_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/r4_s9_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_s9_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_glm_kernel.py --reps 5 --rounds 400 \
  --configs "u=2,b=224;u=2,b=224,ov=1;u=2,b=256,ov=1;u=1,b=512,ov=1;u=2,b=192,ov=1" > gpurun_out/r4_overlap_ab.jsonl 2>&1 || exit $?
cat gpurun_out/r4_overlap_ab.jsonl
for ov in 0 1 0 1; do
  FMLX_GLM_OVERLAP=$ov timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench_ov$ov.json 2>&1 || exit $?
  echo "ov=$ov $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4_bench_ov$ov.json)"
done
