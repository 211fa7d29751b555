#!/bin/bash
# Round-4 session 19: the bf16 row loop issuing a buffer's next loads right after widening it —
# exactness, kernel A/B (interleaved), bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_glm_gpu.py -x -q --timeout 150 --timeout-method thread -m gpu \
  > gpurun_out/r4_s19_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4_s19_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_glm_kernel.py --reps 7 --rounds 400 \
  --configs "u=2,b=224,early=1;u=2,b=224,early=0;u=1,b=512,early=1;u=1,b=512,early=0;u=2,b=256,early=1" > gpurun_out/r4_early_ab.jsonl 2>&1 || exit $?
cat gpurun_out/r4_early_ab.jsonl
for e in 1 0 1 0; do
  FMLX_GLM_EARLY=$e timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench_e$e.json 2>&1 || exit $?
  echo "early=$e $(grep -o '"ms_per_step": [0-9.]*, "kernel_us_per_step": [0-9.]*' gpurun_out/r4_bench_e$e.json)"
done
