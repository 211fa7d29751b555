#!/bin/bash
set -o pipefail
O=gpurun_out/r3dyn3
mkdir -p $O
timeout -k 10 120 python -u scripts/debug_dyn_state.py 2>&1 | tee $O/state.log | cut -c1-400 || exit 1
timeout -k 10 150 python -u scripts/debug_dyn_perf.py 2000000 2>&1 | tee $O/perf.log || exit 1
timeout -k 10 200 python -u scripts/debug_dyn_census.py 2>&1 | tee $O/census.jsonl | cut -c1-200 || exit 1
timeout -k 10 300 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 3 --configs "dyn=0;dyn=1" 2>&1 | tee $O/ab.jsonl || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "dynamic or flagship_shape or deferred or multi_round" 2>&1 | tee $O/pytest.log | grep -E "PASS|FAIL|ERROR|passed|failed" || exit 1
