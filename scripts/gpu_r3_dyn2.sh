#!/bin/bash
set -o pipefail
O=gpurun_out/r3dyn2
mkdir -p $O
timeout -k 10 200 python -u scripts/debug_dyn_census.py > $O/census.jsonl 2>&1 || { echo census failed; tail $O/census.jsonl; exit 1; }
cat $O/census.jsonl | cut -c1-200
timeout -k 10 300 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 3 --configs "dyn=0;dyn=1;dyn=0;dyn=1" > $O/ab.jsonl 2>&1 || { echo "ab failed"; tail -20 $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "dynamic or flagship_shape or deferred or multi_round" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_rccl_gpu.py > $O/rccl.log 2>&1 || { echo "rccl failed"; tail -40 $O/rccl.log; exit 1; }
tail -8 $O/rccl.log
