#!/bin/bash
set -o pipefail
O=gpurun_out/r3l2
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "l2_replica" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 4 \
  --configs "l2=0;l2=1;l2=0,rm=1;l2=1,rm=1" > $O/ab.jsonl 2>&1 || { echo "ab failed"; tail -20 $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
TRACE_L2ACC=1 timeout -k 10 200 python -u scripts/trace_glm_blocks.py --rounds 20 > $O/trace_l2.jsonl 2>&1 || { echo "trace failed"; tail -20 $O/trace_l2.jsonl; exit 1; }
tail -2 $O/trace_l2.jsonl
