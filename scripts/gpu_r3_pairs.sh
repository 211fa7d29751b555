#!/bin/bash
# Round-3 pair schedule: exact-coverage + torch tests, interleaved A/B of the static fraction at
# the flagship shape, block timelines with and without pairs.
set -o pipefail
O=gpurun_out/r3pairs
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "pair_schedule or flagship_shape or deferred" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 3 \
  --configs "rm=0;rm=1;pairs=1,q=205;pairs=1,q=192,rm=1;pairs=1,q=205,rm=1;pairs=1,q=218,rm=1;pairs=1,q=230,rm=1" > $O/ab.jsonl 2>&1 || { echo "ab failed"; tail -20 $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
TRACE_PAIRS=0.8 timeout -k 10 200 python -u scripts/trace_glm_blocks.py --rounds 20 --rowmap 1 > $O/trace_pairs.jsonl 2>&1 || { echo "trace failed"; tail -20 $O/trace_pairs.jsonl; exit 1; }
tail -2 $O/trace_pairs.jsonl
