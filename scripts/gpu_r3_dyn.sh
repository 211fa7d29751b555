#!/bin/bash
# Round-3 dynamic-row-schedule check: GPU tests of the fused round, interleaved A/B of the
# schedule at the flagship shape, the flagship bench and a block timeline.
set -o pipefail
O=gpurun_out/r3dyn
mkdir -p $O
timeout -k 10 200 python -u scripts/debug_dyn_census.py > $O/census.jsonl 2>&1 || { echo census failed; tail $O/census.jsonl; exit 1; }
cat $O/census.jsonl
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "dynamic or flagship_shape or deferred or multi_round" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 3 \
  --configs "dyn=0;dyn=1,ch=8;dyn=1,ch=16;dyn=1,ch=32" > $O/ab.jsonl 2>&1 || { echo "ab failed"; tail -20 $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 200 python -u scripts/trace_glm_blocks.py --rounds 20 > $O/trace.jsonl 2>&1 || { echo "trace failed"; tail -20 $O/trace.jsonl; exit 1; }
tail -2 $O/trace.jsonl
