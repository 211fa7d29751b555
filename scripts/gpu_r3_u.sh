#!/bin/bash
# Rows in flight per wave (U) x grid size at the flagship shape: confirmation + bench.py both ways
set -o pipefail
O=gpurun_out/r3u2
mkdir -p $O
timeout -k 10 400 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 4 \
  --configs "u=1,b=512;u=2,b=256;u=2,b=512;u=2,b=320;u=2,b=192" > $O/ab.jsonl 2>&1 || { echo "ab failed"; tail -20 $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
for cfg in "1 512" "2 256" "1 512" "2 256"; do
  set -- $cfg
  FMLX_GLM_UNROLL=$1 FMLX_GLM_BLOCKS=$2 timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench_u$1_b$2.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_u$1_b$2.log; exit 1; }
  echo "u=$1 b=$2 $(tail -1 $O/bench_u$1_b$2.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["kernel_us_per_step"])')"
done
timeout -k 10 150 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
exit $rc
