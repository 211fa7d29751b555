#!/bin/bash
# 224 vs 256 blocks (U=2): exactness at 224 through the default-grid tests, kernel A/B, bench.py both ways
set -o pipefail
O=gpurun_out/r3u4
mkdir -p $O
FMLX_GLM_BLOCKS=224 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "tail_prefetch or l2_replica" > $O/pytest224.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest224.log; exit 1; }
tail -1 $O/pytest224.log
timeout -k 10 300 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 4 \
  --configs "u=2,b=256;u=2,b=224;u=2,b=208;u=2,b=240" > $O/ab.jsonl 2>&1 || { echo "ab failed"; tail -20 $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
for b in 256 224 256 224; do
  FMLX_GLM_BLOCKS=$b timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench_b$b.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_b$b.log; exit 1; }
  echo "b=$b $(tail -1 $O/bench_b$b.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["kernel_us_per_step"])')"
done
