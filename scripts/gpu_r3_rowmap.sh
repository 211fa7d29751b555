#!/bin/bash
# Round-3 static row-mapping A/B (glm.ROWMAP_*): interleaved timing at the flagship shape and a
# block timeline per mapping (per-XCD mean rows-done times).
set -o pipefail
O=gpurun_out/r3rowmap
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 3 \
  --configs "rm=0;rm=1;rm=2" > $O/ab.jsonl 2>&1 || { echo "ab failed"; tail -20 $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
for m in 0 1 2; do
  timeout -k 10 200 python -u scripts/trace_glm_blocks.py --rounds 20 --rowmap $m > $O/trace_rm$m.jsonl 2>&1 || { echo "trace failed"; tail -20 $O/trace_rm$m.jsonl; exit 1; }
  tail -2 $O/trace_rm$m.jsonl
done
