#!/bin/bash
# U=2 grid sweep below one block per CU at the flagship shape, interleaved 4x
set -o pipefail
O=gpurun_out/r3u3
mkdir -p $O
timeout -k 10 400 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 4 \
  --configs "u=2,b=256;u=2,b=128;u=2,b=160;u=2,b=192;u=2,b=224" > $O/ab.jsonl 2>&1 || { echo "ab failed"; tail -20 $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
