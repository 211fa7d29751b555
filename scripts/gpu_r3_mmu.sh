#!/bin/bash
# Are the ~20-35 ms whole-fit stalls queue evictions after host memory is unmapped (MMU notifier on
# pages the runtime pinned for a pageable copy)? A/B: glibc never returns large frees to the OS.
set -o pipefail
mkdir -p gpurun_out/r3j
for v in a b c; do
  BENCH_REFIT=1 timeout -k 10 200 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 \
    > gpurun_out/r3j/plain_$v.jsonl 2> gpurun_out/r3j/plain_$v.err || exit 1
  echo "plain $v $(grep -o '"totalTimeMs": [0-9.]*' gpurun_out/r3j/plain_$v.jsonl) $(grep second gpurun_out/r3j/plain_$v.err)"
  MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=68719476736 BENCH_REFIT=1 timeout -k 10 200 python -u \
    scripts/bench_north.py --config svc_sparse --scale 0.125 > gpurun_out/r3j/nomunmap_$v.jsonl 2> gpurun_out/r3j/nomunmap_$v.err || exit 1
  echo "nomunmap $v $(grep -o '"totalTimeMs": [0-9.]*' gpurun_out/r3j/nomunmap_$v.jsonl) $(grep second gpurun_out/r3j/nomunmap_$v.err)"
done
