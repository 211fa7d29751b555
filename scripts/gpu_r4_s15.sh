#!/bin/bash
# Round-4 session 15: is the whole-fit stall tied to freeing host memory (munmap of the previous
# fit's read-back buffers)? 10 whole fits each: default; glibc kept from returning freed memory to
# the OS; every fit's trainer and result kept alive.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r4_svc_stall_mmap_ab.jsonl
: > $O
for rep in 1 2; do
for cfg in "X=0" "MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=4294967296" "BENCH_KEEP_RESULTS=1"; do
  env $cfg BENCH_FIT_SAMPLES=10 timeout -k 10 300 python scripts/bench_north.py --config svc_sparse --scale 0.125 \
    --steady-rounds 20 > gpurun_out/r4_svc_mm.tmp 2>&1 || exit $?
  echo "{\"env\": \"$cfg\", \"samples\": $(grep -o '"whole_fit_samples_ms": \[[^]]*\]' gpurun_out/r4_svc_mm.tmp | cut -d: -f2)}" >> $O
  tail -1 $O
done
done
