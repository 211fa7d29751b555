#!/bin/bash
# Round-4 session 16: whole SVC fits with no device->host copy before the final read-back
# (batch bounds cached per indptr) — 10 samples x 3 processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r4_svc_nosync.jsonl
: > $O
for rep in 1 2; do
  BENCH_WARM_FITS=${WARM:-0} BENCH_FIT_SAMPLES=10 timeout -k 10 300 python scripts/bench_north.py --config svc_sparse --scale 0.125 \
    --steady-rounds 20 > gpurun_out/r4_svc_ns.tmp 2>&1 || exit $?
  echo "{\"samples\": $(grep -o '"whole_fit_samples_ms": \[[^]]*\]' gpurun_out/r4_svc_ns.tmp | cut -d: -f2)}" >> $O
  tail -1 $O
done
