#!/bin/bash
# Round-4 session 14: same-box A/B of the assign block's LDS footprint (36 KB now; +4 KB pad
# reproduces the old 40 KB block) x split 1 / 4, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r4_km_lds_ab.jsonl
: > $O
for rep in 1 2; do
  for pad in 0 4096; do
    for sp in 1 4; do
      FMLX_KMEANS_LDSPAD=$pad FMLX_KMEANS_SPLIT=$sp timeout -k 10 300 python scripts/bench_north.py --config kmeans --scale 0.125 \
        > gpurun_out/r4_km_sp.tmp 2>&1 || exit $?
      echo "{\"ldspad\": $pad, \"split\": $sp, $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r4_km_sp.tmp)}" >> $O
    done
  done
  for pad in 0 4096; do
    FMLX_KMEANS_LDSPAD=$pad timeout -k 10 200 python scripts/prof_kmeans_assign.py --sched 4 --reps 5 2>&1 | tail -1 | sed "s/^/ldspad=$pad /" >> gpurun_out/r4_km_assign_lds.log
  done
done
cat $O gpurun_out/r4_km_assign_lds.log
