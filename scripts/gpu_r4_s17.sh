#!/bin/bash
# Round-4 session 17: 4-slot centroid ring (DMA three tiles ahead) vs 3 — tests with the knob on,
# assign A/B and shard-round A/B, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
FMLX_KMEANS_RING=4 timeout -k 10 400 python -u -m pytest tests/test_kmeans.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/r4_s17_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4_s17_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/r4_km_ring_ab.log
: > $O
for rep in 1 2; do
  for ring in 3 4; do
    FMLX_KMEANS_RING=$ring timeout -k 10 200 python scripts/prof_kmeans_assign.py --sched 4 --reps 5 2>&1 | tail -1 | sed "s/^/ring=$ring /" >> $O
    FMLX_KMEANS_RING=$ring timeout -k 10 200 python scripts/prof_kmeans_assign.py --sched 4 --reps 5 --d 64 --k 256 --n 2000000 2>&1 | tail -1 | sed "s/^/ring=$ring /" >> $O
    FMLX_KMEANS_RING=$ring timeout -k 10 300 python scripts/bench_north.py --config kmeans --scale 0.125 > gpurun_out/r4_km_sp.tmp 2>&1 || exit $?
    echo "ring=$ring shard $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r4_km_sp.tmp)" >> $O
  done
done
cat $O
