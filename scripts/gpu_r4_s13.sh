#!/bin/bash
# Round-4 session 13: 36 KB assign blocks (gather-sum co-resident) — KMeans tests, shard A/B split 1 vs 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kmeans.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/r4_s13_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4_s13_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/prof_kmeans_assign.py --sched 4 --reps 5 2>&1 | tail -1
: > gpurun_out/r4_km_split_ab.jsonl
for sp in 1 4 1 4; do
  FMLX_KMEANS_SPLIT=$sp timeout -k 10 300 python scripts/bench_north.py --config kmeans --scale 0.125 > gpurun_out/r4_km_sp.tmp 2>&1 || exit $?
  echo "{\"split\": $sp, $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r4_km_sp.tmp)}" >> gpurun_out/r4_km_split_ab.jsonl
done
cat gpurun_out/r4_km_split_ab.jsonl
