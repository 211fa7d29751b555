#!/bin/bash
# Round-4: KMeans GPU tests + north-star shard (12.5M x 128, k=1024) and 100M x 128 on one GPU,
# and the assign-kernel A/B at the shard shape (scripts/prof_kmeans_assign.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py tests/test_online.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_kmeans_tests.log 2>&1 || { tail -30 gpurun_out/r4_kmeans_tests.log; exit 1; }
tail -2 gpurun_out/r4_kmeans_tests.log
timeout -k 10 180 python -u scripts/prof_kmeans_assign.py --n 12500000 --d 128 --k 1024 --sched 4 --reps 10 > gpurun_out/r4_kmeans_assign.log 2>&1 || exit $?
tail -2 gpurun_out/r4_kmeans_assign.log
timeout -k 10 200 python -u scripts/bench_north.py --config kmeans --scale 0.125 > gpurun_out/r4_kmeans_shard.jsonl 2>&1 || exit $?
grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r4_kmeans_shard.jsonl
timeout -k 10 300 python -u scripts/bench_north.py --config kmeans > gpurun_out/r4_kmeans_100M.jsonl 2>&1 || exit $?
grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r4_kmeans_100M.jsonl
