#!/bin/bash
# Round-4 session 18: KMeans north-star config 3 on one GPU (100M x 128, k = 1024, 10 iterations).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python scripts/bench_north.py --config kmeans --scale 1.0 > gpurun_out/r4_km_100M.jsonl 2>&1 || exit $?
grep -o '"totalTimeMs[^}]*tflops_per_s": [0-9.]*' gpurun_out/r4_km_100M.jsonl
