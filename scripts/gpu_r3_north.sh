#!/bin/bash
# Round-3 north-star whole-fit measurements (1 GPU): sparse LinearSVC shard (whole fit incl. the
# trainer set-up), KMeans shard and 100M, plus a kernel trace of the KMeans shard fit.
set -o pipefail
O=gpurun_out/r3north
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "sparse or svc or csc or kmeans or group" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 > $O/svc_shard.jsonl 2>&1 || { echo svc failed; tail -20 $O/svc_shard.jsonl; exit 1; }
tail -1 $O/svc_shard.jsonl
timeout -k 10 300 python -u scripts/bench_north.py --config kmeans --scale 0.125 > $O/kmeans_shard.jsonl 2>&1 || { echo km failed; tail -20 $O/kmeans_shard.jsonl; exit 1; }
tail -1 $O/kmeans_shard.jsonl
timeout -k 10 400 python -u scripts/bench_north.py --config kmeans --scale 1.0 > $O/kmeans_100M.jsonl 2>&1 || { echo km100 failed; tail -20 $O/kmeans_100M.jsonl; exit 1; }
tail -1 $O/kmeans_100M.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o km -- python3 scripts/bench_north.py --config kmeans --scale 0.125 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv"
