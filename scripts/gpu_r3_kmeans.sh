#!/bin/bash
set -o pipefail
O=gpurun_out/r3km
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kmeans.py -m gpu 2>&1 | tee $O/pytest.log | grep -E "PASS|FAIL|ERROR|passed|failed" ; test ${PIPESTATUS[0]} -eq 0 || { tail -40 $O/pytest.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_north.py --config kmeans --scale 0.125 2>&1 | tee $O/north_shard.jsonl | tail -1 || exit 1
timeout -k 10 400 python -u scripts/bench_north.py --config kmeans --scale 1.0 2>&1 | tee $O/north_100M.jsonl | tail -1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o km -- python3 scripts/bench_north.py --config kmeans --scale 0.125 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
