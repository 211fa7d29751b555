#!/bin/bash
set -o pipefail
O=gpurun_out/r3km2
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_reservoir_device.py -m gpu 2>&1 | tail -2 || exit 1
timeout -k 10 200 python -u scripts/bench_reservoir.py 2>&1 | tee $O/reservoir.jsonl || exit 1
timeout -k 10 300 python -u scripts/bench_north.py --config kmeans --scale 0.125 2>&1 | tee $O/north_shard.jsonl | tail -1 || exit 1
timeout -k 10 400 python -u scripts/bench_north.py --config kmeans --scale 1.0 2>&1 | tee $O/north_100M.jsonl | tail -1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o km -- python3 scripts/bench_north.py --config kmeans --scale 0.125 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv"
