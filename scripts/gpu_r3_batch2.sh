#!/bin/bash
# Round-3 batch 2: stable grouping (bitonic ranks) tests + KMeans shard timing and kernel trace,
# sparse SVC whole fit / steady with the always-on lazy column-major copies, the flagship bench
# with the one-replay default, then the GPU suite.
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step groupsort
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kmeans.py \
  -k "group_by_key or round_payload" > $O/kmeans_pytest.log 2>&1 || { echo "kmeans pytest failed"; tail -40 $O/kmeans_pytest.log; exit 1; }
tail -2 $O/kmeans_pytest.log
step kmeans
BENCH_PYPROFILE=1 timeout -k 10 300 python -u scripts/bench_north.py --config kmeans --scale 0.125 > $O/kmeans_shard.jsonl 2> $O/kmeans_shard_pyprof.txt || { echo km failed; tail -20 $O/kmeans_shard.jsonl $O/kmeans_shard_pyprof.txt; exit 1; }
tail -1 $O/kmeans_shard.jsonl
step svc
BENCH_PYPROFILE=1 timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 > $O/svc_shard.jsonl 2> $O/svc_pyprof.txt || { echo svc failed; tail -20 $O/svc_shard.jsonl $O/svc_pyprof.txt; exit 1; }
tail -1 $O/svc_shard.jsonl
step bench
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_20.log 2>&1 || { echo bench failed; tail -20 $O/bench_20.log; exit 1; }
tail -1 $O/bench_20.log
timeout -k 10 200 python -u bench.py > $O/bench_200.log 2>&1 || { echo bench failed; tail -20 $O/bench_200.log; exit 1; }
tail -1 $O/bench_200.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step kmeans_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/km_prof -o km -- python3 scripts/bench_north.py --config kmeans --scale 0.125 > $O/km_prof.log 2>&1 || { tail -20 $O/km_prof.log; exit 1; }
grep -h "st_\|assign\|chunk_sum" $O/km_prof/km_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
step suite
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -4 $O/gputest.log
exit $rc
