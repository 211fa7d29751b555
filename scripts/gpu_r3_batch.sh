#!/bin/bash
# Round-3 measurement batch (1 GPU): xGMI two-shot rehearsal tests, north-star whole fits (sparse
# SVC shard, KMeans shard + 100M), high-cardinality string stages, OnlineLR host ingest over 200
# batches with a copy/kernel overlap trace, KMeans shard kernel trace, then the GPU suite.
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step xgmi
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "allreduce" > $O/xgmi_pytest.log 2>&1 || { echo "xgmi pytest failed"; tail -40 $O/xgmi_pytest.log; exit 1; }
tail -3 $O/xgmi_pytest.log
step groupsort
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kmeans.py \
  -k "group_by_key or round_payload" > $O/kmeans_pytest.log 2>&1 || { echo "kmeans pytest failed"; tail -40 $O/kmeans_pytest.log; exit 1; }
tail -3 $O/kmeans_pytest.log
step svc
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 > $O/svc_shard.jsonl 2>&1 || { echo svc failed; tail -20 $O/svc_shard.jsonl; exit 1; }
tail -1 $O/svc_shard.jsonl
step kmeans
timeout -k 10 300 python -u scripts/bench_north.py --config kmeans --scale 0.125 > $O/kmeans_shard.jsonl 2>&1 || { echo km failed; tail -20 $O/kmeans_shard.jsonl; exit 1; }
tail -1 $O/kmeans_shard.jsonl
timeout -k 10 400 python -u scripts/bench_north.py --config kmeans --scale 1.0 > $O/kmeans_100M.jsonl 2>&1 || { echo km100 failed; tail -20 $O/kmeans_100M.jsonl; exit 1; }
tail -1 $O/kmeans_100M.jsonl
step strings
timeout -k 10 400 python -u -m flink_ml_amd.bench.run flink_ml_amd/bench/conf/high-cardinality.json --warmup 1 \
  --output-file $O/high_cardinality.json > $O/high_cardinality.log 2>&1 || { echo strings failed; tail -20 $O/high_cardinality.log; exit 1; }
grep -E "stageTimeMs" -o $O/high_cardinality.log | head -1; grep -E "^[a-z-]+1Mdistinct:" $O/high_cardinality.log | cut -c1-220
step online
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/online_prof -o ol -- python3 scripts/bench_north.py --config online_lr --host-stream --iters 200 > $O/online_host.jsonl 2>&1 || { echo online failed; tail -20 $O/online_host.jsonl; exit 1; }
grep metric $O/online_host.jsonl | tail -1
python scripts/trace_overlap.py $O/online_prof > $O/online_overlap.json && cat $O/online_overlap.json
step kmeans_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/km_prof -o km -- python3 scripts/bench_north.py --config kmeans --scale 0.125 > $O/km_prof.log 2>&1 || { tail -20 $O/km_prof.log; exit 1; }
find $O/km_prof -name "*kernel_stats.csv" | head -2
step suite
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -4 $O/gputest.log
exit $rc
