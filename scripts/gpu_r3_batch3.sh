#!/bin/bash
# Round-3 batch 3: graph capture without empty_cache, batched CSC transpose — whole-fit timings
# (sparse SVC shard, KMeans shard + 100M), high-cardinality strings, the graph/sparse GPU tests.
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu \
  -k "sparse or svc or csc or kmeans or graph or rccl or xgmi or deferred" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
step svc
BENCH_PYPROFILE=1 timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 > $O/svc_shard.jsonl 2> $O/svc_pyprof.txt || { echo svc failed; tail -20 $O/svc_shard.jsonl $O/svc_pyprof.txt; exit 1; }
tail -1 $O/svc_shard.jsonl
step kmeans
BENCH_PYPROFILE=1 timeout -k 10 300 python -u scripts/bench_north.py --config kmeans --scale 0.125 > $O/kmeans_shard.jsonl 2> $O/kmeans_shard_pyprof.txt || { echo km failed; tail -20 $O/kmeans_shard.jsonl; exit 1; }
tail -1 $O/kmeans_shard.jsonl
timeout -k 10 400 python -u scripts/bench_north.py --config kmeans --scale 1.0 > $O/kmeans_100M.jsonl 2>&1 || { echo km100 failed; tail -20 $O/kmeans_100M.jsonl; exit 1; }
tail -1 $O/kmeans_100M.jsonl
step strings
timeout -k 10 400 python -u -m flink_ml_amd.bench.run flink_ml_amd/bench/conf/high-cardinality.json --warmup 1 \
  --output-file $O/high_cardinality.json > $O/high_cardinality.log 2>&1 || { echo strings failed; tail -20 $O/high_cardinality.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r3d/high_cardinality.json"))
for k, v in d.items():
    if k != "version":
        r = v["results"]
        print(k, round(r.get("totalTimeMs", 0), 1), round(r.get("stageTimeMs", 0), 1))
PY
