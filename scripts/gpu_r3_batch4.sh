#!/bin/bash
# Round-3 batch 4: kernel trace of the sparse SVC whole fit; the whole reference suite at its
# configured sizes.
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
echo "== svc_prof $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/svc_prof -o svc -- python3 scripts/bench_north.py --config svc_sparse --scale 0.125 --steady-rounds 20 > $O/svc_prof.log 2>&1 || { tail -20 $O/svc_prof.log; exit 1; }
grep metric $O/svc_prof.log | cut -c1-300
echo "== suite $(date +%T)"
timeout -k 10 900 python -u -m flink_ml_amd.bench.run flink_ml_amd/bench/conf/reference-suite.json --warmup 1 \
  --output-file $O/reference_suite.json > $O/reference_suite.log 2>&1 || { echo suite failed; tail -30 $O/reference_suite.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r3e/reference_suite.json"))
bad = [k for k, v in d.items() if k != "version" and "exception" in v.get("results", {})]
print("configs", len(d) - 1, "exceptions", bad)
PY
