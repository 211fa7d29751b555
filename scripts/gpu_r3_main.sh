#!/bin/bash
# Round-3 session check: smoke, flagship bench, row-mapping A/B, then the GPU test suite.
set -o pipefail
O=gpurun_out/r3main
mkdir -p $O
timeout -k 10 150 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
bash scripts/gpu_r3_rowmap.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
exit $rc
