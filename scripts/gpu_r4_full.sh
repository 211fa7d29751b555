#!/bin/bash
# Round-4: the whole GPU suite + the 1-GPU flagship bench (driver contract) + smoke().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r4_full_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r4_full_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r4_smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench_final.json 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r4_bench_final.json
