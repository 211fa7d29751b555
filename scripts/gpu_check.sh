#!/bin/bash
# GPU validation run used with gpurun: tests, bench, profile. Stops at the first GPU fault/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_testfail() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }

STEPS="${STEPS:-tests bench prof}"
for step in $STEPS; do
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
      ok_or_testfail $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/${PROF_SCRIPT:-bench.py}" ${PROF_ARGS:---steps 50 --warmup 5}) > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc ;;
    extra)
      timeout -k 10 900 bash -c "${EXTRA_CMD}" > gpurun_out/extra.log 2>&1
      rc=$?; echo "extra rc=$rc"; tail -20 gpurun_out/extra.log; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
