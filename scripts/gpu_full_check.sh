set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1e_pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r1e_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1e_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r1e_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r1e_bench1.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/r1e_bench1.log; [ $rc -eq 0 ] || exit $rc
