set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 1000 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/r6/gpu_tests_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6/gpu_tests_full.log; grep -E "FAILED|ERROR" gpurun_out/r6/gpu_tests_full.log | head -20
exit $rc
