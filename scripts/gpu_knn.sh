set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/knn_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/knn_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_knn.py > gpurun_out/knn_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; cat gpurun_out/knn_bench.log | grep bench; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_knn -o run -- python3 scripts/bench_knn.py --reps 2 > gpurun_out/prof_knn.log 2>&1; echo "prof rc=$?"
