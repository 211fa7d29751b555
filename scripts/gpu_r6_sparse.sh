set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_glm_sparse_gpu.py tests/test_rccl_gpu.py > gpurun_out/r6/t_sparse.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/r6/t_sparse.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 > gpurun_out/r6/north_svc_bkt.jsonl 2> gpurun_out/r6/north_svc_bkt.err
rc=$?
echo "north rc=$rc"; tail -3 gpurun_out/r6/north_svc_bkt.err; cat gpurun_out/r6/north_svc_bkt.jsonl
exit $rc
