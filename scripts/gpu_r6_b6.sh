set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_glm_sparse_gpu.py tests/test_outofcore.py tests/test_rccl_gpu.py -k "bucket or transpose_path or weighted or two_ranks or sparse or stream or rccl" > gpurun_out/r6/t_b6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6/t_b6.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r6/t_b6.log | head -20; exit $rc; }
bash scripts/gpu_r6_abprof.sh 32768 || exit $?
for it in 10 20; do
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters $it > gpurun_out/r6/north_svc_b6_it$it.jsonl 2> gpurun_out/r6/north_svc_b6_it$it.err
rc=$?; echo "north$it rc=$rc"; cut -c1-420 gpurun_out/r6/north_svc_b6_it$it.jsonl; [ $rc -eq 0 ] || exit $rc
done
