set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_glm_sparse_gpu.py tests/test_rccl_gpu.py tests/test_outofcore.py -k "bucket or transpose_path or weighted or two_ranks or rccl or sparse" > gpurun_out/r6/t_bk.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6/t_bk.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r6/t_bk.log | head -20; exit $rc; }
bash scripts/gpu_r6_abprof.sh 32768 || exit $?
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 > gpurun_out/r6/north_svc_bkt3.jsonl 2> gpurun_out/r6/north_svc_bkt3.err
rc=$?; echo "north rc=$rc"; cut -c1-700 gpurun_out/r6/north_svc_bkt3.jsonl
exit $rc
