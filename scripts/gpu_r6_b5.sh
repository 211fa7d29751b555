set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_glm_sparse_gpu.py tests/test_outofcore.py tests/test_dct_gpu.py -k "f64 or bucket or transpose_path or weighted or two_ranks or sparse or stream" > gpurun_out/r6/t_b5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6/t_b5.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r6/t_b5.log | head -20; exit $rc; }
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r6/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r6/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 > gpurun_out/r6/north_svc_bkt5.jsonl 2> gpurun_out/r6/north_svc_bkt5.err
rc=$?; echo "north rc=$rc"; cut -c1-500 gpurun_out/r6/north_svc_bkt5.jsonl; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6_fitprof.sh
