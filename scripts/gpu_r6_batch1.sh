set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u scripts/ab_bkt.py 32768,16384 > gpurun_out/r6/ab_bkt.jsonl 2> gpurun_out/r6/ab_bkt.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r6/ab_bkt.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/ab_bkt.err; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_glm_sparse_gpu.py tests/test_rccl_gpu.py tests/test_outofcore.py tests/test_catstats_gpu.py > gpurun_out/r6/t_batch1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r6/t_batch1.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r6/t_batch1.log | head -20; exit $rc; }
FMLX_BACKEND=gloo FMLX_XGMI=force timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r6/bench_gpus2_verify.log 2>&1
rc=$?; echo "bench2 rc=$rc"; tail -3 gpurun_out/r6/bench_gpus2_verify.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 > gpurun_out/r6/north_svc_bkt2.jsonl 2> gpurun_out/r6/north_svc_bkt2.err
rc=$?; echo "north rc=$rc"; cat gpurun_out/r6/north_svc_bkt2.jsonl | cut -c1-900
exit $rc
