set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_glm_sparse_gpu.py tests/test_outofcore.py tests/test_rccl_gpu.py > gpurun_out/r6/t_b9.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6/t_b9.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r6/t_b9.log | head -20; exit $rc; }
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r6/smoke_b9.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r6/smoke_b9.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6_abprof.sh 32768 || exit $?
rm -rf gpurun_out/r6/prof_fit9
BENCH_FIT_SAMPLES=5 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r6/prof_fit9 -o run -- python3 scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 --steady-rounds 20 > gpurun_out/r6/prof_fit9.jsonl 2> gpurun_out/r6/prof_fit9.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/prof_fit9.err; exit $rc; }
python3 scripts/fit_timeline.py gpurun_out/r6/prof_fit9 > gpurun_out/r6/fit9_timeline.jsonl
for it in 10 20; do
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters $it > gpurun_out/r6/north_svc_b9_it$it.jsonl 2> gpurun_out/r6/north_svc_b9_it$it.err
rc=$?; echo "north$it rc=$rc"; cut -c1-420 gpurun_out/r6/north_svc_b9_it$it.jsonl; [ $rc -eq 0 ] || exit $rc
done
