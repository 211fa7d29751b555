set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_glm_sparse_gpu.py tests/test_outofcore.py tests/test_rccl_gpu.py > gpurun_out/r6/t_b12.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6/t_b12.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r6/t_b12.log | head -20; exit $rc; }
timeout -k 10 180 python -u scripts/trace_bkt_fwd.py --rounds 3 > gpurun_out/r6/trace_bkt_fwd3.jsonl 2> gpurun_out/r6/trace_bkt_fwd3.err
rc=$?; echo "trace rc=$rc"; cat gpurun_out/r6/trace_bkt_fwd3.jsonl; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6_abprof.sh 32768 || exit $?
for it in 10 20; do
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters $it > gpurun_out/r6/north_svc_b12_it$it.jsonl 2> gpurun_out/r6/north_svc_b12_it$it.err
rc=$?; echo "north$it rc=$rc"; cut -c1-420 gpurun_out/r6/north_svc_b12_it$it.jsonl; [ $rc -eq 0 ] || exit $rc
done
rm -rf gpurun_out/r6/prof_chisq
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6/prof_chisq -o run -- python3 scripts/chisq_2rank_prof.py > gpurun_out/r6/chisq_2rank.jsonl 2> gpurun_out/r6/chisq_2rank.err
rc=$?; echo "chisq rc=$rc"; cat gpurun_out/r6/chisq_2rank.jsonl | cut -c1-200; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/chisq_2rank.err; exit $rc; }
python3 scripts/kstats.py gpurun_out/r6/prof_chisq 40 > gpurun_out/r6/chisq_2rank_kernels.txt; ls gpurun_out/r6/prof_chisq | head
