set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_glm_sparse_gpu.py > gpurun_out/r6/t_b13.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r6/t_b13.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r6/t_b13.log | head -20; exit $rc; }
timeout -k 10 180 python -u scripts/trace_bkt_fwd.py --rounds 3 > gpurun_out/r6/trace_bkt_fwd4.jsonl 2> gpurun_out/r6/trace_bkt_fwd4.err
rc=$?; echo "trace rc=$rc"; cat gpurun_out/r6/trace_bkt_fwd4.jsonl; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6_abprof.sh 32768 || exit $?
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 > gpurun_out/r6/north_svc_b13_it10.jsonl 2> gpurun_out/r6/north_svc_b13_it10.err
rc=$?; echo "north rc=$rc"; cut -c1-420 gpurun_out/r6/north_svc_b13_it10.jsonl; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/r6/prof_chisq
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6/prof_chisq -o run_%pid% -- python3 scripts/chisq_2rank_prof.py > gpurun_out/r6/chisq_2rank.jsonl 2> gpurun_out/r6/chisq_2rank.err
rc=$?; echo "chisq rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/chisq_2rank.err; exit $rc; }
ls -R gpurun_out/r6/prof_chisq | head; python3 scripts/kstats.py gpurun_out/r6/prof_chisq 40 > gpurun_out/r6/chisq_2rank_kernels.txt; wc -l gpurun_out/r6/chisq_2rank_kernels.txt
