set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo start; timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6/gpu_tests_full_b15.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6/gpu_tests_full_b15.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r6/gpu_tests_full_b15.log | head -20; exit $rc; }
P=/tmp/prof_chisq; rm -rf $P
timeout -k 10 300 rocprofv3 --kernel-trace -d $P -o run_%pid% -- python3 scripts/chisq_2rank_prof.py > gpurun_out/r6/chisq_2rank.jsonl 2> gpurun_out/r6/chisq_2rank.err
rc=$?; echo "chisq rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/chisq_2rank.err; exit $rc; }
for f in $P/*.db; do echo "== $(basename $f)"; python3 scripts/kstats.py $f 80; done > gpurun_out/r6/chisq_2rank_kernels.txt; grep -ciE "sort|unique" gpurun_out/r6/chisq_2rank_kernels.txt
for it in 10 20; do
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters $it > gpurun_out/r6/north_svc_b15_it$it.jsonl 2> gpurun_out/r6/north_svc_b15_it$it.err
rc=$?; echo "north$it rc=$rc"; cut -c1-330 gpurun_out/r6/north_svc_b15_it$it.jsonl; [ $rc -eq 0 ] || exit $rc
done
