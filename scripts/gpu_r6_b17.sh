set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_knn_gpu.py tests/test_glm_sparse_gpu.py tests/test_outofcore.py > gpurun_out/r6/t_b17.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r6/t_b17.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r6/t_b17.log | head -20; exit $rc; }
for it in 10 20; do
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters $it > gpurun_out/r6/north_svc_b17_it$it.jsonl 2> gpurun_out/r6/north_svc_b17_it$it.err
rc=$?; echo "north$it rc=$rc"; cut -c1-330 gpurun_out/r6/north_svc_b17_it$it.jsonl; [ $rc -eq 0 ] || exit $rc
done
P=/tmp/prof_ab; rm -rf $P
timeout -k 10 300 rocprofv3 --kernel-trace -d $P -o run -- python3 scripts/ab_bkt.py 32768 > gpurun_out/r6/ab_bkt.jsonl 2> gpurun_out/r6/ab_bkt.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r6/ab_bkt.jsonl; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py $P 8 | tee gpurun_out/r6/ab_bkt_kernels.txt
