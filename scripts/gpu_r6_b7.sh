set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_rccl_gpu.py > gpurun_out/r6/t_b7.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6/t_b7.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/r6/prof_fit7
BENCH_FIT_SAMPLES=5 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r6/prof_fit7 -o run -- python3 scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 --steady-rounds 20 > gpurun_out/r6/prof_fit7.jsonl 2> gpurun_out/r6/prof_fit7.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/prof_fit7.err; exit $rc; }
python3 scripts/fit_timeline.py gpurun_out/r6/prof_fit7 > gpurun_out/r6/fit7_timeline.jsonl; cut -c1-700 gpurun_out/r6/fit7_timeline.jsonl
for it in 10 20; do
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters $it > gpurun_out/r6/north_svc_b7_it$it.jsonl 2> gpurun_out/r6/north_svc_b7_it$it.err
rc=$?; echo "north$it rc=$rc"; cut -c1-420 gpurun_out/r6/north_svc_b7_it$it.jsonl; [ $rc -eq 0 ] || exit $rc
done
