# Round-end checks on one MI355X (run from the repo root through gpurun): the GPU suite, smoke(),
# the flagship bench in the driver's form and the default form, and the sparse-SVC whole-fit
# north-star record. Every step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out/check
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo start
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/check/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/check/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/check/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/check/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/check/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/check/bench_20x5.json 2> gpurun_out/check/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/check/bench_20x5.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/check/bench_default.json 2>> gpurun_out/check/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
for it in 10 20; do
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters $it > gpurun_out/check/north_svc_it$it.jsonl 2> gpurun_out/check/north_svc.err
rc=$?; echo "north$it rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
