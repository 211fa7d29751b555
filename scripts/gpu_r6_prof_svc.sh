set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH_FIT_SAMPLES=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_svc -o run -- python3 scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 --steady-rounds 50 > gpurun_out/r6/prof_svc.jsonl 2> gpurun_out/r6/prof_svc.err
rc=$?
echo "rc=$rc"
find gpurun_out/r6/prof_svc -name "*kernel_stats.csv" | head
exit $rc
