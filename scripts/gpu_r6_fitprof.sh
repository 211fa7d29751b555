set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH_FIT_SAMPLES=5 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r6/prof_fit -o run -- python3 scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 --steady-rounds 20 > gpurun_out/r6/prof_fit.jsonl 2> gpurun_out/r6/prof_fit.err
rc=$?; echo "rc=$rc"; cut -c1-400 gpurun_out/r6/prof_fit.jsonl; exit $rc
