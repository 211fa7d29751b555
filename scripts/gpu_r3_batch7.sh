#!/bin/bash
# native per-batch CSC build + storage sized for the fit: sparse GPU tests, then the SVC whole fit
set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_glm_sparse_gpu.py \
  tests/test_batch_csc.py > gpurun_out/r3g/sparse_tests.log 2>&1 || { tail -30 gpurun_out/r3g/sparse_tests.log; exit 1; }
tail -3 gpurun_out/r3g/sparse_tests.log
timeout -k 10 200 python -u scripts/debug_svc_init.py > gpurun_out/r3g/svc_init.log 2>&1 || { tail -30 gpurun_out/r3g/svc_init.log; exit 1; }
cat gpurun_out/r3g/svc_init.log
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 > gpurun_out/r3g/svc_north.jsonl 2> gpurun_out/r3g/svc_north.err || { tail -30 gpurun_out/r3g/svc_north.err; exit 1; }
cat gpurun_out/r3g/svc_north.jsonl
BENCH_PYPROFILE=1 timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 > gpurun_out/r3g/svc_north_prof.jsonl 2> gpurun_out/r3g/svc_north_prof.txt
