#!/bin/bash
# Round-4 session 7: radix digit-width A/B at the SVC transpose shape + PMC of the scatter pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_radix.py --bits 10,7,8 --reps 4 > gpurun_out/r4_radix_ab.jsonl 2>&1 || exit $?
cat gpurun_out/r4_radix_ab.jsonl
PMC_TAG=r4_radix PMC_CMD="python3 $(pwd)/scripts/bench_radix.py --bits 10 --reps 1 --iters 2" bash scripts/gpu_prof_pmc.sh \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR" \
  "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD TCC_HIT_sum TCC_MISS_sum" \
  "FETCH_SIZE WRITE_SIZE"
timeout -k 10 400 python -u -m pytest tests/test_radix_gpu.py tests/test_glm_sparse_gpu.py tests/test_batch_csc.py -x -v \
  --timeout 150 --timeout-method thread -m gpu > gpurun_out/r4_s7_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4_s7_tests.log; [ $rc -eq 0 ] || exit $rc
BENCH_FIT_SAMPLES=10 timeout -k 10 300 python scripts/bench_north.py --config svc_sparse --scale 0.125 > gpurun_out/r4_svc_shard_d.jsonl 2>&1 || exit $?
grep -o '"whole_fit_samples_ms[^]]*]' gpurun_out/r4_svc_shard_d.jsonl
