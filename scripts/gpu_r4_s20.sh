#!/bin/bash
# Round-4 session 20: the column-major copy alone — timing (bucket vs LSD) and counters of its kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$(pwd)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/bench_csc_transpose.py > gpurun_out/r4_csc_t.log 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_csc_transpose.py --lsd >> gpurun_out/r4_csc_t.log 2>&1 || exit $?
grep "csc transpose" gpurun_out/r4_csc_t.log
PMC_TAG=r4_csc PMC_CMD="python3 $root/scripts/bench_csc_transpose.py --iters 2" bash scripts/gpu_prof_pmc.sh \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR" \
  "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" || exit $?
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/r4_csc_trace" -o run --output-format csv \
  -- python3 "$root/scripts/bench_csc_transpose.py" --iters 3) > gpurun_out/r4_csc_trace.log 2>&1 || exit $?
