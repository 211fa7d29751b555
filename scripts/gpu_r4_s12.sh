#!/bin/bash
# Round-4 session 12: fresh counters of the shipped KMeans assign (pipelined MFMA kernel, sched 4)
# at the north-star shard shape, + a kernel trace of the shard round.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$(pwd)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/prof_kmeans_assign.py --sched 4 --reps 5 > gpurun_out/r4_km_assign.log 2>&1 || exit $?
tail -3 gpurun_out/r4_km_assign.log
PMC_TAG=r4_km PMC_CMD="python3 $root/scripts/prof_kmeans_assign.py --sched 4 --reps 2" bash scripts/gpu_prof_pmc.sh \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/r4_km_trace" -o run --output-format csv \
  -- python3 "$root/scripts/bench_north.py" --config kmeans --scale 0.125) > gpurun_out/r4_km_trace.log 2>&1 || exit $?
grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r4_km_trace.log
