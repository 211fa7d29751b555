#!/bin/bash
# Round-4 LR session 1: launch-structure floor probes, shipped-kernel trace + PMC, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/bin_sp_persist > gpurun_out/r4_probe_persist.log 2>&1; echo "persist rc=$?"; cat gpurun_out/r4_probe_persist.log
timeout -k 10 120 ./scripts/bin_sp_lds > gpurun_out/r4_probe_lds.log 2>&1; echo "lds rc=$?"; cat gpurun_out/r4_probe_lds.log
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_bench_a.log 2>&1 || exit $?
cat gpurun_out/r4_bench_a.log
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/r4_lr_trace" -o run --output-format csv -- python3 "$root/bench.py" --gpus 1 --steps 20 --warmup 5) > gpurun_out/r4_lr_trace.log 2>&1 || exit $?
PMC_TAG=r4_lr PMC_CMD="python3 $root/scripts/prof_glm_round.py --rounds 30" bash scripts/gpu_prof_pmc.sh \
  "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES" \
  "SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum" \
  "FETCH_SIZE"
