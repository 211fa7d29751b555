#!/bin/bash
# PMC passes of the sparse SVC round kernels (cell forward, tiled backward) over bench_north steady
# rounds, one rocprofv3 run per counter set, each under its own KILL timeout (profiles/r5/svc_cell_round_pmc.json)
set -u
cd "$GRAFT_REPO_ROOT"
root=$(pwd)
mkdir -p gpurun_out/cellpmc
export TMPDIR=/tmp
i=0
run() {  # tag cmd counters...
  local tag=$1; shift; local cmd=$1; shift
  for set_ in "$@"; do
    i=$((i + 1))
    (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $set_ -d "$root/gpurun_out/cellpmc/${tag}_$i" -o run --output-format csv -- $cmd) > "$root/gpurun_out/cellpmc/${tag}_$i.log" 2>&1
    rc=$?; echo "$tag pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
run svc "python3 $root/scripts/bench_north.py --config svc_sparse --scale 0.125 --steady-rounds 40" \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY" \
  "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
  "SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM TCC_MISS_sum TCC_EA0_RDREQ_sum"
