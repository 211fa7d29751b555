#!/bin/bash
# Round-4 session 4: KMeans split-round overlap (kernel trace, side-stream priority), sparse SVC
# whole-fit stall (SDMA off A/B + system trace), LR block timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$(pwd)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "4 0" "4 1" "1 0"; do
  set -- $cfg
  FMLX_KMEANS_SPLIT=$1 FMLX_KMEANS_SIDE_PRIO=$2 timeout -k 10 300 python scripts/bench_north.py --config kmeans --scale 0.125 \
    >> gpurun_out/r4_kmeans_split_prio.jsonl 2>&1 || exit $?
done
grep metric gpurun_out/r4_kmeans_split_prio.jsonl | cut -c1-260
(cd /tmp && FMLX_KMEANS_SPLIT=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/r4_kmeans_split_trace" -o run \
  --output-format csv -- python3 "$root/scripts/bench_north.py" --config kmeans --scale 0.125 --iters 5) > gpurun_out/r4_kmeans_split_trace.log 2>&1 || exit $?
for sd in 1 0; do
  HSA_ENABLE_SDMA=$sd timeout -k 10 400 python scripts/bench_north.py --config svc_sparse --scale 0.125 \
    >> gpurun_out/r4_svc_sdma.jsonl 2>&1 || exit $?
done
grep metric gpurun_out/r4_svc_sdma.jsonl | cut -c1-420
(cd /tmp && timeout -k 10 400 rocprofv3 --sys-trace -d "$root/gpurun_out/r4_svc_systrace" -o run --output-format csv \
  -- python3 "$root/scripts/bench_north.py" --config svc_sparse --scale 0.125 --steady-rounds 20) > gpurun_out/r4_svc_systrace.log 2>&1 || exit $?
timeout -k 10 200 python scripts/trace_glm_blocks.py --rounds 20 > gpurun_out/r4_lr_block_timeline.jsonl 2>&1 || exit $?
tail -2 gpurun_out/r4_lr_block_timeline.jsonl
