#!/bin/bash
# Round-4 session 23: final SVC whole-fit kernel timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$(pwd)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r4_svc_ktrace9
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/r4_svc_ktrace9" -o run --output-format csv \
  -- python3 "$root/scripts/bench_north.py" --config svc_sparse --scale 0.125 --steady-rounds 20) > gpurun_out/r4_svc_ktrace9.log 2>&1 || exit $?
grep -o '"whole_fit_samples_ms[^]]*]' gpurun_out/r4_svc_ktrace9.log
