#!/bin/bash
# PMC passes (one rocprofv3 run per counter set) over a short program; every pass time-limited.
# usage: PMC_TAG=name PMC_CMD="python3 scripts/x.py ..." bash scripts/gpu_prof_pmc.sh "C1 C2 ..." "C3 C4 ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for set_ in "$@"; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set_ -d "$root/gpurun_out/pmc_${PMC_TAG}_$i" -o run --output-format csv -- $PMC_CMD) > "gpurun_out/pmc_${PMC_TAG}_$i.log" 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; tail -2 "gpurun_out/pmc_${PMC_TAG}_$i.log"; [ $rc -eq 0 ] || exit $rc
done
