#!/bin/bash
# Interleaved A/B of the round kernel's grid size on one box (bench.py, 200 steps, 3 repeats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do for b in ${AB_BLOCKS:-256 512}; do
  echo -n "rep=$rep BLOCKS=$b: "
  FMLX_GLM_BLOCKS=$b timeout -k 10 120 python bench.py --steps 200 --warmup 20 2>/dev/null | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], r['kernel_us_per_step'])" || exit 1
done; done
