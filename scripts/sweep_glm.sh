#!/bin/bash
# A/B sweep of GLM kernel knobs on one GPU (one bench process per config, short runs)
for u in ${SWEEP_U:-2 4}; do for b in ${SWEEP_B:-128 256 512}; do
  echo -n "U=$u BLOCKS=$b: "
  FMLX_GLM_UNROLL=$u FMLX_GLM_BLOCKS=$b timeout -k 10 120 python bench.py --steps 200 --warmup 20 | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], r['value'], r['config']['hbm_gb_per_s'])" || exit 1
done; done
