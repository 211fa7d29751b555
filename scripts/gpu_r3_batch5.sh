#!/bin/bash
# batch 4 (SVC fit trace, reference suite) + the 2-rank rehearsals
set -o pipefail
bash scripts/gpu_r3_multirank.sh || exit 1
bash scripts/gpu_r3_batch4.sh || exit 1
