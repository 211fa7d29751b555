#!/bin/bash
# ISA of the flagship fused-round kernel (bf16, 16-byte chunks, 2 chunks per lane) for one row-loop
# variant: bash scripts/isa_glm.sh [U] [out.s]   (device-only, seconds)
U=${1:-2}; OUT=${2:-/tmp/glm_u$U.s}; SRC=$(cd "$(dirname "$0")/../flink_ml_amd/ops/csrc" && pwd)
cd /tmp && hipcc --offload-arch=gfx950 -O3 -std=c++17 --offload-device-only -S -DFMLX_ISA_PROBE -DFMLX_ISA_PROBE_U=$U \
  -mllvm -amdgpu-atomic-optimizer-strategy=None -I"$SRC" \
  "$SRC/glm.hip" -o "$OUT" 2>&1 | grep -v warning | grep -A5 error
echo "$OUT"
