#!/bin/bash
set -o pipefail
O=gpurun_out/r3xgmi
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "allreduce" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -6 $O/pytest.log
