#!/bin/bash
set -o pipefail
O=gpurun_out/r3rccl
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_rccl_gpu.py tests/test_reservoir_device.py -m gpu 2>&1 | tee $O/pytest.log | grep -E "PASS|FAIL|ERROR|passed|failed|Error" ; test ${PIPESTATUS[0]} -eq 0 || { tail -60 $O/pytest.log; exit 1; }
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 2>&1 | tee $O/bench.log | tail -1
