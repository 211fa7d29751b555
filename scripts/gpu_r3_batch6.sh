#!/bin/bash
set -o pipefail
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_glm_sparse_gpu.py tests/test_rccl_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BENCH_PYPROFILE=1 timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 > $O/svc_shard.jsonl 2> $O/svc_pyprof.txt || { echo svc failed; tail -20 $O/svc_shard.jsonl $O/svc_pyprof.txt; exit 1; }
tail -1 $O/svc_shard.jsonl | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/svc_prof -o svc -- python3 scripts/bench_north.py --config svc_sparse --scale 0.125 > $O/svc_prof.log 2>&1 || { tail -20 $O/svc_prof.log; exit 1; }
