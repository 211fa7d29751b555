#!/bin/bash
# Tail prefetch of the next round's rows: exactness, interleaved A/B, bench.py both ways, GPU suite
set -o pipefail
O=gpurun_out/r3pf
mkdir -p $O
timeout -k 10 150 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "tail_prefetch" > $O/pytest_pf.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_pf.log; exit 1; }
tail -3 $O/pytest_pf.log
timeout -k 10 400 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 3 \
  --configs "pf=0;pf=2;pf=4;pf=8;pf=16;pf=4,ps=200;pf=8,ps=250" > $O/ab.jsonl 2>&1 || { echo "ab failed"; tail -20 $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
for pf in 0 4 0 4; do
  FMLX_GLM_PF=$pf timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench_pf$pf.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_pf$pf.log; exit 1; }
  echo "pf=$pf $(tail -1 $O/bench_pf$pf.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["kernel_us_per_step"])')"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
exit $rc
