#!/bin/bash
# Tail prefetch of the next round's rows (time-gated per wave): exactness, interleaved A/B, bench.py
set -o pipefail
O=gpurun_out/r3pf2
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "tail_prefetch" > $O/pytest_pf.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_pf.log; exit 1; }
tail -3 $O/pytest_pf.log
timeout -k 10 500 python -u scripts/bench_glm_kernel.py --rows 10000000 --reps 3 \
  --configs "pf=0;pf=2,ps=30;pf=2,ps=33;pf=4,ps=30;pf=4,ps=33;pf=8,ps=30;pf=8,ps=33;pf=4,ps=36;pf=2,ps=1000" > $O/ab.jsonl 2>&1 || { echo "ab failed"; tail -20 $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
for sc in 4 5 6 4 5; do
  timeout -k 10 200 python -u scripts/prof_kmeans_assign.py --sched $sc --reps 5 > $O/km_sched$sc.log 2>&1 || { echo "kmeans sched $sc failed"; tail -20 $O/km_sched$sc.log; exit 1; }
  tail -1 $O/km_sched$sc.log
done
