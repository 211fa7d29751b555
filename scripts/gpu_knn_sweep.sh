set -o pipefail
export PYTHONUNBUFFERED=1
for w in 2048 4096 8192; do
  FMLX_KNN_WAVES=$w timeout -k 10 300 python -u scripts/bench_knn.py --reps 3 > gpurun_out/knn_sweep_$w.log 2>&1 || exit $?
  echo "waves=$w"; grep bench gpurun_out/knn_sweep_$w.log
done
