set -e
cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-"--n 12500000 --d 128 --k 1024" "--n 1000003 --d 128 --k 32" "--n 2000001 --d 64 --k 256"}; do
  for sc in ${SCHEDS:-0 3}; do
    timeout -k 10 120 python3 scripts/prof_kmeans_assign.py $cfg --sched $sc --reps 10
  done
done
