set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r6/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r6/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6_abprof.sh 32768 || exit $?
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 > gpurun_out/r6/north_svc_bkt4.jsonl 2> gpurun_out/r6/north_svc_bkt4.err
rc=$?; echo "north rc=$rc"; cut -c1-600 gpurun_out/r6/north_svc_bkt4.jsonl
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 20 > gpurun_out/r6/north_svc_bkt4_iter20.jsonl 2> gpurun_out/r6/north_svc_bkt4_iter20.err
rc=$?; echo "north20 rc=$rc"; cut -c1-600 gpurun_out/r6/north_svc_bkt4_iter20.jsonl
exit $rc
