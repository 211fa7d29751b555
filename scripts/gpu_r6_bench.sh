set -o pipefail
mkdir -p gpurun_out/r6
for i in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/bench_1gpu_$i.json 2> gpurun_out/r6/bench_1gpu_$i.err
rc=$?; echo "bench $i rc=$rc"; cat gpurun_out/r6/bench_1gpu_$i.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
FMLX_BACKEND=gloo FMLX_XGMI=force timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r6/bench_gpus2_rehearsal.json 2> gpurun_out/r6/bench_gpus2_rehearsal.err
rc=$?; echo "bench2 rc=$rc"; cat gpurun_out/r6/bench_gpus2_rehearsal.json | cut -c1-900; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/bench_gpus2_rehearsal.err; exit $rc; }
FMLX_BACKEND=gloo FMLX_XGMI=force FMLX_BENCH_INJECT_EXCHANGE_ERROR=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r6/bench_gpus2_inject.json 2> gpurun_out/r6/bench_gpus2_inject.err
echo "inject rc=$? (expected non-zero)"; cat gpurun_out/r6/bench_gpus2_inject.json | cut -c1-400; tail -2 gpurun_out/r6/bench_gpus2_inject.err
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 20 > gpurun_out/r6/north_svc_iter20.jsonl 2> gpurun_out/r6/north_svc_iter20.err
rc=$?; echo "north20 rc=$rc"; cut -c1-500 gpurun_out/r6/north_svc_iter20.jsonl
exit $rc
