set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u scripts/bench_outofcore_sparse.py > gpurun_out/r6/ooc_svc_sparse_budget1G.jsonl 2> gpurun_out/r6/ooc_svc_sparse.err
rc=$?; echo "ooc rc=$rc"; cat gpurun_out/r6/ooc_svc_sparse_budget1G.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/ooc_svc_sparse.err; exit $rc; }
P=/tmp/prof_fit; rm -rf $P
BENCH_FIT_SAMPLES=5 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $P -o run -- python3 scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 --steady-rounds 20 > gpurun_out/r6/prof_fit_final.jsonl 2> gpurun_out/r6/prof_fit_final.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/prof_fit_final.err; exit $rc; }
python3 scripts/fit_timeline.py $P > gpurun_out/r6/fit_timeline_final.jsonl; python3 scripts/kstats.py $P 25 > gpurun_out/r6/north_svc_final_kernels.txt; cut -c1-300 gpurun_out/r6/fit_timeline_final.jsonl
timeout -k 10 300 python -u bench.py > gpurun_out/r6/bench_1gpu_final.json 2> gpurun_out/r6/bench_1gpu_final.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r6/bench_1gpu_final.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r6/smoke_final.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r6/smoke_final.log; exit $rc
