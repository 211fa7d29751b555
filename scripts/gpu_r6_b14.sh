set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P=/tmp/prof_chisq; rm -rf $P
timeout -k 10 300 rocprofv3 --kernel-trace -d $P -o run_%pid% -- python3 scripts/chisq_2rank_prof.py > gpurun_out/r6/chisq_2rank.jsonl 2> gpurun_out/r6/chisq_2rank.err
rc=$?; echo "chisq rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/chisq_2rank.err; exit $rc; }
for f in $P/*.db; do echo "== $(basename $f)"; python3 scripts/kstats.py $f 60; done > gpurun_out/r6/chisq_2rank_kernels.txt; wc -l gpurun_out/r6/chisq_2rank_kernels.txt
for it in 10 20; do
timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters $it > gpurun_out/r6/north_svc_b14_it$it.jsonl 2> gpurun_out/r6/north_svc_b14_it$it.err
rc=$?; echo "north$it rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
BENCH_LINETRACE=1 BENCH_FIT_SAMPLES=3 timeout -k 10 300 python -u scripts/bench_north.py --config svc_sparse --scale 0.125 --iters 10 --steady-rounds 20 > gpurun_out/r6/north_linetrace.jsonl 2> gpurun_out/r6/north_linetrace.err
rc=$?; echo "linetrace rc=$rc"; grep "lines" gpurun_out/r6/north_linetrace.err | cut -c1-900; exit $rc
