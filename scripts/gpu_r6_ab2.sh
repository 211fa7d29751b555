set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for f in 1 0; do
FMLX_BKT_FORK=$f timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6/prof_ab_f$f -o run -- python3 scripts/ab_bkt.py 32768 > gpurun_out/r6/ab_bkt_f$f.jsonl 2> gpurun_out/r6/ab_bkt_f$f.err
rc=$?; echo "fork=$f rc=$rc"; cat gpurun_out/r6/ab_bkt_f$f.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/ab_bkt_f$f.err; exit $rc; }
python3 scripts/kstats.py gpurun_out/r6/prof_ab_f$f 6
done
