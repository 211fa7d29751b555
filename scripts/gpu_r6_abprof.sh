set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6/prof_ab -o run -- python3 scripts/ab_bkt.py "$@" > gpurun_out/r6/ab_bkt.jsonl 2> gpurun_out/r6/ab_bkt.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r6/ab_bkt.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/ab_bkt.err; exit $rc; }
python3 scripts/kstats.py gpurun_out/r6/prof_ab 12
