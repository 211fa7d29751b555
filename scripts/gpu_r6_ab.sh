set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u scripts/ab_bkt.py "$@" > gpurun_out/r6/ab_bkt.jsonl 2> gpurun_out/r6/ab_bkt.err
rc=$?; echo rc=$rc; cat gpurun_out/r6/ab_bkt.jsonl; tail -3 gpurun_out/r6/ab_bkt.err; exit $rc
