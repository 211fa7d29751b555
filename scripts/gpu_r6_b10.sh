set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 180 python -u scripts/trace_bkt_fwd.py --rounds 4 > gpurun_out/r6/trace_bkt_fwd.jsonl 2> gpurun_out/r6/trace_bkt_fwd.err
rc=$?; echo "trace rc=$rc"; cat gpurun_out/r6/trace_bkt_fwd.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6/trace_bkt_fwd.err; exit $rc; }
