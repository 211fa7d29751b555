set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 120 ./scripts/bin/micro_lds_atomic > gpurun_out/r6/micro_lds_atomic.jsonl
rc=$?; echo "micro rc=$rc"; cat gpurun_out/r6/micro_lds_atomic.jsonl; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6_abprof.sh 32768
