set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u scripts/prof_svc_fit_host.py > gpurun_out/r6/svc_fit_host_profile.txt 2>&1
rc=$?; echo "host rc=$rc"; head -c 1800 gpurun_out/r6/svc_fit_host_profile.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6_fitprof.sh
