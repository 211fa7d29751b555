set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u scripts/prof_svc_fit_host.py --first > gpurun_out/r6/svc_first_fit_host.txt 2>&1
rc=$?; echo "rc=$rc"; grep phases gpurun_out/r6/svc_first_fit_host.txt; exit $rc
