set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r03f
timeout -k 10 120 python -u tools/sleep_diag.py > gpurun_out/r03f/sleep_diag.log 2>&1; echo "sleep_diag rc=$?"; tail -2 gpurun_out/r03f/sleep_diag.log
bash tools/gpu_r03e.sh
