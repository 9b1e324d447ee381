# round 2, first GPU pass: GPU suite, smoke, rocprof trace + PMC, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
bash tools/gpu_profile.sh 1e8
