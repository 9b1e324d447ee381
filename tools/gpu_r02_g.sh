# round 2: full GPU suite after the ADVICE fixes (coop occupancy clamp, VF geometry edges)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_gpu.log
exit $rc
