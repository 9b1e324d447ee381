# round 2: batched trials + full GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batched_trials.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_batched.log 2>&1; rc=$?
tail -20 gpurun_out/pytest_batched.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
exit $rc
