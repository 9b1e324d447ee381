# round 2: dense quadratic objective on the device + C++ drop-in + full GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_cxx_dropin.py -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|mat500" gpurun_out/pytest_dense.log | tail -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
exit $rc
