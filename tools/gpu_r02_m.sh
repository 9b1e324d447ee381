set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stress.py -v --timeout 200 --timeout-method thread > gpurun_out/pytest_stress.log 2>&1; rc=$?
grep -E "PASS|FAIL|SKIP|Error|assert" gpurun_out/pytest_stress.log | tail -40
exit $rc
