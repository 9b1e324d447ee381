# round 2: host-callback call sequence (reference order / one call per point) + parity suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_callbacks.py tests/test_matrices_kat.py tests/test_cxx_dropin.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_host.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_host.log
exit $rc
