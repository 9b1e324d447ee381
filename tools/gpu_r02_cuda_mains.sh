# the CUDA path's own main() callers (parallel-implementation/*.cu) and the C++ drop-in tests on the GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cxx_dropin.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_cxx.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_cxx.log; exit $rc
