# smoke and the C++ drop-in GPU tests (CUDA-path callers, progress lines) on the closing library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_cxx_dropin.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_cxx.log 2>&1; rc=$?; tail -14 gpurun_out/pytest_cxx.log; exit $rc
