# round 2: LDS row-halo exchange - full GPU suite, default bench, rocprof trace + PMC on the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile.sh 1e8 || exit 1
python tools/pmc_summary.py gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/pmc_bench_n1e8.json 1e8 | grep -E "commit|axpy|mid|trial" || true
