# round-2 close-out on the final library: smoke, the full GPU suite, the bench line with the
# rocprofv3 kernel trace + PMC passes of the bench command
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_profile.sh 1e8 || exit 1
python tools/pmc_summary.py gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/pmc_bench_n1e8.json 1e8 > gpurun_out/pmc_summary.txt
