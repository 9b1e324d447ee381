# refresh the small-n tables on the current build (flagged partials, speculative launches,
# cooperative limit 256): the paper's Table I comparison, the five-seed protocol, every config
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_speculative.py tests/test_gpu_parity.py > gpurun_out/pytest_spec2.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_spec2.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/paper_table.py gpurun_out/paper_table.json > gpurun_out/paper_table.log 2>&1 || { tail -5 gpurun_out/paper_table.log; exit 1; }
tail -8 gpurun_out/paper_table.log
timeout -k 10 300 python tools/seeds5.py gpurun_out/seeds5.json > gpurun_out/seeds5.log 2>&1 || { tail -5 gpurun_out/seeds5.log; exit 1; }
tail -4 gpurun_out/seeds5.log
timeout -k 10 600 python tools/bench_configs.py gpurun_out/configs.json > gpurun_out/configs.log 2>&1 || { tail -5 gpurun_out/configs.log; exit 1; }
tail -12 gpurun_out/configs.log
