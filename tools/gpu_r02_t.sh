# queued launches behind recommits and the coop commit's candidate step: parity, then n = 1e4
# for every line search with LBFGS_SPEC=0 / 1 and the paper-table comparison
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_speculative.py tests/test_gpu_stress.py tests/test_gpu_parity.py tests/test_gpu_batched_trials.py > gpurun_out/pytest_spec3.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_spec3.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_spec3.log | head -20; exit 1; }
for LS in backtracking wolfe; do for s in 0 1; do
  LBFGS_SPEC=$s timeout -k 10 120 python bench.py --size 1e4 --history 5 --line-search $LS --steps 3000 --warmup 100 --no-cpu-baseline --no-vector-free --no-prof > gpurun_out/small_${LS}_$s.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/small_${LS}_$s.json')); print('n=1e4 $LS spec=$s', d['value'], d['ms_per_step'])"
done; done
timeout -k 10 300 python tools/paper_table.py gpurun_out/paper_table.json > gpurun_out/paper_table.log 2>&1 || { tail -5 gpurun_out/paper_table.log; exit 1; }
grep -o '^[a-z_]* \|"speedup_default": [0-9.]*\|"speedup_vector_free": [0-9.]*' gpurun_out/paper_table.log | paste - - - 
