# cooperative small-group form without the broadcast barriers: parity, then n = 1e4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_speculative.py tests/test_gpu_stress.py tests/test_gpu_parity.py > gpurun_out/pytest_spec5.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_spec5.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_spec5.log | head -20; exit 1; }
for r in 1 2; do for LS in backtracking wolfe; do
  timeout -k 10 120 python bench.py --size 1e4 --history 5 --line-search $LS --steps 3000 --warmup 100 --no-cpu-baseline --no-vector-free --no-prof > gpurun_out/small_v_${LS}.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/small_v_${LS}.json')); print('n=1e4 $LS', d['value'], d['ms_per_step'])"
done; done
for N in 3e4 1e5; do
  timeout -k 10 120 python bench.py --size $N --steps 1000 --warmup 50 --no-cpu-baseline --no-vector-free --no-prof > gpurun_out/small_v_$N.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/small_v_$N.json')); print('n=$N', d['value'], d['ms_per_step'])"
done
