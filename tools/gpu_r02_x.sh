# ticket launches' completion words (host waits without a stream sync): parity, then n = 1e4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_x.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_x.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_x.log | head -20; exit 1; }
for r in 1 2; do for LS in backtracking wolfe; do
  timeout -k 10 120 python bench.py --size 1e4 --history 5 --line-search $LS --steps 3000 --warmup 100 --no-cpu-baseline --no-prof > gpurun_out/small_x_${LS}.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/small_x_${LS}.json')); print('n=1e4 $LS', d['value'], d['ms_per_step'], 'vf', d['vector_free']['value'])"
done; done
