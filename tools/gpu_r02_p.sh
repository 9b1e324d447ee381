# speculative next iteration at small n: its tests, the cooperative / stress parity tests, and
# n = 1e4 (configs[0]) with LBFGS_SPEC=0 / 1, plus a kernel trace of the speculative run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_speculative.py tests/test_gpu_stress.py "tests/test_gpu_parity.py::test_cooperative_iteration_bit_exact" > gpurun_out/pytest_spec.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_spec.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_spec.log | head -30; exit 1; }
for s in 0 1 0 1; do
  LBFGS_SPEC=$s timeout -k 10 120 python bench.py --size 1e4 --history 5 --steps 3000 --warmup 100 --no-cpu-baseline --no-vector-free --no-prof > gpurun_out/small_spec$s.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/small_spec$s.json')); print('n=1e4 spec=$s', d['value'], d['ms_per_step'])"
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small_spec -o run --output-format csv -- python3 bench.py --size 1e4 --history 5 --steps 3000 --warmup 100 --no-cpu-baseline --no-vector-free --no-prof > gpurun_out/prof_small_spec.log 2>&1; rc=$?; echo "prof rc=$rc"
