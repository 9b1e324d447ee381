# deferred stage 2 with the all-groups prologue: bit-exactness, then A/B across groups counts
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider -k "deferred or cooperative or trajectory" --timeout 200 --timeout-method thread > gpurun_out/pytest_defer.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_defer.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_defer.log | head -20; exit 1; }
for rep in 1 2; do for n in 5e5 1e6 2e6 4e6; do for ab in 0 8192; do
  LBFGS_DEFER=$ab timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size $n --steps 300 --warmup 20 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('DEFER=$ab n=$n', d['value'], 'it/s')"
done; done; done
