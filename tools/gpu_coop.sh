# cooperative small-n iteration: bit-exactness tests, then A/B at small n
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider -k "cooperative or small_persistent" --timeout 120 --timeout-method thread > gpurun_out/pytest_coop.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/pytest_coop.log | tail -12
[ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_coop.log; exit 1; }
for rep in 1 2; do for ab in 0 1; do for cfg in "1e4 5 3000" "3e4 10 2000"; do
  set -- $cfg
  LBFGS_COOP=$ab timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size $1 --history $2 --steps $3 --warmup 20 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('COOP=$ab n=$1', d['value'], 'it/s', d['roofline']['kernel_share'] if d['roofline'] else '')"
done; done; done
