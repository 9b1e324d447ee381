# cooperative iteration: bit-exactness tests, then A/B of the segment limit across small/mid n
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider -k "cooperative or small_persistent" --timeout 120 --timeout-method thread > gpurun_out/pytest_coop.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -cE "PASSED" gpurun_out/pytest_coop.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|k_coop" gpurun_out/pytest_coop.log | head -20; exit 1; }
for rep in 1 2; do for cfg in "1e4 5 3000" "3e4 10 2000" "1e5 10 1000" "2e5 10 600" "2.6e5 10 600"; do for ab in 0 512; do
  set -- $cfg
  LBFGS_COOP=$ab timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size $1 --history $2 --steps $3 --warmup 20 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('COOP=$ab n=$1', d['value'], 'it/s')"
done; done; done
