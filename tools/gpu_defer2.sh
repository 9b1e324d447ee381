# full GPU suite with the deferred stage 2 on by default (<= 1024 segments), then A/B near the limit
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head; exit 1; }
for rep in 1 2; do for n in 2e5 3e5 4e5 5e5; do for ab in 0 1024; do
  LBFGS_DEFER=$ab timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size $n --steps 500 --warmup 20 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('DEFER=$ab n=$n', d['value'], 'it/s')"
done; done; done
