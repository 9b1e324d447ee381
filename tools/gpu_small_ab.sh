# GPU suite, then small-n benches (default and vector-free) for the stage-2 small-group fast path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head; exit 1; }
for rep in 1 2; do for cfg in "1e4 5 3000" "3e4 10 2000" "1e5 10 1000"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu-baseline --size $1 --history $2 --steps $3 --warmup 20 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));v=d['vector_free'];print('n=$1', d['value'], 'it/s', 'vf', v['value'])"
done; done
