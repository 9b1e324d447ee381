set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head; exit 1; }
for n in 1e8 1e7 5e5 3e5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --size $n > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('n=$n', d['value'], 'it/s', r['kernel'], r['achieved'], 'vf', d['vector_free']['value'])"
done
