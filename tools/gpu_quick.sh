# quick check: GPU suite + default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print(d['value'], r['kernel'], r['achieved'], r['frac'], r['avg_launch_us'], r['kernel_share'], d['vector_free']['value'])"
for S in ${SIZES:-}; do
  timeout -k 10 200 python bench.py --size $S --steps 60 --warmup 10 --no-cpu-baseline --no-config4 > gpurun_out/bench_$S.json 2> gpurun_out/bench_$S.err || { tail gpurun_out/bench_$S.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$S.json'));r=d['roofline'];print('$S', d['value'], r['kernel'], r['achieved'], d['vector_free']['value'])"
done
