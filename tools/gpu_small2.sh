set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_vector_free.py -x -q -m gpu > gpurun_out/pytest_small2.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_small2.log; exit 1; }
tail -1 gpurun_out/pytest_small2.log
for mode in "" "--vector-free"; do for n in 1e4 3e4; do
  timeout -k 10 300 python bench.py --size $n --history 5 --steps 1000 --warmup 20 --no-cpu-baseline --no-vector-free $mode > gpurun_out/s2.json 2>gpurun_out/s2.err || { tail gpurun_out/s2.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/s2.json'));print('n=$n $mode', d['value'], 'it/s', d['ms_per_step'], 'ms', d['roofline']['kernel'] if d['roofline'] else None, d['roofline']['avg_launch_us'] if d['roofline'] else None)"
done; done
