set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_unfused.py tests/test_matrices_kat.py tests/test_cxx_dropin.py -x -q -m gpu > gpurun_out/pytest_small.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_small.log; exit 1; }
tail -1 gpurun_out/pytest_small.log
for n in 1e4 3e4; do for segs in 0 256; do
  LBFGS_SMALL_SEGS=$segs timeout -k 10 300 python bench.py --size $n --history 5 --steps 1000 --warmup 20 --no-cpu-baseline --no-vector-free > gpurun_out/sm.json 2>gpurun_out/sm.err || { tail gpurun_out/sm.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/sm.json'));print('n=$n segs=$segs', d['value'], 'it/s', d['ms_per_step'], 'ms', d['roofline']['kernel'] if d['roofline'] else None, d['roofline']['avg_launch_us'] if d['roofline'] else None)"
done; done
