set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "trajectory_bit_exact or sharded or deterministic" > gpurun_out/pytest_pp.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_pp.log; exit 1; }
tail -1 gpurun_out/pytest_pp.log
for rep in 1 2; do for pp in 0 1; do for n in 1e8 1e7; do
  LBFGS_PINGPONG=$pp timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size $n > gpurun_out/pp.json 2>gpurun_out/pp.err || { tail gpurun_out/pp.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/pp.json'));r=d['roofline'];print('pp=$pp n=$n', d['value'], 'it/s', r['kernel'], r['achieved'], r['avg_launch_us'], r['kernel_share'])"
done; done; done
