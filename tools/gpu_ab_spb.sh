set -o pipefail
mkdir -p gpurun_out
for spb in 4 3; do
LBFGS_SPB=$spb timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_vector_free.py -x -q -k "trajectory_bit_exact or sharded or deterministic or bit_exact_vs_oracle or at_scale" > gpurun_out/pytest_spb.log 2>&1 || { echo "pytest spb=$spb rc=$?"; tail -30 gpurun_out/pytest_spb.log; exit 1; }
echo "spb=$spb $(tail -1 gpurun_out/pytest_spb.log)"
done
for n in 1e7 1e6 1e8; do for spb in 1 2 4; do
  LBFGS_SPB=$spb timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size $n --steps 200 > gpurun_out/spb.json 2>gpurun_out/spb.err || { tail gpurun_out/spb.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/spb.json'));r=d['roofline'];print('n=$n spb=$spb', d['value'], 'it/s', r['kernel'], r['avg_launch_us'])"
done; done
