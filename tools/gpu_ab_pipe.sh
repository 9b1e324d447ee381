set -o pipefail
mkdir -p gpurun_out
P=$PWD/cuda-lbfgs_amd/liblbfgs_hip_pipe1.so
LBFGS_LIB=$P timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -x -k "trajectory_bit_exact or twoloop or deterministic" > gpurun_out/pytest_pipe.log 2>&1; rc=$?
echo "pytest pipe rc=$rc"; tail -3 gpurun_out/pytest_pipe.log
[ $rc -le 1 ] || exit $rc
for rep in 1 2; do for lib in default pipe; do for n in 1e8 1e7; do
  if [ $lib = pipe ]; then export LBFGS_LIB=$P; else unset LBFGS_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --size $n > gpurun_out/ab_${lib}_${n}.json 2>gpurun_out/ab.err || exit 3
  python -c "import json;d=json.load(open('gpurun_out/ab_${lib}_${n}.json'));r=d['roofline'];print('$lib n=$n', d['value'], 'it/s', d['ms_per_step'],'ms', r['kernel'], r['achieved'], r['avg_launch_us'])"
done; done; done
