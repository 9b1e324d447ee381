# A/B of the default-mode bench between the in-tree lib and variant libs (tools/build_variant.sh)
# usage: tools/gpu_ab_lib.sh variant [sizes...]
set -o pipefail
mkdir -p gpurun_out
V=$PWD/cuda-lbfgs_amd/liblbfgs_hip_$1.so; shift
SIZES=${@:-1e8 1e7}
LBFGS_LIB=$V timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "trajectory_bit_exact or twoloop or deterministic or sharded or trial" > gpurun_out/pytest_ab.log 2>&1; rc=$?
echo "pytest variant rc=$rc"; tail -1 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in default variant; do for n in $SIZES; do
  if [ $lib = variant ]; then export LBFGS_LIB=$V; else unset LBFGS_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size $n > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];ks=r['kernel_share'];print('$lib n=$n', d['value'], 'it/s', r['kernel'], r['achieved'], 'commit share', ks.get('commit'))"
done; done; done
