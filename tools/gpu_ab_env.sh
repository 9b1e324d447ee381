# A/B of the default-mode bench between runtime settings of the in-tree library.
# usage: tools/gpu_ab_env.sh "VAR=value ..." [sizes...]   (A = environment as given, B = with VARS)
set -o pipefail
mkdir -p gpurun_out
VARS="$1"; shift
SIZES=${@:-1e8 1e7}
env $VARS timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "trajectory_bit_exact or twoloop or sharded" > gpurun_out/pytest_ab.log 2>&1; rc=$?
echo "pytest B rc=$rc"; tail -1 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for ab in A B; do for n in $SIZES; do
  if [ $ab = B ]; then E="$VARS"; else E=""; fi
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size $n > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];ks=r['kernel_share'];print('$ab n=$n', d['value'], 'it/s', r['kernel'], r['achieved'], 'commit share', ks.get('commit'))"
done; done; done
