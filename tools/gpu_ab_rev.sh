# LBFGS_REV=1 (alternating segment walk direction): parity subset with it on, then A/B benches
set -o pipefail
mkdir -p gpurun_out
LBFGS_REV=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vector_free.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_rev.log 2>&1; rc=$?
echo "pytest REV=1 rc=$rc"; tail -1 gpurun_out/pytest_rev.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do for ab in 0 1; do for n in 1e8 1e7; do
  LBFGS_REV=$ab timeout -k 10 300 python bench.py --no-cpu-baseline --size $n > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];v=d['vector_free'];print('REV=$ab n=$n', d['value'], 'it/s', r['kernel'], r['achieved'], 'vf', v['value'])"
done; done; done
