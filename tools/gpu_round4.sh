set -o pipefail
mkdir -p gpurun_out
for t in 0 1; do
  LBFGS_TICKET=$t timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu_t$t.log 2>&1; rc=$?
  echo "pytest ticket=$t rc=$rc"; tail -3 gpurun_out/pytest_gpu_t$t.log
  [ $rc -le 1 ] || exit $rc
done
for t in 0 1; do for n in 1e8 1e7 1e6; do
  LBFGS_TICKET=$t timeout -k 10 300 python bench.py --no-cpu-baseline --size $n > gpurun_out/ab_t${t}_n${n}.json 2>gpurun_out/ab.err || exit 3
  python -c "import json;d=json.load(open('gpurun_out/ab_t${t}_n${n}.json'));r=d['roofline'];print('ticket=$t n=$n', d['value'], 'it/s', d['ms_per_step'],'ms', d['achieved_hbm_gbps'],'GB/s', r['kernel'], r['achieved'], r['avg_launch_us'])"
done; done
