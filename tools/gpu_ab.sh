set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for nt in 1 0; do for n in 1e8 1e7; do
  LBFGS_NT=$nt timeout -k 10 300 python bench.py --no-cpu-baseline --size $n > gpurun_out/ab_nt${nt}_n${n}.json 2>gpurun_out/ab.err || exit 3
  python -c "import json;d=json.load(open('gpurun_out/ab_nt${nt}_n${n}.json'));print('NT=$nt n=$n', d['value'], 'it/s', d['ms_per_step'],'ms', d['achieved_hbm_gbps'],'GB/s', d['roofline']['kernel'], d['roofline']['achieved'])"
done; done
