set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for n in 1e4 1e5 1e6; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --size $n > gpurun_out/b_n${n}.json 2>gpurun_out/b.err || exit 3
  python -c "import json;d=json.load(open('gpurun_out/b_n${n}.json'));r=d['roofline'];print('n=$n', d['value'], 'it/s', d['ms_per_step'],'ms', d['achieved_hbm_gbps'],'GB/s', r['kernel'], r['avg_launch_us'])"
done
