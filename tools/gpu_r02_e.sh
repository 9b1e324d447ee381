# round 2: configs[3] batched vs one pass per step; configs[2] bench A/B of LBFGS_BATCH
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/config3.py gpurun_out/config3.json > gpurun_out/config3.log 2>&1; rc=$?
tail -4 gpurun_out/config3.log
[ $rc -eq 0 ] || exit $rc
for b in 1 0 1 0; do
  LBFGS_BATCH=$b timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free > gpurun_out/bench_batch$b.json 2> gpurun_out/bench_batch$b.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_batch$b.json'));print('batch=$b', d['value'], d['solver'], d['roofline']['frac'])"
done
