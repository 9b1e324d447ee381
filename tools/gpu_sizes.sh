# default and vector-free mode over n on one GPU (bench.py lines, no CPU baseline)
set -o pipefail
mkdir -p gpurun_out/sizes
for S in ${SIZES:-1e5 1e6 3e6 1e7 2e7 1e8}; do
  timeout -k 10 200 python bench.py --size $S --steps ${STEPS:-60} --warmup 12 --no-cpu-baseline --no-config4 > gpurun_out/sizes/b_$S.json 2> gpurun_out/sizes/b_$S.err || { tail gpurun_out/sizes/b_$S.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sizes/b_$S.json'));r=d['roofline'] or {};v=d['vector_free'];vr=v.get('roofline') or {};print('$S', d['value'], r.get('kernel'), r.get('achieved'), 'vf', v['value'], vr.get('kernel'), vr.get('achieved'))"
done
