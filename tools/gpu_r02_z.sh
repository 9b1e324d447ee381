# does the concurrent CPU baseline (two pinned host processes) move the GPU number?
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-vector-free > gpurun_out/z_with.json 2>/dev/null || exit 1
  timeout -k 10 300 python bench.py --no-vector-free --no-cpu-baseline > gpurun_out/z_without.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('gpurun_out/z_with.json')); b=json.load(open('gpurun_out/z_without.json')); print('with cpu baseline', a['value'], ' without', b['value'])"
done
