set -o pipefail
for r in 1 2; do for v in 0 1; do
LBFGS_COLLECT=$v timeout -k 10 300 python bench.py --unfused --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/abu_$v.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/abu_$v.json'));print('unfused collect=$v', d['value'])"
done; done
