# host wait policy at small n: ROC_ACTIVE_WAIT_TIMEOUT (HIP runtime's active-wait window before an
# interrupt wait) default vs raised
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for ab in default 200 2000; do for cfg in "1e4 5 3000" "1e5 10 1000"; do
  set -- $cfg
  if [ $ab = default ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$ab; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --size $1 --history $2 --steps $3 --warmup 20 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));v=d['vector_free'];print('WAIT=$ab n=$1', d['value'], 'it/s', 'vf', v['value'])"
done; done; done
