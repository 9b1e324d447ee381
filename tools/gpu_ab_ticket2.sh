# stage-2 form A/B across mid n: reduce kernel (LBFGS_TICKET=0) vs in-launch tickets (=1)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for n in 1e5 3e5 1e6 3e6; do for ab in 0 1; do
  LBFGS_TICKET=$ab timeout -k 10 300 python bench.py --no-cpu-baseline --size $n --steps 500 --warmup 20 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));v=d['vector_free'];print('TICKET=$ab n=$n', d['value'], 'it/s', 'vf', v['value'])"
done; done; done
