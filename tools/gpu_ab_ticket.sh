set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for t in 0 1; do for n in 1e8 1.25e7; do
  LBFGS_TICKET=$t timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size $n > gpurun_out/tk.json 2>gpurun_out/tk.err || { tail gpurun_out/tk.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/tk.json'));r=d['roofline'];print('ticket=$t n=$n', d['value'], 'it/s', d['ms_per_step'], r['kernel'], r['avg_launch_us'])"
done; done; done
