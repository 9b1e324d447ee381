set -o pipefail
mkdir -p gpurun_out
for n in 1e7 3e7 1e6; do for nt in 0 1; do
  LBFGS_NT=$nt timeout -k 10 300 python bench.py --vector-free --no-cpu-baseline --size $n --steps 200 > gpurun_out/nt_$nt_$n.json 2>gpurun_out/nt.err || { tail gpurun_out/nt.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/nt_$nt_$n.json'));r=d['roofline'];print('n=$n NT=$nt', d['value'], 'it/s', r['kernel'], r['achieved'], r['avg_launch_us'])"
done; done
