set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for lib in default prespb; do for n in 1e6 1e7; do
  if [ $lib = prespb ]; then export LBFGS_LIB=$PWD/cuda-lbfgs_amd/liblbfgs_hip_prespb.so; else unset LBFGS_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size $n --steps 500 > gpurun_out/pp.json 2>gpurun_out/pp.err || { tail gpurun_out/pp.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/pp.json'));r=d['roofline'];print('$lib n=$n', d['value'], 'it/s', r['kernel'], r['avg_launch_us'])"
done; done; done
