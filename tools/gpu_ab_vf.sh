# A/B of vector-free kernel variants: tools/gpu_ab_vf.sh name1 name2 ... (default = in-tree lib)
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  if [ $lib = default ]; then unset LBFGS_LIB; else export LBFGS_LIB=$PWD/cuda-lbfgs_amd/liblbfgs_hip_$lib.so; fi
  timeout -k 10 300 python bench.py --vector-free --no-cpu-baseline --size ${VF_N:-1e8} > gpurun_out/abvf_$lib.json 2>gpurun_out/abvf.err || { tail gpurun_out/abvf.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/abvf_$lib.json'));r=d['roofline'];print('$lib', d['value'], 'it/s', d['ms_per_step'],'ms', r['kernel'], r['achieved'], r['avg_launch_us'])"
done
