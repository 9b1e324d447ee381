# one rank of an 8-GPU n=1e8 run, approximated on one GPU: n = 1.25e7 with the shard's segment
# length 12288 (1017 workgroups per pass; variant build), reduce-kernel vs ticket stage 2
set -o pipefail
mkdir -p gpurun_out
export LBFGS_LIB=$PWD/cuda-lbfgs_amd/liblbfgs_hip_seg12k.so
for rep in 1 2; do for t in 0 1; do
  LBFGS_TICKET=$t timeout -k 10 300 python bench.py --no-cpu-baseline --no-vector-free --size 1.25e7 --steps 200 > gpurun_out/sg.json 2>gpurun_out/sg.err || { tail gpurun_out/sg.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/sg.json'));r=d['roofline'];print('seg12k ticket=$t', d['value'], 'it/s', d['ms_per_step'], r['kernel'], r['avg_launch_us'])"
done; done
