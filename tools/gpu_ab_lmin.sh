# canonical minimum segment length 512 (default) vs 1024 / 2048 (variant builds; timing only,
# the bits then differ from the oracle's canonical order)
set -o pipefail
mkdir -p gpurun_out/lmin
D=$PWD/cuda-lbfgs_amd
for S in ${SIZES:-1e4 1e5 3e5 6e5 1e6 2e6 4e6}; do
for rep in 1 2; do
for V in base lmin1024 lmin2048; do
  if [ $V = base ]; then E=""; else E="LBFGS_LIB=$D/liblbfgs_hip_$V.so"; fi
  env $E timeout -k 10 200 python bench.py --size $S --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline --no-config4 --no-prof > gpurun_out/lmin/b_${S}_${V}_${rep}.json 2> gpurun_out/lmin/err.log || { tail gpurun_out/lmin/err.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/lmin/b_${S}_${V}_${rep}.json'));print('$S $V $rep', d['value'], 'vf', d['vector_free']['value'])"
done; done; done
