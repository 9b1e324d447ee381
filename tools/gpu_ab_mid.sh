# A/B: k_mid with 8-row load groups (LBK_MID_UNROLL=8, liblbfgs_hip_mid8.so) against the default 4:
# parity suite on the variant, rocprofv3 kernel stats of both, then the bench line alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/cuda-lbfgs_amd/liblbfgs_hip_mid8.so
LBFGS_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_mid_parity.log 2>&1; rc=$?; tail -2 gpurun_out/ab_mid_parity.log; [ $rc -eq 0 ] || exit 1
for lib in base mid8; do
  if [ $lib = mid8 ]; then export LBFGS_LIB=$V; else unset LBFGS_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_mid_$lib -o run --output-format csv -- python3 bench.py --steps 30 --warmup 12 --no-cpu-baseline --no-prof > gpurun_out/ab_mid_$lib.log 2>&1 || exit 2
  grep -h 'k_mid\|k_axpy_dot' gpurun_out/ab_mid_$lib/*/run_kernel_stats.csv gpurun_out/ab_mid_$lib/run_kernel_stats.csv 2>/dev/null | cut -d, -f1-4 | sed "s/^/$lib /"
done
for rep in 1 2; do for lib in base mid8; do
  if [ $lib = mid8 ]; then export LBFGS_LIB=$V; else unset LBFGS_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_mid_bench_${lib}_$rep.json 2>/dev/null || exit 3
  python -c "import json;d=json.load(open('gpurun_out/ab_mid_bench_${lib}_$rep.json'));ks=d['roofline']['kernel_share'];print('$lib', d['value'], d['ms_per_step'], 'mid share', ks.get('mid'), d['roofline']['avg_launch_us'])"
done; done
