# Non-temporal policy at per-rank sizes of the 8-GPU headline (n_loc = 1.25e7) and above on one
# GPU: does the 256 MiB Infinity Cache hold the work vectors (q/r/d) when the history streams
# NT? base0/1 = all temporal / all NT; wt1 = NT history, temporal q/r/d; wt2 = + x, g; wt3 = + new s, y.
set -o pipefail
mkdir -p gpurun_out/nt
D=$PWD/cuda-lbfgs_amd
rc=0; [ -n "$SKIP_PYTEST" ] || LBFGS_LIB=$D/liblbfgs_hip_wt3.so LBFGS_NT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/nt/pytest_wt.log 2>&1; rc=$?
echo "pytest wt rc=$rc"; tail -1 gpurun_out/nt/pytest_wt.log
[ $rc -eq 0 ] || exit 1
for S in ${SIZES:-1.25e7 2.5e7 1e8}; do
for rep in 1 2; do
for V in ${VARS:-base1 wt1 wt2 wt3}; do
  case $V in base0) E="LBFGS_NT=0";; base1) E="LBFGS_NT=1";; *) E="LBFGS_NT=1 LBFGS_LIB=$D/liblbfgs_hip_$V.so";; esac
  env $E timeout -k 10 200 python bench.py --size $S --steps 60 --warmup 10 --no-cpu-baseline --no-config4 > gpurun_out/nt/b_${S}_${V}_${rep}.log 2>&1; rc=$?
  echo -n "size=$S $V rep=$rep rc=$rc "; grep '^{' gpurun_out/nt/b_${S}_${V}_${rep}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['achieved'], d['vector_free'] and d['vector_free'].get('value'))" || tail -20 gpurun_out/nt/b_${S}_${V}_${rep}.log
  [ $rc -eq 0 ] || exit 1
done; done; done
