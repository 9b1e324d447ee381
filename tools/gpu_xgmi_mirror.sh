# Host mirror filled by the xGMI exchange (LBFGS_XGMI_MIRROR): multi-process parity tests, then
# A/B bench rehearsals on the one-GPU box (BENCH_DEVICE_MOD=1), alternating the setting.
set -o pipefail
mkdir -p gpurun_out/mirror
timeout -k 10 600 python -u -m pytest tests/test_gpu_xgmi.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/mirror/pytest_xgmi.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/mirror/pytest_xgmi.log
[ $rc -eq 0 ] || exit 1
for S in 4e6 2e7; do
for rep in 1 2; do
for M in 0 1; do
  LBFGS_XGMI_MIRROR=$M BENCH_DEVICE_MOD=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 2952$M bench.py --gpus 4 --size $S --steps 30 --warmup 12 --no-cpu-baseline --no-config4 > gpurun_out/mirror/b_${S}_${M}_${rep}.log 2>&1; rc=$?
  echo -n "size=$S mirror=$M rep=$rep rc=$rc "; grep '^{' gpurun_out/mirror/b_${S}_${M}_${rep}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['exchange'], d['vector_free'] and d['vector_free'].get('value'))" || tail -20 gpurun_out/mirror/b_${S}_${M}_${rep}.log
  [ $rc -eq 0 ] || exit 1
done; done; done
