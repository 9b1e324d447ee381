# xGMI peer exchange on the one-GPU box: multi-process tests, then 2- and 4-rank bench
# rehearsals on one card (BENCH_DEVICE_MOD=1; no RCCL communicator).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_xgmi.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_xgmi.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_xgmi.log
[ $rc -eq 0 ] || exit 1
for W in 2 4; do
  BENCH_DEVICE_MOD=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 2951$W bench.py --gpus $W --size ${SIZE:-2e7} --steps 20 --warmup 12 --no-cpu-baseline > gpurun_out/xgmi_bench$W.log 2>&1; rc=$?
  echo "bench W=$W rc=$rc"; grep '^{' gpurun_out/xgmi_bench$W.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['exchange'], d['vector_free'] and d['vector_free'].get('value'))" || tail -20 gpurun_out/xgmi_bench$W.log
  [ $rc -eq 0 ] || exit 1
done
