# exchange latency of the xGMI mailbox path on the one-GPU box (2 and 8 ranks on one card,
# no RCCL), from bench.py's sharded JSON line (exchange_latency_us)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_xgmi.log 2>&1 || { tail -30 gpurun_out/pytest_xgmi.log; exit 1; }
tail -1 gpurun_out/pytest_xgmi.log
for W in 2 8; do
  BENCH_DEVICE_MOD=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 2952$W bench.py --gpus $W --size 2e7 --steps 10 --warmup 12 --no-cpu-baseline --no-vector-free > gpurun_out/xgmi_lat$W.log 2>&1; rc=$?
  echo "W=$W rc=$rc"; grep '^{' gpurun_out/xgmi_lat$W.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['exchange_latency_us'])" || { tail -20 gpurun_out/xgmi_lat$W.log; exit 1; }
done
