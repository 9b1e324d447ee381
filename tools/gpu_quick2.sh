set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_xgmi.log 2>&1; rc=$?
echo "pytest xgmi rc=$rc"; tail -1 gpurun_out/pytest_xgmi.log
[ $rc -eq 0 ] || exit 1
BENCH_DEVICE_MOD=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 2 --size 2e7 --steps 10 --warmup 12 --no-cpu-baseline > gpurun_out/w2.log 2>&1; rc=$?
echo "W=2 rc=$rc"; grep '^{' gpurun_out/w2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['exchange'], d['exchange_latency_us'], d['vector_free']['value'])" || tail -20 gpurun_out/w2.log
HIP_VISIBLE_DEVICES=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 2 --size 2e7 --steps 10 --warmup 12 --no-cpu-baseline --no-vector-free > gpurun_out/w2v.log 2>&1; rc=$?
echo "W=2 visible=1 rc=$rc (RCCL refuses two ranks on one device; expected to fall back or fail cleanly)"; tail -3 gpurun_out/w2v.log
