# round 2: rehearse the driver's N=2 and N=8 bench lines on the one-GPU box (ranks share the card;
# xGMI mailboxes over same-device IPC, RCCL cannot run two ranks on one device)
set -o pipefail
mkdir -p gpurun_out
BENCH_DEVICE_MOD=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/rehearsal_w2.log 2>&1; rc=$?
echo "bench W=2 rc=$rc"; grep '^{' gpurun_out/rehearsal_w2.log > gpurun_out/rehearsal_w2.json || { tail -30 gpurun_out/rehearsal_w2.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/rehearsal_w2.json')); print(d['value'], d['h_min'], d['config']['exchange'], d['exchange_latency_us'], d['vector_free']['value'] if d['vector_free'] else None)"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_config4.sh
