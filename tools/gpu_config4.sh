# 8 ranks on the one-GPU box: the driver's N=8 bench line including the n=1e9 (configs[4])
# sub-measurement (8 x 30 GB of vectors on one 288 GB card)
set -o pipefail
mkdir -p gpurun_out
BENCH_DEVICE_MOD=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --steps 5 --warmup 12 --no-vector-free > gpurun_out/config4_w8.log 2>&1; rc=$?
echo "bench W=8 rc=$rc"; grep '^{' gpurun_out/config4_w8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['config4_n1e9']), d['exchange_latency_us'])" || tail -30 gpurun_out/config4_w8.log
