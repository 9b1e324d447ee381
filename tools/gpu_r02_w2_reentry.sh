# the driver's N=2 bench line (its own --steps/--warmup) rehearsed with 2 ranks on one card, on
# the rebuilt library: the sharded headline, shard_check against one GPU, vector-free
set -o pipefail
mkdir -p gpurun_out
BENCH_DEVICE_MOD=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/w2_reentry.log 2>&1; rc=$?
echo "bench W=2 rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/w2_reentry.log; exit 1; }
grep '^{' gpurun_out/w2_reentry.log > gpurun_out/w2_reentry.json
python -c "import json; d=json.load(open('gpurun_out/w2_reentry.json')); print(d['value'], d['ms_per_step'], d['h_min'], d['config']['exchange'], d['shard_check'], d['exchange_latency_us'], (d['vector_free'] or {}).get('value'))"
