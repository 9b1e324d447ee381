# the driver's N=8 bench line rehearsed with 8 ranks on one card (default steps/warmup, the
# vector-free sub-measurement, shard_check against one GPU, configs[4] at n = 1e9)
set -o pipefail
mkdir -p gpurun_out
BENCH_DEVICE_MOD=1 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 8 > gpurun_out/w8_close.log 2>&1; rc=$?
echo "bench W=8 rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/w8_close.log; exit 1; }
grep '^{' gpurun_out/w8_close.log > gpurun_out/w8_close.json
python -c "import json; d=json.load(open('gpurun_out/w8_close.json')); print(d['value'], d['ms_per_step'], d['config']['exchange'], d['shard_check'], d['exchange_latency_us'], (d['vector_free'] or {}).get('value'), json.dumps(d['config4_n1e9']))"
