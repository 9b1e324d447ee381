set -o pipefail
mkdir -p gpurun_out
export BENCH_DEVICE_MOD=1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --size 2e7 --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/rccl2.log 2>&1; rc=$?
echo "rc=$rc"; tail -30 gpurun_out/rccl2.log
