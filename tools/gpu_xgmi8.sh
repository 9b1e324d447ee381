# 8 ranks on the one-GPU box (BENCH_DEVICE_MOD=1, xGMI peer exchange without RCCL): the exact
# geometry of the driver's 8-GPU n = 1e8 run (ticket stage 2, 1017 workgroups per pass).
set -o pipefail
mkdir -p gpurun_out
BENCH_DEVICE_MOD=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --size ${SIZE:-1e8} --steps 10 --warmup 12 --no-cpu-baseline > gpurun_out/xgmi_bench8.log 2>&1; rc=$?
echo "bench W=8 rc=$rc"; grep '^{' gpurun_out/xgmi_bench8.log || tail -30 gpurun_out/xgmi_bench8.log
