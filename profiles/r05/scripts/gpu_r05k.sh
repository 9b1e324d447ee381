# the driver's N = 8 command rehearsed on one card (8 self-launched ranks, each on its own 32 CUs):
# the n = 1e8 line, the vector-free line, configs[4] at n = 1e9, then the RCCL comparison leg last
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05k
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 timeout -k 10 1000 python -u bench.py --gpus 8 > gpurun_out/r05k/selflaunch_w8.json 2> gpurun_out/r05k/selflaunch_w8.err
