# the RCCL leg with a peer that never joins its init (BENCH_RCCL_STALL): the line must still print
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05a2
BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 BENCH_RCCL_STALL=0 LBFGS_RCCL_TIMEOUT=15 timeout -k 10 240 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-vector-free > gpurun_out/r05a2/w2stall.json 2> gpurun_out/r05a2/w2stall.err
