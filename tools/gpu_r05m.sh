# device memory around every context of the one-card N = 8 rehearsal (tools/meminfo_wrap.py): is
# configs[4]'s slow solve after the n = 1e8 lines a memory-state effect?
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05m
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
BENCH_RANK_WRAPPER="python -u $PWD/tools/meminfo_wrap.py --" BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 timeout -k 10 600 python -u bench.py --gpus 8 > gpurun_out/r05m/full.json 2> gpurun_out/r05m/full.err
