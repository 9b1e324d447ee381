# KFD user queues per process during the one-card N = 8 rehearsal (tools/kfd_queues.sh): does
# configs[4]'s solve, after the n = 1e8 lines, run with more queues on the card than the hardware
# scheduler maps at once?
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05n
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
bash tools/kfd_queues.sh gpurun_out/r05n/queues.txt 400 & mon=$!
trap 'kill $hb $mon 2> /dev/null' EXIT
BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 timeout -k 10 600 python -u bench.py --gpus 8 > gpurun_out/r05n/full.json 2> gpurun_out/r05n/full.err
