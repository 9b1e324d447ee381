# CPU time of every rank thread and the job's cgroup throttling during the one-card N = 8
# rehearsal (tools/cpu_monitor.sh): configs[4] after the n = 1e8 lines runs with the ranks out of
# step and the card at ~720 W against ~1060 W when they stream together (r05p)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05q
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
bash tools/cpu_monitor.sh gpurun_out/r05q/cpu.txt 300 & mon=$!
trap 'kill $hb $mon 2> /dev/null' EXIT
BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 timeout -k 10 600 python -u bench.py --gpus 8 > gpurun_out/r05q/full.json 2> gpurun_out/r05q/full.err
