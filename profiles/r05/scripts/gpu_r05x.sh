# slot fetches without a completion word poll one written by k_slot_publish instead of waiting on
# the stream: the runtime thread should stay idle (tools/thread_probe.py), the -m gpu suite green,
# and the one-card N = 8 rehearsal unthrottled (tools/cpu_monitor.sh)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05x
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb $mon 2> /dev/null' EXIT
timeout -k 10 120 python -u tools/thread_probe.py --solves 4 gpurun_out/r05x/threads.json > gpurun_out/r05x/threads.log 2>&1 &&
bash tools/gpu.sh smoke && bash tools/gpu.sh suite &&
{ bash tools/cpu_monitor.sh gpurun_out/r05x/cpu.txt 300 & mon=$!; } &&
BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 timeout -k 10 600 python -u bench.py --gpus 8 > gpurun_out/r05x/full.json 2> gpurun_out/r05x/full.err
