# small_wait asks the stream only after 0.25 s: the runtime thread that spun beside each waiting
# rank (tools/query_probe.hip) should stay idle; then the one-card N = 8 rehearsal with the CPU
# monitor (configs[4] at 4.2-5.0 it/s before, the job's 16-CPU quota throttled)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05t
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb $mon 2> /dev/null' EXIT
timeout -k 10 300 python -u tools/thread_probe.py gpurun_out/r05t/threads.json > gpurun_out/r05t/threads.log 2>&1 &&
{ bash tools/cpu_monitor.sh gpurun_out/r05t/cpu.txt 300 & mon=$!; } &&
BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 timeout -k 10 600 python -u bench.py --gpus 8 > gpurun_out/r05t/full.json 2> gpurun_out/r05t/full.err
