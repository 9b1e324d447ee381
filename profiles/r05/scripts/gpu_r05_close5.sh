# round 5 close, part 5: the driver's N = 8 command self-launched on this one card again, now that
# bench.py sets GPU_MAX_HW_QUEUES=1 for rehearsal ranks over the box's default of 4 (part 4 kept
# the default and configs[4] ran at 3.69 it/s); then the host-thread regression test. A line a
# minute for the watchdog.
set -o pipefail
cd /root/repo
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 bash tools/gpu.sh selflaunch 8 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_threads.py tests/test_gpu_context_reuse.py -m gpu -v \
    --timeout 120 --timeout-method thread > gpurun_out/host_threads_tests.log 2>&1
