# the stream-pooled library (solver streams reused across contexts) in the one-card N = 8 rehearsal,
# with the KFD queue monitor grouped by GPU: configs[4] against r05k / r05l / r05n (4.2-5.0 it/s)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05o
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
bash tools/kfd_queues.sh gpurun_out/r05o/queues.txt 400 & mon=$!
trap 'kill $hb $mon 2> /dev/null' EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_context_reuse.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05o/reuse_tests.log 2>&1 &&
BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 timeout -k 10 600 python -u bench.py --gpus 8 > gpurun_out/r05o/full.json 2> gpurun_out/r05o/full.err
