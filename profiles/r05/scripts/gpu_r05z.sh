# the one-card N = 8 rehearsal with every rank held to one unmasked hardware queue
# (GPU_MAX_HW_QUEUES=1; the CU-masked solver queue comes on top): at most 2-3 compute queues per
# rank instead of 3-4, under the 24 the card's scheduler maps at once? configs[4] ran at 4.3 it/s
# with 25+ (tools/prectx_wrap.py: 2.45 it/s after three idle contexts per rank, 8.7 after none)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05z
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
bash tools/kfd_queues.sh gpurun_out/r05z/queues.txt 400 & mon=$!
trap 'kill $hb $mon 2> /dev/null' EXIT
GPU_MAX_HW_QUEUES=1 BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 timeout -k 10 600 python -u bench.py --gpus 8 > gpurun_out/r05z/full.json 2> gpurun_out/r05z/full.err
