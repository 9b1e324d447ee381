# do long HBM-bound runs slow down on this box as the card heats (DESIGN.md §5, configs[4] on one
# card)? rocm-smi once a second over (1) n = 1e9 on one GPU for 400 timed steps (~60 s of
# streaming), kernel-traced, and (2) the one-card N = 8 rehearsal
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05p
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
bash tools/smi_monitor.sh gpurun_out/r05p/smi.txt 500 & mon=$!
trap 'kill $hb $mon 2> /dev/null' EXIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r05p/prof_long -o long -- python -u bench.py --size 1e9 --steps 400 --warmup 5 --no-vector-free --no-cpu-baseline --no-prof > gpurun_out/r05p/long.json 2> gpurun_out/r05p/long.err &&
BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 timeout -k 10 600 python -u bench.py --gpus 8 > gpurun_out/r05p/full.json 2> gpurun_out/r05p/full.err
