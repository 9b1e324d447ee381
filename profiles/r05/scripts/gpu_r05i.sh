# configs[4] on one card, the slow second solve: the 8-process n = 1e9 bench traced again with
# --exchange xgmi (no RCCL leg between the sharded solve and rank 0's one-GPU repeat); then the
# round's closing smoke and -m gpu suite (tools/gpu_r05_close1.sh). A line a minute for the watchdog.
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05i
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
BENCH_RANK_WRAPPER="rocprofv3 --kernel-trace --stats -f csv -d $PWD/gpurun_out/r05i/prof_xgmi -o %pid% --" BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 timeout -k 10 500 python -u bench.py --gpus 8 --size 1e9 --steps 5 --warmup 2 --no-vector-free --no-prof --exchange xgmi > gpurun_out/r05i/w8_xgmi.json 2> gpurun_out/r05i/w8_xgmi.err &&
python tools/config4_trace.py gpurun_out/r05i/prof_xgmi 5 > gpurun_out/r05i/trace_summary.txt 2>&1 &&
echo "traced run done" &&
bash tools/gpu.sh smoke && bash tools/gpu.sh suite
