# configs[4] in the one-card N = 8 rehearsal ran at 4.95 it/s (r05k) against 8.5 it/s for the same
# n = 1e9 sharded solve run as the headline for 5 steps (r05b): kernel traces of every rank for
# (A) the full rehearsal and (B) n = 1e9 as the headline for 100 steps with nothing run before it
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05l
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
W="rocprofv3 --kernel-trace --stats -f csv -o %pid% -d"
BENCH_RANK_WRAPPER="$W $PWD/gpurun_out/r05l/prof_full --" BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 timeout -k 10 600 python -u bench.py --gpus 8 --no-prof > gpurun_out/r05l/full.json 2> gpurun_out/r05l/full.err &&
BENCH_RANK_WRAPPER="$W $PWD/gpurun_out/r05l/prof_1e9 --" BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 timeout -k 10 600 python -u bench.py --gpus 8 --size 1e9 --steps 100 --warmup 20 --no-vector-free --no-prof --exchange xgmi > gpurun_out/r05l/n1e9_100.json 2> gpurun_out/r05l/n1e9_100.err &&
python tools/config4_trace.py gpurun_out/r05l/prof_full 10 > gpurun_out/r05l/full_trace.txt &&
python tools/config4_trace.py gpurun_out/r05l/prof_1e9 10 > gpurun_out/r05l/n1e9_trace.txt
