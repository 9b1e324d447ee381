# does the slow configs[4] regime follow from queues the earlier contexts created (no computation
# on them)? n = 1e9 as the headline over 8 one-card ranks, after (a) 2 sharded + 1 one-GPU
# contexts created and closed in every rank, (b) none (tools/prectx_wrap.py)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05y
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
B="python -u bench.py --gpus 8 --size 1e9 --steps 50 --warmup 10 --no-vector-free --no-prof --no-box-probe --exchange xgmi"
PRECTX_SHARDED=2 PRECTX_ONE=1 BENCH_RANK_WRAPPER="python -u $PWD/tools/prectx_wrap.py --" BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 timeout -k 10 400 $B > gpurun_out/r05y/pre2_1.json 2> gpurun_out/r05y/pre2_1.err &&
PRECTX_SHARDED=0 PRECTX_ONE=0 BENCH_RANK_WRAPPER="python -u $PWD/tools/prectx_wrap.py --" BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 timeout -k 10 400 $B > gpurun_out/r05y/pre0_0.json 2> gpurun_out/r05y/pre0_0.err &&
PRECTX_SHARDED=1 PRECTX_ONE=0 BENCH_RANK_WRAPPER="python -u $PWD/tools/prectx_wrap.py --" BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 timeout -k 10 400 $B > gpurun_out/r05y/pre1_0.json 2> gpurun_out/r05y/pre1_0.err
