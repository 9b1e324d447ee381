# configs[4]'s sharded rate on one card: one rank's geometry alone, on the
# full GPU and on its own 32 CUs, 8 independent 32-CU jobs at once (no exchange), and a kernel
# trace of every rank of the 8-process n = 1e9 rehearsal
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05b
LIB=$PWD/cuda-lbfgs_amd
B="python -u bench.py --size 1.25e8 --no-cpu-baseline --no-vector-free"
LBFGS_LIB=$LIB/liblbfgs_hip_seg122k.so LBFGS_TICKET=1 timeout -k 10 300 $B --steps 50 --warmup 3 > gpurun_out/r05b/rank_geo_fullgpu_ticket.json 2> gpurun_out/r05b/rank_geo_fullgpu_ticket.err &&
LBFGS_LIB=$LIB/liblbfgs_hip_seg122k.so LBFGS_TICKET=0 timeout -k 10 300 $B --steps 50 --warmup 3 > gpurun_out/r05b/rank_geo_fullgpu_collect.json 2> gpurun_out/r05b/rank_geo_fullgpu_collect.err &&
LBFGS_LIB=$LIB/liblbfgs_hip_seg122k_cuw8.so LBFGS_TICKET=1 timeout -k 10 300 $B --steps 50 --warmup 3 > gpurun_out/r05b/rank_geo_cu32_ticket.json 2> gpurun_out/r05b/rank_geo_cu32_ticket.err &&
LBFGS_LIB=$LIB/liblbfgs_hip_cuw8.so timeout -k 10 300 $B --steps 50 --warmup 3 > gpurun_out/r05b/n125e6_cu32_default.json 2> gpurun_out/r05b/n125e6_cu32_default.err &&
{ pids=""; for r in 0 1 2 3 4 5 6 7; do
    LBFGS_DEBUG_CU_RANK=$r LBFGS_LIB=$LIB/liblbfgs_hip_seg122k_cuw8.so LBFGS_TICKET=1 timeout -k 10 400 $B --steps 300 --warmup 3 --no-prof --no-box-probe > gpurun_out/r05b/indep8_r$r.json 2> gpurun_out/r05b/indep8_r$r.err & pids="$pids $!"
  done; ok=0; for p in $pids; do wait $p || ok=1; done; [ $ok = 0 ]; } &&
BENCH_RANK_WRAPPER="rocprofv3 --kernel-trace --stats -f csv -d $PWD/gpurun_out/r05b/prof_w8 -o %pid% --" BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 timeout -k 10 500 python -u bench.py --gpus 8 --size 1e9 --steps 5 --warmup 2 --no-vector-free --no-prof > gpurun_out/r05b/w8_n1e9_traced.json 2> gpurun_out/r05b/w8_n1e9_traced.err
