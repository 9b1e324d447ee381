# one box: (1) the two-loop passes issuing their first rows' loads before the previous pass's total
# (variant liblbfgs_hip_pfcoef.so, -DLBK_PREFETCH_COEF=1): configs[2] full-size parity on it, then
# bench lines alternating default / variant; (2) configs[4]'s sharded rate on one card
# (tools/gpu_r05b.sh). A line a minute for the watchdog.
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05g
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
V=$PWD/cuda-lbfgs_amd/liblbfgs_hip_pfcoef.so
B="python -u bench.py --no-cpu-baseline --no-vector-free --steps 40 --warmup 5"
LBFGS_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_fullsize.py::test_fullsize_parity" tests/test_gpu_parity.py > gpurun_out/r05g/pytest_pfcoef.log 2>&1 &&
timeout -k 10 200 $B > gpurun_out/r05g/def_1.json 2> gpurun_out/r05g/def_1.err &&
LBFGS_LIB=$V timeout -k 10 200 $B > gpurun_out/r05g/pf_1.json 2> gpurun_out/r05g/pf_1.err &&
timeout -k 10 200 $B > gpurun_out/r05g/def_2.json 2> gpurun_out/r05g/def_2.err &&
LBFGS_LIB=$V timeout -k 10 200 $B > gpurun_out/r05g/pf_2.json 2> gpurun_out/r05g/pf_2.err &&
echo "A/B done" &&
bash tools/gpu_r05b.sh
