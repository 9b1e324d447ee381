# one box: (1) re-allocation probe (configs[4] on one card: is a large solve slower after another
# one's vectors were freed?); (2) the per-wave flagged partials of the collect stage 2 (variant
# liblbfgs_hip_wavep.so, -DLBK_WAVE_PARTIALS=1): parity tests on it, then bench lines alternating
# default / variant at n = 1e8. A line a minute for the watchdog.
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05h
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
V=$PWD/cuda-lbfgs_amd/liblbfgs_hip_wavep.so
B="python -u bench.py --no-cpu-baseline --no-vector-free --steps 40 --warmup 5"
timeout -k 10 300 python -u tools/realloc_probe.py gpurun_out/r05h/realloc.json > gpurun_out/r05h/realloc.txt 2>&1 &&
LBFGS_LIB=$V timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_fullsize.py::test_fullsize_parity" tests/test_gpu_collect.py tests/test_gpu_parity.py > gpurun_out/r05h/pytest_wavep.log 2>&1 &&
timeout -k 10 200 $B > gpurun_out/r05h/def_1.json 2> gpurun_out/r05h/def_1.err &&
LBFGS_LIB=$V timeout -k 10 200 $B > gpurun_out/r05h/wp_1.json 2> gpurun_out/r05h/wp_1.err &&
timeout -k 10 200 $B > gpurun_out/r05h/def_2.json 2> gpurun_out/r05h/def_2.err &&
LBFGS_LIB=$V timeout -k 10 200 $B > gpurun_out/r05h/wp_2.json 2> gpurun_out/r05h/wp_2.err &&
LBFGS_LIB=$V timeout -k 10 200 $B --size 3e7 > gpurun_out/r05h/wp_3e7.json 2> gpurun_out/r05h/wp_3e7.err &&
timeout -k 10 200 $B --size 3e7 > gpurun_out/r05h/def_3e7.json 2> gpurun_out/r05h/def_3e7.err
