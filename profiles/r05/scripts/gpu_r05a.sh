set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05a
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_coop_safety.py tests/test_gpu_rccl.py "tests/test_gpu_fullsize.py::test_fullsize_parity[config1_n1e7-True]" tests/test_gpu_speculative.py > gpurun_out/r05a/pytest.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05a/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --cpu-n2 0 > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err &&
BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=20 timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-vector-free > gpurun_out/r05a/w2.json 2> gpurun_out/r05a/w2.err &&
BENCH_DEVICE_MOD=1 LBFGS_CU_PARTITION=1 BENCH_RCCL_STALL=0 LBFGS_RCCL_TIMEOUT=15 timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-vector-free > gpurun_out/r05a/w2stall.json 2> gpurun_out/r05a/w2stall.err
