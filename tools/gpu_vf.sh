set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_vector_free.py -x -q > gpurun_out/pytest_vf.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_vf.log; exit 1; }
tail -3 gpurun_out/pytest_vf.log
timeout -k 10 300 python bench.py --vector-free --no-cpu-baseline > gpurun_out/bench_vf.json 2> gpurun_out/bench_vf.err || { echo "bench rc=$?"; tail gpurun_out/bench_vf.err; exit 1; }
cat gpurun_out/bench_vf.json
timeout -k 10 300 python bench.py --vector-free --no-cpu-baseline --size 1e7 --steps 200 > gpurun_out/bench_vf_1e7.json 2>&1 && cat gpurun_out/bench_vf_1e7.json
