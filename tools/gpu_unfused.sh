set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 900 python tools/bench_configs.py gpurun_out/configs.json > gpurun_out/configs.log 2>&1 || { echo "configs rc=$?"; tail -20 gpurun_out/configs.log; exit 1; }
cat gpurun_out/configs.log
