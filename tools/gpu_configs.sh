set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/bench_configs.py gpurun_out/configs.json > gpurun_out/configs.log 2>&1; rc=$?
echo "rc=$rc"; cat gpurun_out/configs.log | tail -20
