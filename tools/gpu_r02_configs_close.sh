# every BASELINE config and the paper's Table I comparison on the closing build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_configs.py gpurun_out/configs.json > gpurun_out/configs.log 2>&1 || { tail -5 gpurun_out/configs.log; exit 1; }
timeout -k 10 300 python tools/paper_table.py gpurun_out/paper_table.json > gpurun_out/paper_table.log 2>&1 || { tail -5 gpurun_out/paper_table.log; exit 1; }
tail -3 gpurun_out/configs.log; tail -6 gpurun_out/paper_table.log
