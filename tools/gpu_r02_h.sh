# round 2: host-callback call policies at n=1e7; every BASELINE config on one GPU (current build)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/host_cb_bench.py gpurun_out/host_cb_bench.json > gpurun_out/host_cb_bench.log 2>&1; rc=$?
tail -3 gpurun_out/host_cb_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/bench_configs.py gpurun_out/configs.json > gpurun_out/configs.log 2>&1; rc=$?
tail -5 gpurun_out/configs.log
exit $rc
