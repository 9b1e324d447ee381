# round 2: the RCCL leg on one GPU and configs[4]'s shard geometry (tests/test_gpu_rccl.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl.py -v --timeout 600 --timeout-method thread > gpurun_out/pytest_rccl.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_rccl.log
exit $rc
