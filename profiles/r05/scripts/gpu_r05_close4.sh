# round 5 close, part 4 (after the slot-publish fetch and the rehearsal queue setting): the driver's
# N = 8 and N = 2 commands self-launched on this one card (CU-partitioned; bench.py holds the
# rehearsal ranks to one unmasked hardware queue), every BASELINE config on one GPU, and the mix
# probe with the passes' reduction tail (tools/mixprobe.hip). A line a minute for the watchdog.
set -o pipefail
cd /root/repo
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 bash tools/gpu.sh selflaunch 8 &&
LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 bash tools/gpu.sh selflaunch 2 &&
bash tools/gpu.sh configs &&
timeout -k 10 300 ./tools/mixprobe > gpurun_out/mixprobe_tail.txt 2>&1
