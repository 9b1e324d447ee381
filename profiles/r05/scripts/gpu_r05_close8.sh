# round 5 close, part 8: the driver's N = 4 command self-launched on this one card (the final
# library; N = 2 and 8 are in parts 4 and 5). A line a minute for the watchdog.
set -o pipefail
cd /root/repo
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
LBFGS_CU_PARTITION=1 LBFGS_RCCL_TIMEOUT=30 bash tools/gpu.sh selflaunch 4
