# configs[4]'s sharded rate on one card (tools/gpu_r05b.sh), with a line a minute for the driver's
# watchdog while its steps (each under its own time limit) run without stdout
set -o pipefail
cd /root/repo
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
echo "r05b start"; bash tools/gpu_r05b.sh; rb=$?; echo "r05b rc=$rb"
exit $rb
