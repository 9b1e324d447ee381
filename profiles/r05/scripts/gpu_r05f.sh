# one box: the device-resident line searches (tools/gpu_r05c.sh), then the paired-row vector-free
# A/B (tools/gpu_r05d.sh); a line a minute for the watchdog while steps run without stdout
set -o pipefail
cd /root/repo
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
echo "r05c start"; bash tools/gpu_r05c.sh; rc=$?; echo "r05c rc=$rc"
[ $rc -eq 0 ] || exit $rc
echo "r05d start"; bash tools/gpu_r05d.sh; rd=$?; echo "r05d rc=$rd"
exit $rd
