# round 5 close, part 1: smoke, the whole -m gpu suite (tools/gpu.sh), a line a minute for the watchdog
set -o pipefail
cd /root/repo
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
bash tools/gpu.sh smoke && bash tools/gpu.sh suite
