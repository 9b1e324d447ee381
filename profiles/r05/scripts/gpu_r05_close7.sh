# round 5 close, part 7: smoke and the whole -m gpu suite on the final tree (tools/gpu.sh)
set -o pipefail
cd /root/repo
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
bash tools/gpu.sh smoke && bash tools/gpu.sh suite
