# round 5 close, part 3: every BASELINE config on one GPU (tools/bench_configs.py via tools/gpu.sh)
set -o pipefail
cd /root/repo
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
bash tools/gpu.sh configs
