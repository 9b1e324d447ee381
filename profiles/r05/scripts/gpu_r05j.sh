# the cooperative-launch probe, then every BASELINE config on one GPU
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05j
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
timeout -k 10 300 tools/cooplaunch_probe > gpurun_out/r05j/cooplaunch_probe.txt 2>&1 &&
bash tools/gpu.sh configs
