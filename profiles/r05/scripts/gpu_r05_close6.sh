# round 5 close, part 6: the default bench line and smoke as the driver runs them, on the final
# library with its PMC file committed (roofline.traffic must be filled, not refused)
set -o pipefail
cd /root/repo
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
bash tools/gpu.sh smoke && bash tools/gpu.sh bench
