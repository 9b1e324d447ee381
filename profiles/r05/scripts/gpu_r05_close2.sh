# round 5 close, part 2: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the bench at n = 1e8
# and the default bench line (tools/gpu.sh profile), then the paper's per-line-search table.
# A line a minute for the watchdog.
set -o pipefail
cd /root/repo
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
bash tools/gpu.sh profile 1e8 &&
timeout -k 10 600 python -u tools/paper_table.py gpurun_out/paper_table.json > gpurun_out/paper_table.log 2>&1
