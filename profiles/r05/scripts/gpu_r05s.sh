# does polling hipStreamQuery while the stream is busy make a runtime thread spin (tools/query_probe.hip)?
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05s
timeout -k 10 120 ./tools/query_probe > gpurun_out/r05s/query_probe.txt 2>&1
