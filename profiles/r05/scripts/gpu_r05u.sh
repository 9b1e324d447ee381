# which host call makes a runtime thread spin while the stream is busy (tools/query_probe.hip, more modes)?
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05u
timeout -k 10 120 ./tools/query_probe > gpurun_out/r05u/query_probe.txt 2>&1
