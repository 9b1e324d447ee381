# the HIP runtime's own log (AMD_LOG_LEVEL=4) over three 30-iteration solves at n = 1e8, the
# spinning runtime thread's onset inside them (tools/thread_probe.py --solves)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05w
AMD_LOG_LEVEL=4 timeout -k 10 120 python -u tools/thread_probe.py --solves 3 gpurun_out/r05w/threads.json > gpurun_out/r05w/log.txt 2>&1
gzip -f gpurun_out/r05w/log.txt
