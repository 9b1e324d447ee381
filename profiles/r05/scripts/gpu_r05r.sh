# which step of bench.py's sequence leaves a host thread spinning beside the solver's (tools/thread_probe.py)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05r
timeout -k 10 300 python -u tools/thread_probe.py gpurun_out/r05r/threads.json > gpurun_out/r05r/threads.log 2>&1
