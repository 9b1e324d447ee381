set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/small_vf_trace -o run --output-format csv -- python3 bench.py --size 1e4 --history 5 --steps 300 --warmup 20 --no-cpu-baseline --vector-free --no-prof > gpurun_out/small_vf_trace.log 2>&1; echo "rc=$?"
