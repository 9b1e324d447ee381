# many-stream bandwidth probe + rocprofv3 trace / FETCH / WRITE of the vector-free bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 ./tools/vfprobe 100000000 7 > gpurun_out/vfprobe.txt 2>&1; rc=$?; echo "probe rc=$rc"; cat gpurun_out/vfprobe.txt
[ $rc -eq 0 ] || exit $rc
A="--vector-free --no-cpu-baseline --size 1e8"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/vf_trace -o run --output-format csv -- python3 bench.py --steps 30 --warmup 12 $A > gpurun_out/vf_trace.log 2>&1; rc=$?; echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/vf_fetch -o run --output-format csv -- python3 bench.py --steps 10 --warmup 12 --no-prof $A > gpurun_out/vf_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/vf_write -o run --output-format csv -- python3 bench.py --steps 10 --warmup 12 --no-prof $A > gpurun_out/vf_write.log 2>&1; rc=$?; echo "write rc=$rc"
