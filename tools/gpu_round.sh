# One GPU session: calibration probe, GPU tests, smoke, full bench, rocprofv3 trace + PMC.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 ./tools/bwprobe 100000000 10 > gpurun_out/bwprobe.txt 2>&1; echo "bwprobe rc=$?"; cat gpurun_out/bwprobe.txt
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full.json; tail -3 gpurun_out/bench_full.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py --steps 30 --warmup 12 --no-cpu-baseline > gpurun_out/prof_trace.log 2>&1; rc=$?; echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python3 bench.py --steps 10 --warmup 12 --no-cpu-baseline --no-prof > gpurun_out/prof_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python3 bench.py --steps 10 --warmup 12 --no-cpu-baseline --no-prof > gpurun_out/prof_write.log 2>&1; rc=$?; echo "write rc=$rc"
