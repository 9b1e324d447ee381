set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_n1e8.json 2>gpurun_out/bench.err || exit 3
cat gpurun_out/bench_n1e8.json
timeout -k 10 300 python bench.py --no-cpu-baseline --size 1e7 > gpurun_out/bench_n1e7.json 2>>gpurun_out/bench.err || exit 3
cat gpurun_out/bench_n1e7.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1e7 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 12 --no-cpu-baseline --size 1e7 > gpurun_out/prof_1e7.log 2>&1; echo "trace rc=$?"
