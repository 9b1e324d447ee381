# rocprofv3 evidence for profiles/: kernel trace + stats, then PMC FETCH_SIZE and WRITE_SIZE in
# separate passes (gfx950 slot limits), all on the bench command; then the full default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${1:-1e8}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py --steps 30 --warmup 12 --no-cpu-baseline --size $N > gpurun_out/prof_trace.log 2>&1; rc=$?; echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python3 bench.py --steps 10 --warmup 12 --no-cpu-baseline --no-prof --size $N > gpurun_out/prof_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python3 bench.py --steps 10 --warmup 12 --no-cpu-baseline --no-prof --size $N > gpurun_out/prof_write.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --size $N > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_default.json
