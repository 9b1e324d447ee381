# Round-end evidence in one call: GPU suite, smoke(), rocprofv3 trace + PMC of the headline
# bench, the headline line with the CPU baseline, every BASELINE config, the published-table
# comparison and the five-seed protocol. Outputs under gpurun_out/final/.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trace -o run --output-format csv -- python3 bench.py --steps 30 --warmup 12 --no-cpu-baseline > $O/prof_trace.log 2>&1 || { echo trace failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch -o run --output-format csv -- python3 bench.py --steps 10 --warmup 12 --no-cpu-baseline --no-prof > $O/prof_fetch.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write -o run --output-format csv -- python3 bench.py --steps 10 --warmup 12 --no-cpu-baseline --no-prof > $O/prof_write.log 2>&1 || { echo write failed; exit 1; }
python tools/pmc_summary.py $O/prof_trace $O/prof_fetch $O/prof_write $O/pmc_bench_n1e8.json 100000000 > $O/pmc_summary.log 2>&1 || { echo pmc_summary failed; tail $O/pmc_summary.log; }
echo profiles done
timeout -k 10 600 python bench.py > $O/bench_n1e8.json 2> $O/bench_n1e8.err || { echo bench failed; tail $O/bench_n1e8.err; exit 1; }
cat $O/bench_n1e8.json
timeout -k 10 900 python -u tools/bench_configs.py $O/configs.json > $O/configs.log 2>&1; echo "configs rc=$?"
timeout -k 10 600 python -u tools/paper_table.py $O/paper_table.json > $O/paper_table.log 2>&1; echo "paper rc=$?"
timeout -k 10 900 python -u tools/seeds5.py $O/seeds5.json > $O/seeds5.log 2>&1; echo "seeds5 rc=$?"
