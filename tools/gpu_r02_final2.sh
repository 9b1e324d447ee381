# final evidence on the final build: smoke, bench line + rocprofv3 trace + PMC, every config,
# the paper's Table I comparison
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_profile.sh 1e8 > gpurun_out/profile.log 2>&1 || { tail -5 gpurun_out/profile.log; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/pmc_bench_n1e8.json 1e8 > gpurun_out/pmc_summary.txt
python -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print('bench', d['value'], d['roofline']['frac'], d['build'])"
timeout -k 10 600 python tools/bench_configs.py gpurun_out/configs.json > gpurun_out/configs.log 2>&1 || { tail -5 gpurun_out/configs.log; exit 1; }
timeout -k 10 300 python tools/paper_table.py gpurun_out/paper_table.json > gpurun_out/paper_table.log 2>&1 || { tail -5 gpurun_out/paper_table.log; exit 1; }
grep -o '^[a-z_]* \|"speedup_default": [0-9.]*\|"speedup_vector_free": [0-9.]*' gpurun_out/paper_table.log | paste - - -
