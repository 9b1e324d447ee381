# round 2 evidence on the current build: rocprofv3 kernel trace + PMC (FETCH_SIZE, WRITE_SIZE in
# their own passes) on the bench command, the default bench line, and the reference's configs[3]
# (tridiagonal quadratic n=1e8, m=20, Wolfe, to convergence) on one pinned host core
set -o pipefail
mkdir -p gpurun_out
(taskset -c 2 timeout -k 10 900 oracle/_ref/ref_lbfgs quad_tridiag 100000000 20 wolfe 1000 1e-5 42 -2 2 /tmp/cfg3 0 > gpurun_out/cpu_config3.log 2>&1; echo "cpu config3 rc=$?" >> gpurun_out/cpu_config3.log) &
CPU_PID=$!
bash tools/gpu_profile.sh 1e8 || exit 1
python tools/pmc_summary.py gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/pmc_bench_n1e8.json 1e8 > gpurun_out/pmc_summary.txt
grep -E "commit|axpy|mid|trials" gpurun_out/pmc_summary.txt | cut -c1-200
python3 - <<'PY'
import time, os, glob, struct, subprocess
PY
wait $CPU_PID
cat gpurun_out/cpu_config3.log | tail -3
python3 -c "
import numpy as np
g = np.fromfile('/tmp/cfg3.g.bin', dtype=np.uint64).reshape(-1, 5)
t = g[:, 3].copy().view(np.float64)
print('cpu config3: grad calls', len(g), 'last grad at', t[-1], 's')
" | tee -a gpurun_out/cpu_config3.log
