# which host interaction of the solver keeps a runtime thread spinning (tools/thread_probe.py
# --solves under the library's switches, one process each)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05v
P="timeout -k 10 120 python -u tools/thread_probe.py --solves 4"
$P gpurun_out/r05v/default.json > gpurun_out/r05v/all.log 2>&1 &&
LBFGS_SPEC=0 $P gpurun_out/r05v/spec0.json >> gpurun_out/r05v/all.log 2>&1 &&
LBFGS_DIRECT=0 $P gpurun_out/r05v/direct0.json >> gpurun_out/r05v/all.log 2>&1 &&
LBFGS_BATCH=0 $P gpurun_out/r05v/batch0.json >> gpurun_out/r05v/all.log 2>&1 &&
LBFGS_TICKET=0 $P gpurun_out/r05v/ticket0.json >> gpurun_out/r05v/all.log 2>&1 &&
LBFGS_COLLECT=0 $P gpurun_out/r05v/collect0.json >> gpurun_out/r05v/all.log 2>&1 &&
LBFGS_SPEC=0 LBFGS_BATCH=0 LBFGS_DIRECT=0 $P gpurun_out/r05v/spec0_batch0_direct0.json >> gpurun_out/r05v/all.log 2>&1
