# Full GPU check of the tree: GPU tests, smoke(), the headline bench line, and a 2-rank RCCL
# rehearsal on one card (BENCH_DEVICE_MOD=1). Every GPU step has its own time limit; any failure
# ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ "${RCCL2:-1}" = 1 ]; then
  BENCH_DEVICE_MOD=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --size 2e7 --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/rccl2.log 2>&1; echo "rccl2 rc=$?"; tail -5 gpurun_out/rccl2.log
fi
