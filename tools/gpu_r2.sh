# GPU suite, then vector-free bench at the sizes its segment geometry changed, then the
# 8-rank one-GPU rehearsal of the sharded default mode (fused TWOLOOP commit)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit 1; }
for n in 1e6 1.5e6 3e6 1e7 2e7 1e8; do
  timeout -k 10 300 python bench.py --vector-free --no-cpu-baseline --size $n --steps 100 --warmup 20 > gpurun_out/vf_$n.json 2>gpurun_out/vf.err || { tail gpurun_out/vf.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/vf_$n.json'));r=d['roofline'];print('vf n=$n', d['value'], 'it/s', r['kernel'], r['achieved'], r['avg_launch_us'])"
done
BENCH_DEVICE_MOD=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --size 1e8 --steps 10 --warmup 12 --no-cpu-baseline > gpurun_out/xgmi_bench8.log 2>&1; rc=$?
echo "bench W=8 rc=$rc"; grep '^{' gpurun_out/xgmi_bench8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['bytes_per_step'], d['roofline']['kernel_share'], d['vector_free']['value'])" || tail -30 gpurun_out/xgmi_bench8.log
