# shard_check in a 2-rank rehearsal on one card; small-n kernel time vs iteration time (n=1e4)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_DEVICE_MOD=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 2 --size 2e7 --steps 20 --warmup 5 --no-cpu-baseline --no-vector-free > gpurun_out/w2_check.log 2>&1; rc=$?
echo "w2 rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/w2_check.log; exit 1; }
grep '^{' gpurun_out/w2_check.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['exchange'], d['shard_check'])"
timeout -k 10 120 python bench.py --size 1e4 --history 5 --steps 3000 --warmup 100 --no-cpu-baseline --no-vector-free --no-prof > gpurun_out/small_plain.json; rc=$?; echo "plain rc=$rc"; [ $rc -eq 0 ] || exit 1
python -c "import json; d=json.load(open('gpurun_out/small_plain.json')); print('n=1e4 default', d['value'], d['ms_per_step'])"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o run --output-format csv -- python3 bench.py --size 1e4 --history 5 --steps 3000 --warmup 100 --no-cpu-baseline --no-vector-free --no-prof > gpurun_out/prof_small.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit 1
cut -c1-60,150-400 gpurun_out/prof_small/run_kernel_stats.csv | head
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small_vf -o run --output-format csv -- python3 bench.py --size 1e4 --history 5 --steps 3000 --warmup 100 --no-cpu-baseline --vector-free --no-prof > gpurun_out/prof_small_vf.log 2>&1; rc=$?; echo "prof vf rc=$rc"; [ $rc -eq 0 ] || exit 1
cut -c1-60,150-400 gpurun_out/prof_small_vf/run_kernel_stats.csv | head
