# kernel trace of the default mode at mid n (where boundaries and stage 2 dominate)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in ${SIZES:-1e6 3e6}; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mid_trace_$S -o run --output-format csv -- python3 bench.py --size $S --steps 100 --warmup 20 --no-cpu-baseline --no-vector-free --no-prof --no-config4 > gpurun_out/mid_trace_$S.log 2>&1; echo "rc=$?"
tail -1 gpurun_out/mid_trace_$S.log | cut -c1-200
done
