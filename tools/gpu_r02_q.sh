# mid n: where an iteration's time goes at n = 1e7 (configs[1]) and 2e6
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for N in 1e7 2e6; do
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mid_$N -o run --output-format csv -- python3 bench.py --size $N --steps 200 --warmup 20 --no-cpu-baseline --no-vector-free --no-prof > gpurun_out/prof_mid_$N.json 2> gpurun_out/prof_mid_$N.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/prof_mid_$N.json')); print('$N', d['value'], d['ms_per_step'], d['achieved_hbm_gbps'])"
done
