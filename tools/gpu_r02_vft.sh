# vector-free n = 1e4: tickets (in-launch stage 2 + completion word) vs the reduce kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for T in 1 0; do
LBFGS_TICKET=$T timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/vft_$T -o run --output-format csv -- python3 bench.py --size 1e4 --history 5 --steps 1000 --warmup 50 --no-cpu-baseline --vector-free --no-prof > gpurun_out/vft_$T.json 2>/dev/null || exit 1
python3 - <<PY
import csv, json
d = json.load(open("gpurun_out/vft_$T.json"))
print("ticket=$T", d["value"])
for r in csv.DictReader(open("gpurun_out/vft_$T/run_kernel_stats.csv")):
    if int(r["Calls"]) > 100: print("   ", r["Name"][:50], r["Calls"], r["AverageNs"])
PY
LBFGS_TICKET=$T timeout -k 10 120 python3 bench.py --size 1e4 --history 5 --steps 3000 --warmup 50 --no-cpu-baseline --vector-free --no-prof > gpurun_out/vft2_$T.json || exit 1
python3 -c "import json; print('ticket=$T uninstrumented', json.load(open('gpurun_out/vft2_$T.json'))['value'])"
done
