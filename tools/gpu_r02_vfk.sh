# vector-free commit kernel time at small n against h (m = 1, 3, 5) and n
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for M in 1 3 5; do for N in 1e4 1e5; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/vfk_${M}_$N -o run --output-format csv -- python3 bench.py --size $N --history $M --steps 1000 --warmup 50 --no-cpu-baseline --vector-free --no-prof > gpurun_out/vfk_${M}_$N.json 2>/dev/null || exit 1
python3 - <<PY
import csv, json
d = json.load(open("gpurun_out/vfk_${M}_$N.json"))
for r in csv.DictReader(open("gpurun_out/vfk_${M}_$N/run_kernel_stats.csv")):
    if "vf_commit" in r["Name"] and int(r["Calls"]) > 100:
        print("m=${M} n=$N", d["value"], r["Name"][:45], r["Calls"], r["AverageNs"])
PY
done; done
