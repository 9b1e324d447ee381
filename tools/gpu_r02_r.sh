# cooperative iteration (flagged partials + speculative launches) vs the launch sequence at mid n:
# where should LBFGS_COOP's default segment limit sit now
set -o pipefail
mkdir -p gpurun_out
for N in 2e5 3e5 5e5 7e5 1e6; do
  for C in 0 512; do
    LBFGS_COOP=$C timeout -k 10 120 python bench.py --size $N --steps 400 --warmup 20 --no-cpu-baseline --no-vector-free --no-prof > gpurun_out/coopab_${N}_$C.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/coopab_${N}_$C.json')); print('n=$N coop=$C', d['value'], d['ms_per_step'])"
  done
done
