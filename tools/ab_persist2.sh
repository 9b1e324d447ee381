# A/B of the persistent forms against the launch sequence: the persistent tests
# first, then alternating bench lines. usage: bash tools/ab_persist2.sh [n ...] (default 1e8)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_persist.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_persist.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, size, env...
    local name=$1 size=$2; shift 2
    local steps=50; [ "${size%e*}" != "$size" ] && [ "${size#*e}" -le 7 ] && steps=300
    env "$@" timeout -k 10 300 python bench.py --size "$size" --steps $steps --warmup 20 --no-cpu-baseline \
        --no-vector-free > "gpurun_out/ab_$name.json" 2> "gpurun_out/ab_$name.err" || { tail -5 "gpurun_out/ab_$name.err"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));print('$name', d['value'], d['ms_per_step'], d['achieved_hbm_gbps'])"
}
sizes=("$@"); [ ${#sizes[@]} -eq 0 ] && sizes=(1e8)
for n in "${sizes[@]}"; do
    for r in 1 2; do
        run "n${n}_seq_$r" "$n" LBFGS_PERSIST=0
        run "n${n}_p2wg1_$r" "$n" LBFGS_PERSIST=2 LBFGS_PERSIST_WG=1
        run "n${n}_p2wg2_$r" "$n" LBFGS_PERSIST=2 LBFGS_PERSIST_WG=2
        run "n${n}_p2wg4_$r" "$n" LBFGS_PERSIST=2 LBFGS_PERSIST_WG=4
    done
done
