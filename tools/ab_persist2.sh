# A/B of the persistent forms against the launch sequence at n = 1e8: the
# persistent tests first, then alternating bench lines (LBFGS_PERSIST=0 / 2 / 1, and grid caps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_persist.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_persist.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-vector-free \
        > "gpurun_out/ab_$name.json" 2> "gpurun_out/ab_$name.err" || { tail -5 "gpurun_out/ab_$name.err"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));print('$name', d['value'], d['ms_per_step'], d['roofline']['kernel_share'])"
}
for r in 1 2 3; do
    run seq_$r LBFGS_PERSIST=0
    run p2_wg1_lds_$r LBFGS_PERSIST=2 LBFGS_PERSIST_WG=1
    run p2_wg2_lds_$r LBFGS_PERSIST=2 LBFGS_PERSIST_WG=2
    run p2_wg1_nolds_$r LBFGS_PERSIST=2 LBFGS_PERSIST_WG=1 LBFGS_PERSIST_LDS=0
done
run p2_wg3_lds LBFGS_PERSIST=2 LBFGS_PERSIST_WG=3
run p1_wg2_lds LBFGS_PERSIST=1 LBFGS_PERSIST_WG=2
