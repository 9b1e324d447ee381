# tools/gpu.sh — the GPU-box steps behind the evidence in profiles/, one parameterised script
# (run on the box through gpurun from the repo root; every GPU step has its own time limit and the
# steps stop at the first failure):
#
#   bash tools/gpu.sh smoke                    __graft_entry__.smoke()
#   bash tools/gpu.sh suite [pytest args]      the -m gpu suite (default: all of tests/)
#   bash tools/gpu.sh bench [bench args]       one bench.py line -> gpurun_out/bench.json
#   bash tools/gpu.sh profile [N]              rocprofv3 kernel trace + stats, FETCH_SIZE and WRITE_SIZE
#                                              passes (separate runs) of the bench command at n = N,
#                                              tools/pmc_summary.py over them, then the default bench
#   bash tools/gpu.sh rehearse W [bench args]  the driver's N = W bench line with W ranks on this one
#                                              card (BENCH_DEVICE_MOD=1, xGMI mailboxes between processes)
#   bash tools/gpu.sh selflaunch W [bench args] the same with NO launcher around bench.py (its own
#                                              self_launch starts the W ranks), as the driver's
#                                              N > 1 command without a wrapper
#   bash tools/gpu.sh cumask                   tools/cumaskprobe: LBFGS_CU_PARTITION's masks give the
#                                              ranks disjoint CUs
#   bash tools/gpu.sh configs [args]           tools/bench_configs.py (every BASELINE config on one GPU)
#   bash tools/gpu.sh close                    smoke, suite, profile 1e8 (a round's closing evidence)
#
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp

step_smoke() {
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    local rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; return $rc
}

step_suite() {
    local args=("$@"); [ ${#args[@]} -eq 0 ] && args=(tests)
    timeout -k 10 1000 python -u -m pytest "${args[@]}" -m gpu -v --timeout 300 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1 &
    local pid=$! n=0
    # a progress line a minute (a multi-process test can run a few minutes without a result line)
    while kill -0 $pid 2> /dev/null; do
        sleep 5; n=$((n + 1))
        [ $((n % 12)) -eq 0 ] && echo "suite running: $(grep -c -E 'PASSED|FAILED|ERROR' gpurun_out/pytest_gpu.log) results"
    done
    wait $pid
    local rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; return $rc
}

step_bench() {
    timeout -k 10 900 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
    local rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -eq 0 ] || tail -20 gpurun_out/bench.err
    return $rc
}

step_profile() {
    local N=${1:-1e8} rc
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- \
        python3 bench.py --steps 30 --warmup 12 --no-cpu-baseline --size "$N" > gpurun_out/prof_trace.log 2>&1
    rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || return $rc
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- \
        python3 bench.py --steps 10 --warmup 12 --no-cpu-baseline --no-prof --no-box-probe --size "$N" \
        > gpurun_out/prof_fetch.log 2>&1
    rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || return $rc
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- \
        python3 bench.py --steps 10 --warmup 12 --no-cpu-baseline --no-prof --no-box-probe --size "$N" \
        > gpurun_out/prof_write.log 2>&1
    rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || return $rc
    python tools/pmc_summary.py gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write \
        "gpurun_out/pmc_bench_n$N.json" "$N" gpurun_out/prof_trace.log gpurun_out/prof_fetch.log \
        gpurun_out/prof_write.log > gpurun_out/pmc_summary.txt || return 1
    # the CPU baseline runs the reference at the bench's n: only at the headline size (at 1e9 it
    # would take ~12 minutes of silent CPU work)
    if [ "$N" = 1e8 ]; then step_bench --size "$N"; else step_bench --size "$N" --no-cpu-baseline; fi
}

step_rehearse() {
    local W=$1; shift
    BENCH_DEVICE_MOD=1 timeout -k 10 1100 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$W" \
        --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus "$W" "$@" > "gpurun_out/rehearse_w$W.log" 2>&1 &
    local pid=$! n=0
    while kill -0 $pid 2> /dev/null; do  # a progress line a minute
        sleep 5; n=$((n + 1)); [ $((n % 12)) -eq 0 ] && echo "rehearse W=$W running ($((n * 5)) s)"
    done
    wait $pid
    local rc=$?; echo "rehearse W=$W rc=$rc"
    [ $rc -eq 0 ] || { tail -30 "gpurun_out/rehearse_w$W.log"; return 1; }
    grep '^{' "gpurun_out/rehearse_w$W.log" > "gpurun_out/rehearse_w$W.json"; cat "gpurun_out/rehearse_w$W.json"
}

step_selflaunch() {
    local W=$1; shift
    BENCH_DEVICE_MOD=1 timeout -k 10 1100 python bench.py --gpus "$W" "$@" \
        > "gpurun_out/selflaunch_w$W.json" 2> "gpurun_out/selflaunch_w$W.err" &
    local pid=$! n=0
    while kill -0 $pid 2> /dev/null; do  # a progress line a minute
        sleep 5; n=$((n + 1)); [ $((n % 12)) -eq 0 ] && echo "selflaunch W=$W running ($((n * 5)) s)"
    done
    wait $pid
    local rc=$?; echo "selflaunch W=$W rc=$rc"
    [ $rc -eq 0 ] || { tail -30 "gpurun_out/selflaunch_w$W.err"; return 1; }
    cat "gpurun_out/selflaunch_w$W.json"
}

step_cumask() {
    [ -x tools/cumaskprobe ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/cumaskprobe.hip -o tools/cumaskprobe || return 1
    timeout -k 10 120 tools/cumaskprobe > gpurun_out/cumaskprobe.txt 2>&1
    local rc=$?; echo "cumask rc=$rc"; cat gpurun_out/cumaskprobe.txt; return $rc
}

step_configs() {
    timeout -k 10 1100 python tools/bench_configs.py gpurun_out/configs.json "$@" > gpurun_out/configs.log 2>&1
    local rc=$?; echo "configs rc=$rc"; tail -5 gpurun_out/configs.log; return $rc
}

[ $# -ge 1 ] || { sed -n '3,21p' "$0"; exit 2; }
case "$1" in
    smoke|suite|bench|profile|rehearse|selflaunch|cumask|configs) cmd=$1; shift; "step_$cmd" "$@"; exit $? ;;
    close) step_smoke && step_suite && step_profile 1e8; exit $? ;;
    *) echo "unknown step $1"; exit 2 ;;
esac
