# tools/gpu_r06.sh — round 6's GPU-box steps (run through gpurun from the repo root). Every GPU step
# has its own time limit; steps are chained so the first failure ends the call. A heartbeat line a
# minute keeps the watchdog informed while a step writes nothing.
#
#   bash tools/gpu_r06.sh first      host facts, smoke, the new / changed GPU tests, the gap probe
#                                    plain and under rocprofv3 (kernel trace), the default bench line
#   bash tools/gpu_r06.sh gapbench   smoke, the stalled-collective test, the gap probe (plain, traced), bench
#   bash tools/gpu_r06.sh waitab     LBFGS_WAIT=spin against adaptive, alternating, n = 1e8 and 1e4
#   bash tools/gpu_r06.sh config4deep  configs[4]'s canonical oracle run at n = 1e9 on the box's host
#   bash tools/gpu_r06.sh cleantrace   kernel trace of the bench steps without any HIP events
#   bash tools/gpu_r06.sh gappmc     SQ / TA counter passes over the gap probe (one pass per run)
#   bash tools/gpu_r06.sh stress R  tools/repeat_stress.py R reps, the default (plain) vectors then contiguous ones
#   bash tools/gpu_r06.sh vflane     tools/vflaneprobe: the vector-free stream shape, one element per lane vs two
#   bash tools/gpu_r06.sh tests ARGS pytest -m gpu over ARGS (default: tests)
#   bash tools/gpu_r06.sh bench ARGS one bench.py line -> gpurun_out/r06/bench.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT

host_facts() {
    { date; free -g; nproc; cat /sys/fs/cgroup/cpu.max 2> /dev/null; cat /sys/fs/cgroup/memory.max 2> /dev/null;
      df -h /tmp . | tail -2; } > $O/host_facts.txt 2>&1
    cat $O/host_facts.txt
}

smoke() {
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
    local rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; return $rc
}

tests() {
    local args=("$@"); [ ${#args[@]} -eq 0 ] && args=(tests)
    timeout -k 10 1000 python -u -m pytest "${args[@]}" -m gpu -v --durations=40 --timeout 300 --timeout-method thread \
        > $O/pytest.log 2>&1 &
    local pid=$! n=0
    while kill -0 $pid 2> /dev/null; do
        sleep 5; n=$((n + 1))
        [ $((n % 12)) -eq 0 ] && echo "tests running: $(grep -c -E 'PASSED|FAILED|ERROR' $O/pytest.log) results"
    done
    wait $pid
    local rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -15; return $rc
}

gap() {
    timeout -k 10 400 python tools/gap_probe.py $O/gap_probe.json 1e8 4 > $O/gap_probe.log 2>&1
    local rc=$?; echo "gap rc=$rc"; tail -6 $O/gap_probe.log; return $rc
}

gap_trace() {
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/gap_trace -o run --output-format csv -- \
        python3 tools/gap_probe.py $O/gap_probe_traced.json 1e8 2 > $O/gap_trace.log 2>&1
    local rc=$?; echo "gap trace rc=$rc"; tail -3 $O/gap_trace.log; return $rc
}

gap_pmc() {  # one counter pass: $1 = tag, rest = counters
    local tag=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" -d $O/gap_pmc_$tag -o run --output-format csv -- \
        python3 tools/gap_probe.py $O/gap_probe_pmc_$tag.json 1e8 1 > $O/gap_pmc_$tag.log 2>&1
    local rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || tail -5 $O/gap_pmc_$tag.log; return $rc
}

bench() {
    timeout -k 10 900 python bench.py "$@" > $O/bench.json 2> $O/bench.err
    local rc=$?; echo "bench rc=$rc"; cut -c1-1500 $O/bench.json; [ $rc -eq 0 ] || tail -20 $O/bench.err
    return $rc
}

case "$1" in
    first)
        host_facts && smoke &&
        tests tests/test_gpu_rccl.py tests/test_gpu_host_threads.py tests/test_gpu_device_search.py \
              tests/test_gpu_coop_safety.py tests/test_gpu_persist.py "tests/test_gpu_fullsize.py::test_fullsize_parity" &&
        gap && gap_trace && bench ;;
    gapbench)
        smoke && tests tests/test_gpu_rccl.py -k stalled && gap && gap_trace && bench && bash $0 waitab ;;
    waitab)  # the spin-then-sleep host wait against the spinning one, alternating, n = 1e8 and 1e4
        for r in 1 2; do
            for w in spin adaptive; do
                LBFGS_WAIT=$w timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline \
                    --no-vector-free --no-persistent > $O/wait_${w}_n1e8_$r.json 2> $O/wait_${w}_n1e8_$r.err || exit 1
                LBFGS_WAIT=$w timeout -k 10 300 python bench.py --size 1e4 --history 5 --steps 20000 --warmup 2000 \
                    --no-cpu-baseline --no-vector-free --no-persistent --no-box-probe > $O/wait_${w}_n1e4_$r.json \
                    2> $O/wait_${w}_n1e4_$r.err || exit 1
                python -c "
import json
for n in ('1e8', '1e4'):
    d = json.load(open('$O/wait_${w}_n' + n + '_$r.json'))
    print('$w', n, '$r', d['value'], d['host'])" | tee -a $O/wait_ab.txt
            done
        done ;;
    config4deep)  # configs[4]'s whole canonical run on this box's host (~265 GB, OpenMP oracle)
        timeout -k 10 1100 python -u tests/golden/make_fullsize.py config4_deep $O/config4_canon_deep.json 13 \
            > $O/config4_deep.log 2>&1
        rc=$?; echo "config4 deep rc=$rc"; tail -5 $O/config4_deep.log; exit $rc ;;
    cleantrace)  # the bench's timed steps under a kernel trace with no HIP events anywhere (--no-prof)
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/clean_trace -o run --output-format csv -- \
            python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-prof --no-box-probe --no-vector-free \
            --no-persistent > $O/clean_trace.log 2>&1
        rc=$?; echo "clean trace rc=$rc"; tail -2 $O/clean_trace.log | cut -c1-300; exit $rc ;;
    gappmc)
        timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
        gap_pmc a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                  SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR &&
        gap_pmc b SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD \
                  SQ_INST_CYCLES_VMEM_WR SQ_WAVES_RESTORED &&
        gap_pmc c FETCH_SIZE &&
        gap_pmc d WRITE_SIZE &&
        gap_pmc e TA_BUSY_avr TA_BUSY_max &&
        python tools/gap_pmc_summary.py $O/gap_pmc_summary.json $O/gap_pmc_? > $O/gap_pmc_summary.txt ;;
    stress)  # the shipped (plain) allocation first, then LBFGS_VEC_ALLOC=contiguous
        R=${2:-20}
        timeout -k 10 500 python -u tools/repeat_stress.py $O/stress_default.json $R > $O/stress_default.log 2>&1
        rc=$?; echo "stress default rc=$rc"; tail -2 $O/stress_default.log; [ $rc -eq 0 ] || exit $rc
        LBFGS_VEC_ALLOC=contiguous timeout -k 10 500 python -u tools/repeat_stress.py $O/stress_contig.json $R \
            > $O/stress_contig.log 2>&1
        rc=$?; echo "stress contiguous rc=$rc"; tail -2 $O/stress_contig.log; exit $rc ;;
    stressab)  # which side's contiguous allocations matter: the destroyed contexts' or the new ones'
        R=${2:-100}
        for modes in contiguous,contiguous contiguous,plain plain,contiguous; do
            timeout -k 10 300 python -u tools/repeat_stress.py $O/stress_$modes.json $R churn,vf4 $modes \
                > $O/stress_$modes.log 2>&1
            rc=$?; echo "stress $modes rc=$rc"; tail -1 $O/stress_$modes.log; [ $rc -eq 0 ] || exit $rc
        done ;;
    pool)  # the contiguous pool: stress with every vector pooled, then pool against plain at n = 1e8
        LBFGS_VEC_POOL_MIN_MB=0 timeout -k 10 400 python -u tools/repeat_stress.py $O/stress_pool_all.json 300 \
            > $O/stress_pool_all.log 2>&1
        rc=$?; echo "stress pool rc=$rc"; tail -1 $O/stress_pool_all.log; [ $rc -eq 0 ] || exit $rc
        for r in 1 2; do
            for v in pool plain; do
                LBFGS_VEC_ALLOC=$v timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline \
                    --no-vector-free --no-persistent > $O/poolab_${v}_$r.json 2> $O/poolab_${v}_$r.err || exit 1
                python -c "
import json
d = json.load(open('$O/poolab_${v}_$r.json'))
print('$v', '$r', d['value'], d['roofline']['avg_launch_us'], d['box_copy_tbps'], d['vectors'])" | tee -a $O/poolab.txt
            done
        done ;;
    vfpool)  # the vector-free line with pooled against plain vectors, alternating
        for r in 1 2; do
            for v in pool plain; do
                LBFGS_VEC_ALLOC=$v timeout -k 10 300 python bench.py --vector-free --steps 100 --warmup 20 \
                    --no-cpu-baseline --no-persistent > $O/vfpool_${v}_$r.json 2> $O/vfpool_${v}_$r.err || exit 1
                python -c "
import json
d = json.load(open('$O/vfpool_${v}_$r.json'))
print('$v', '$r', d['value'], d['roofline']['avg_launch_us'], d['box_copy_tbps'])" | tee -a $O/vfpool.txt
            done
        done ;;
    midn)  # mid n on the final library: collect against the reduce kernel, alternating, and a trace
        for r in 1 2; do
            for n in 2.5e6 5e6; do
                for col in 0 1; do
                    LBFGS_COLLECT=$col timeout -k 10 200 python bench.py --size $n --steps 400 --warmup 40 \
                        --no-cpu-baseline --no-vector-free --no-persistent --no-box-probe \
                        > $O/midn_${n}_c${col}_$r.json 2> $O/midn_${n}_c${col}_$r.err || exit 1
                    python -c "
import json
d = json.load(open('$O/midn_${n}_c${col}_$r.json'))
print('$n', 'collect=$col', '$r', d['value'], d['ms_per_step'], d['roofline']['kernel_share'])" | tee -a $O/midn.txt
                done
            done
        done
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/midn_trace -o run --output-format csv -- \
            python3 bench.py --size 2.5e6 --steps 200 --warmup 20 --no-cpu-baseline --no-vector-free --no-persistent \
            --no-box-probe --no-prof > $O/midn_trace.log 2>&1
        rc=$?; echo "midn trace rc=$rc"; exit $rc ;;
    stressbig)  # the stress at 10x sizes (churn 0.65-10 M, 4 ranks of 1e7: pooled vectors), default
        # allocation, then freed-contiguous as the positive control
        for md in default contiguous; do
            LBFGS_VEC_ALLOC=$([ $md = default ] && echo pool || echo contiguous) timeout -k 10 400 python -u \
                tools/repeat_stress.py $O/stressbig_$md.json ${2:-120} small,churn,vf4 default,default 10 \
                > $O/stressbig_$md.log 2>&1
            rc=$?; echo "stressbig $md rc=$rc"; tail -1 $O/stressbig_$md.log; [ $rc -eq 0 ] || exit $rc
        done ;;
    persistab)  # the persistent two-loop (noinline passes): 4 waves (shipped) / 6 / 8 per SIMD
        for r in 1 2; do
            for v in base pw6 pw8; do
                lib=cuda-lbfgs_amd/liblbfgs_hip.so; wg=4
                [ $v = pw6 ] && lib=cuda-lbfgs_amd/liblbfgs_hip_pw6.so && wg=6
                [ $v = pw8 ] && lib=cuda-lbfgs_amd/liblbfgs_hip_pw8.so && wg=8
                LBFGS_LIB=$lib LBFGS_PERSIST_WG=$wg timeout -k 10 300 python bench.py --steps 100 --warmup 20 \
                    --no-cpu-baseline --no-vector-free > $O/persistab_${v}_$r.json 2> $O/persistab_${v}_$r.err || exit 1
                python -c "
import json
d = json.load(open('$O/persistab_${v}_$r.json'))
p = d['persistent']
print('$v', '$r', d['value'], p['value'], p['vs_default'], p['trajectory_bit_identical_to_default'], p['roofline']['avg_launch_us'])" | tee -a $O/persistab.txt
            done
        done ;;
    segbarab)  # the persistent two-loop with one barrier per pass (shipped candidate) against two per segment
        bash $0 tests tests/test_gpu_persist.py "tests/test_gpu_fullsize.py::test_fullsize_parity" || exit 1
        for r in 1 2; do
            for v in onebar segbar; do
                lib=cuda-lbfgs_amd/liblbfgs_hip.so
                [ $v = segbar ] && lib=cuda-lbfgs_amd/liblbfgs_hip_segbar.so
                LBFGS_LIB=$lib timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline \
                    --no-vector-free > $O/segbar_${v}_$r.json 2> $O/segbar_${v}_$r.err || exit 1
                python -c "
import json
d = json.load(open('$O/segbar_${v}_$r.json'))
p = d['persistent']
print('$v', '$r', d['value'], p['value'], p['vs_default'], p['trajectory_bit_identical_to_default'], p['roofline']['avg_launch_us'])" | tee -a $O/segbar.txt
            done
        done ;;
    persisttrace)  # kernel trace of the persistent mode's timed steps (LBFGS_PERSIST=2 as the headline mode)
        LBFGS_PERSIST=2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/persist_trace -o run --output-format csv -- \
            python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-prof --no-box-probe --no-vector-free \
            --no-persistent > $O/persist_trace.log 2>&1
        rc=$?; echo "persist trace rc=$rc"; tail -1 $O/persist_trace.log | cut -c1-200; exit $rc ;;
    strideab)  # persistent ownership: contiguous chunks (shipped) against strided segments (variant)
        for r in 1 2; do
            for v in chunk stride; do
                lib=cuda-lbfgs_amd/liblbfgs_hip.so
                [ $v = stride ] && lib=cuda-lbfgs_amd/liblbfgs_hip_stride.so
                LBFGS_LIB=$lib timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline \
                    --no-vector-free > $O/stride_${v}_$r.json 2> $O/stride_${v}_$r.err || exit 1
                python -c "
import json
d = json.load(open('$O/stride_${v}_$r.json'))
p = d['persistent']
print('$v', '$r', d['value'], p['value'], p['vs_default'], p['trajectory_bit_identical_to_default'], p['roofline']['avg_launch_us'])" | tee -a $O/stride.txt
            done
        done ;;
    vflane)
        timeout -k 10 300 tools/vflaneprobe 1e8 9 > $O/vflaneprobe.txt 2>&1
        rc=$?; echo "vflane rc=$rc"; cat $O/vflaneprobe.txt; exit $rc ;;
    tests) shift; tests "$@" ;;
    bench) shift; bench "$@" ;;
    *) echo "unknown part $1"; exit 2 ;;
esac
