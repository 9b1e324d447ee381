# tools/cpu_monitor.sh OUT [SECONDS] — once a second, this job's CPU budget and use (cgroup
# cpu.max / cpu.stat: periods, throttled periods and time; read only) and, for every bench.py
# process, each thread's name and cumulative user + system ticks (/proc/<pid>/task/*/stat), for
# SECONDS (default 600) or until killed (do the one-card N = 8 rehearsal's ranks get
# the CPU time to keep their queues fed?)
out=${1:?out file}
secs=${2:-600}
{
    echo "nproc $(nproc) clk_tck $(getconf CLK_TCK)"
    for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu/cpu.cfs_quota_us /sys/fs/cgroup/cpu/cpu.cfs_period_us \
             /sys/fs/cgroup/cpuset.cpus.effective; do
        [ -r "$f" ] && echo "$f: $(cat "$f")"
    done
    end=$((SECONDS + secs))
    while [ $SECONDS -lt $end ]; do
        echo "=== $(date +%T)"
        for f in /sys/fs/cgroup/cpu.stat /sys/fs/cgroup/cpu/cpu.stat; do
            [ -r "$f" ] && echo "cgroup $(tr '\n' ' ' < "$f")"
        done
        for p in /proc/[0-9]*; do
            grep -q "bench\.py" "$p/cmdline" 2> /dev/null || continue
            pid=${p#/proc/}
            for t in "$p"/task/*; do
                # comm may hold spaces: fields after the closing parenthesis; utime, stime = 14, 15
                s=$(cat "$t/stat" 2> /dev/null) || continue
                name=${s#*(}
                name=${name%%)*}
                rest=${s##*) }
                set -- $rest
                echo "t $pid ${t##*/} ${name// /_} $((${12} + ${13}))"
            done
        done
        sleep 1
    done
} > "$out" 2>&1
