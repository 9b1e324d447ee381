# tools/kfd_queues.sh OUT [SECONDS] — every second, the KFD user queues of every process on the
# host (/sys/class/kfd/kfd/proc/<pid>/queues/<id>/{gpuid,type}, read only), counted per GPU and
# queue type and per process, for SECONDS (default 600) or until killed; first the amdgpu
# scheduler parameters that bound how many queues the hardware scheduler maps at once (DESIGN.md §5,
# configs[4] on one card). The host may run other jobs on other GPUs: group by gpuid.
out=${1:?out file}
secs=${2:-600}
{
    for p in sched_policy hws_max_conc_proc cwsr_enable mes; do
        f=/sys/module/amdgpu/parameters/$p
        [ -r "$f" ] && echo "param $p=$(cat "$f")"
    done
    q=$(ls -d /sys/class/kfd/kfd/proc/*/queues/* 2> /dev/null | head -1)
    [ -n "$q" ] && echo "queue attributes: $(ls "$q" | tr '\n' ' ')"
    end=$((SECONDS + secs))
    while [ $SECONDS -lt $end ]; do
        declare -A per_gt=() per_pid=()
        for d in /sys/class/kfd/kfd/proc/*/queues/*; do
            [ -d "$d" ] || continue
            g=$(cat "$d/gpuid" 2> /dev/null)
            t=$(cat "$d/type" 2> /dev/null)
            pid=${d#/sys/class/kfd/kfd/proc/}
            pid=${pid%%/*}
            per_gt["$g/$t"]=$((${per_gt["$g/$t"]:-0} + 1))
            per_pid["$g:$pid"]=$((${per_pid["$g:$pid"]:-0} + 1))
        done
        line="$(date +%T) |"
        for k in $(printf '%s\n' "${!per_gt[@]}" | sort); do line="$line $k=${per_gt[$k]}"; done
        line="$line ||"
        for k in $(printf '%s\n' "${!per_pid[@]}" | sort); do line="$line $k=${per_pid[$k]}"; done
        echo "$line"
        unset per_gt per_pid
        sleep 1
    done
} > "$out" 2>&1
