# tools/smi_monitor.sh OUT [SECONDS] — once a second, rocm-smi's power, temperatures, clocks and
# use for every GPU it sees (read only), for SECONDS (default 600) or until killed (DESIGN.md §5:
# do long HBM-bound runs slow down as the card heats?)
out=${1:?out file}
secs=${2:-600}
{
    rocm-smi --showmaxpower --showperflevel 2>&1
    end=$((SECONDS + secs))
    while [ $SECONDS -lt $end ]; do
        echo "=== $(date +%T.%N | cut -c1-12)"
        rocm-smi --showpower --showtemp --showclocks --showuse --showmemuse --csv 2>&1
        sleep 1
    done
} > "$out" 2>&1
