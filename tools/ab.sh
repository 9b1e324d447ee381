# Alternating A/B bench lines (no CPU baseline, no vector-free line) for environment variants.
# usage: bash tools/ab.sh "<sizes>" "name:VAR=v VAR2=w" "name2:VAR=u" ...   (2 rounds each)
# e.g.   bash tools/ab.sh "2.5e6 1e8" "seq:LBFGS_COLLECT=0" "collect:LBFGS_COLLECT=1"
# AB_ARGS: extra bench.py arguments (e.g. AB_ARGS=--vector-free to A/B the vector-free mode)
set -o pipefail
mkdir -p gpurun_out
sizes=$1; shift
for n in $sizes; do
    steps=50; case $n in *e5|*e6|1e7|2e7|3e7) steps=300 ;; esac
    for r in 1 2; do
        for v in "$@"; do
            name=${v%%:*}; envs=${v#*:}
            out="gpurun_out/ab_n${n}_${name}_$r"
            env $envs timeout -k 10 300 python bench.py --size "$n" --steps $steps --warmup 20 --no-cpu-baseline \
                --no-vector-free --no-box-probe $AB_ARGS > "$out.json" 2> "$out.err" || { tail -5 "$out.err"; exit 1; }
            python -c "import json;d=json.load(open('$out.json'));r=d['roofline'] or {};print('n=$n $name $r', d['value'], d['ms_per_step'], d['achieved_hbm_gbps'], r.get('kernel'), r.get('avg_launch_us'), r.get('achieved'))"
        done
    done
done
