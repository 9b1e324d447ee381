# the 2-7 % between k_axpy_dot and the box probe of its stream: the pass's
# time under each stage-2 form - collect (the default at n = 1e8: the group's collector polls the
# other workgroups' flagged words inside the launch), a reduce kernel after the launch
# (LBFGS_COLLECT=0) and tickets (LBFGS_TICKET=1) - beside the probe, alternating, 2 rounds
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/gap
( while sleep 60; do echo "running $(date +%T)"; done ) & hb=$!
trap 'kill $hb 2> /dev/null' EXIT
for r in 1 2; do
  for v in "collect:LBFGS_COLLECT=1" "reduce:LBFGS_COLLECT=0" "ticket:LBFGS_TICKET=1"; do
    name=${v%%:*}; envs=${v#*:}
    out=gpurun_out/gap/${name}_$r
    env $envs timeout -k 10 300 python bench.py --steps 50 --warmup 20 --no-cpu-baseline --no-vector-free > $out.json 2> $out.err || exit 1
    python -c "import json;d=json.load(open('$out.json'));k=d['roofline']['kernel_rates'];p=d['box_probe'];print('$name $r', d['value'], 'axpy_dot', k['axpy_dot']['avg_launch_us'], 'axpy2', k['axpy2_dot']['avg_launch_us'], 'probe', p['avg_launch_us'], 'busy', d['kernel_busy']['share'])" | tee -a gpurun_out/gap/summary.txt
  done
done
