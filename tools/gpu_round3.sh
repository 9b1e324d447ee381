set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 ./tools/bwprobe 10000000 20 > gpurun_out/bwprobe_1e7.txt 2>&1; echo "probe rc=$?"; cat gpurun_out/bwprobe_1e7.txt
timeout -k 10 180 ./tools/bwprobe 100000000 10 > gpurun_out/bwprobe_1e8.txt 2>&1; echo "probe rc=$?"; grep -E "segS|seg_nt2 p0|read1|copy" gpurun_out/bwprobe_1e8.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_n1e8.json 2>gpurun_out/bench.err || exit 3
cat gpurun_out/bench_n1e8.json
timeout -k 10 300 python bench.py --no-cpu-baseline --size 1e7 > gpurun_out/bench_n1e7.json 2>>gpurun_out/bench.err || exit 3
cat gpurun_out/bench_n1e7.json
