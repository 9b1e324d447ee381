set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_vector_free.py -x -q > gpurun_out/pytest_vf.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_vf.log; exit 1; }
tail -2 gpurun_out/pytest_vf.log
for n in 1e8 1e7 1e6; do VF_N=$n bash tools/gpu_ab_vf.sh default || exit 3; done
timeout -k 10 300 python bench.py --size 1e6 --steps 500 --no-cpu-baseline --no-vector-free > gpurun_out/b1e6.json && python -c "import json;d=json.load(open('gpurun_out/b1e6.json'));print('default 1e6', d['value'])"
