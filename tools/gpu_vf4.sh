set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_vector_free.py -x -q > gpurun_out/pytest_vf.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_vf.log; exit 1; }
tail -1 gpurun_out/pytest_vf.log
for n in 1e8 1e7 3e6 1e6; do VF_N=$n bash tools/gpu_ab_vf.sh default || exit 3; done
