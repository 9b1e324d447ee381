set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_vector_free.py -x -q > gpurun_out/pytest_vf.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_vf.log; exit 1; }
tail -2 gpurun_out/pytest_vf.log
bash tools/gpu_ab_vf.sh default
VF_N=1e7 bash tools/gpu_ab_vf.sh default
