# vector-free history in paired rows (LBK_VF_PAIRED, variant build liblbfgs_hip_vfpair.so; VERDICT
# r04 item 4): the vector-free GPU tests on the variant, then bench lines alternating default /
# variant (vector-free mode at n = 1e8, and the default mode to show it is unchanged)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05d
V=$PWD/cuda-lbfgs_amd/liblbfgs_hip_vfpair.so
B="python -u bench.py --no-cpu-baseline --steps 30 --warmup 5"
LBFGS_LIB=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vector_free.py tests/test_gpu_vf_geometry.py > gpurun_out/r05d/pytest_vfpair.log 2>&1 &&
timeout -k 10 300 $B --vector-free > gpurun_out/r05d/vf_sep_1.json 2> gpurun_out/r05d/vf_sep_1.err &&
LBFGS_LIB=$V timeout -k 10 300 $B --vector-free > gpurun_out/r05d/vf_pair_1.json 2> gpurun_out/r05d/vf_pair_1.err &&
timeout -k 10 300 $B --vector-free > gpurun_out/r05d/vf_sep_2.json 2> gpurun_out/r05d/vf_sep_2.err &&
LBFGS_LIB=$V timeout -k 10 300 $B --vector-free > gpurun_out/r05d/vf_pair_2.json 2> gpurun_out/r05d/vf_pair_2.err &&
timeout -k 10 300 $B --no-vector-free > gpurun_out/r05d/def_sep.json 2> gpurun_out/r05d/def_sep.err &&
LBFGS_LIB=$V timeout -k 10 300 $B --no-vector-free > gpurun_out/r05d/def_pair.json 2> gpurun_out/r05d/def_pair.err
