#!/bin/bash
# build cuda-lbfgs_amd/liblbfgs_hip_<name>.so with extra -D flags on the device layer (A/B runs;
# select with LBFGS_LIB=<path>). usage: tools/build_variant.sh <name> "-DFOO=1 ..."
# The device layer is three translation units over lbfgs_kernels_impl.h; all three take the flags.
set -e
cd "$(dirname "$0")/../cuda-lbfgs_amd"
make -s csrc/lbfgs_cxx.o csrc/lbfgs_xgmi.o
make -s -B csrc/lbfgs_driver_var.o VARIANT="$1"  # provenance: src=<hash>+<name>
for tu in lbfgs_kernels lbfgs_kernels_commit lbfgs_kernels_vf; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-result \
      -Wno-unused-function -I../include -Icsrc $2 -c csrc/$tu.hip -o csrc/${tu}_$1.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o liblbfgs_hip_$1.so csrc/lbfgs_kernels_$1.o \
    csrc/lbfgs_kernels_commit_$1.o csrc/lbfgs_kernels_vf_$1.o csrc/lbfgs_xgmi.o csrc/lbfgs_driver_var.o \
    csrc/lbfgs_cxx.o -L/opt/rocm/lib -lrccl -lamdhip64 -lrocprofiler-sdk-roctx -ldl -Wl,-rpath,/opt/rocm/lib
