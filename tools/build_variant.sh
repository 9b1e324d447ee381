#!/bin/bash
# build cuda-lbfgs_amd/liblbfgs_hip_<name>.so with extra -D flags on the device layer (A/B runs;
# select with LBFGS_LIB=<path>). usage: tools/build_variant.sh <name> "-DFOO=1 ..."
set -e
cd "$(dirname "$0")/../cuda-lbfgs_amd"
make -s csrc/lbfgs_driver.o csrc/lbfgs_cxx.o csrc/lbfgs_xgmi.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-result \
    -I../include -Icsrc $2 -c csrc/lbfgs_kernels.hip -o csrc/lbfgs_kernels_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o liblbfgs_hip_$1.so csrc/lbfgs_kernels_$1.o csrc/lbfgs_xgmi.o csrc/lbfgs_driver.o \
    csrc/lbfgs_cxx.o -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
