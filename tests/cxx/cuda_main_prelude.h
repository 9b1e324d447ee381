// The CUDA path's caller as an integrator would keep it: the reference's .cu files hold their
// own main() (parallel-implementation/L-BFGS.cu:384 and the four variants) next to the
// LBFGS_CUDA definition, its CUDA kernels and cuBLAS calls. The Makefile's `cuda` target builds
// one translation unit per file: this prelude (the includes of L-BFGS.cu:3-13 without
// cuda_runtime.h / cublas_v2.h, plus lbfgs.h for the LBFGS_CUDA declaration the removed
// definition provided) followed by that file's main() taken unchanged from where it lies under
// /root/reference (never copied into the repo), linked against liblbfgs_hip.so.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <functional>
#include <iostream>
#include <random>
#include <vector>

#include "constants.h"
#include "line_search.h"
#include "functions.h"
#include "vector_utils.h"
#include "lbfgs.h"
