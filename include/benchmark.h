/* benchmark.h — drop-in for the objective surface of sequential-implementation/benchmark.h:12-16
 * and main.cpp:7-21 (= parallel-implementation/functions.h:6-12).
 *
 * These are ordinary host functions with the reference's exact formulas, so user code that
 * calls them directly gets the reference's values. When they are passed to LBFGS() /
 * LBFGS_CUDA() (lbfgs.h) the shim recognises them and evaluates the objective on the GPU
 * (LBFGS_OBJ_ROSENBROCK / _QUAD_TRIDIAG / _QUAD_SEPARABLE); any other callable runs through
 * the host-callback path (LBFGS_OBJ_HOST). */
#ifndef LBFGS_AMD_BENCHMARK_H
#define LBFGS_AMD_BENCHMARK_H
#include <functional>
#include <string>
#include <vector>

#include "lbfgs.h"
#include "vector_utils.h"

using namespace std;  // as the reference header (benchmark.h:10); main.cpp relies on it

namespace lbfgs_amd {
/* named callables so that LBFGS() can identify generate_quadratic_*(n) through std::function */
struct QuadTridiagF {
    int n;
    double operator()(const std::vector<double>& x) const;
};
struct QuadTridiagG {
    int n;
    std::vector<double> operator()(const std::vector<double>& x) const;
};
}  // namespace lbfgs_amd

std::function<double(const std::vector<double>&)> generate_quadratic_function(int n);
std::function<std::vector<double>(const std::vector<double>&)> generate_quadratic_gradient(int n);

double rosenbrock(const std::vector<double>& X);
std::vector<double> rosenbrock_grad(const std::vector<double>& X);

double quadratic(const std::vector<double>& X);
std::vector<double> quadratic_grad(const std::vector<double>& X);

#endif
