/* benchmark.h — drop-in for sequential-implementation/benchmark.h:12-26 (the objectives and the
 * benchmark() timing harness that the reference's main.cpp:45-53 calls) and the separable
 * quadratic of main.cpp:7-21 (= parallel-implementation/functions.h:6-12).
 *
 * These are ordinary host functions with the reference's exact formulas, so user code that
 * calls them directly gets the reference's values. When they are passed to LBFGS() /
 * LBFGS_CUDA() (lbfgs.h) the shim recognises them and evaluates the objective on the GPU
 * (LBFGS_OBJ_ROSENBROCK / _QUAD_TRIDIAG / _QUAD_SEPARABLE); any other callable runs through
 * the host-callback path (LBFGS_OBJ_HOST). */
#ifndef LBFGS_AMD_BENCHMARK_H
#define LBFGS_AMD_BENCHMARK_H
#include <chrono>
#include <functional>
#include <iostream>
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

/* a caller may define its own quadratic / quadratic_grad (the reference's main.cpp:7-21 does);
 * those are the caller's functions and run through the host-callback path */
double quadratic(const std::vector<double>& X);
std::vector<double> quadratic_grad(const std::vector<double>& X);

/* benchmark.h:19-26 / benchmark.cpp:83-105: times LBFGS(f, grad, x0, "backtracking",
 * max_iterations, m, tolerance, false) and prints
 *   Function: <name> / Optimum value: <f(optimum)> / Elapsed time: <s> seconds / a rule,
 * returning the elapsed seconds. */
double benchmark(const std::string function_name, const std::function<double(std::vector<double>)> f,
                 const std::function<std::vector<double>(std::vector<double>)> grad,
                 const std::vector<double> x0, const int max_iterations, const int m, const double tolerance);

#endif
