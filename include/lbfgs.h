/* lbfgs.h — C++ drop-in for the reference's L-BFGS entry points, same signatures:
 *   LBFGS(...)       sequential-implementation/lbfgs.h:17-25 (defaults as in the header)
 *   LBFGS_CUDA(...)  parallel-implementation/L-BFGS.cu:105-112 (with method string) and the
 *                    string-less form of the four variants, e.g. L-BFGS-Backtracking.cu:139-145
 * implemented on the GPU through the C ABI in lbfgs_hip.h (no CPU fallback).
 *
 * Behaviour as in the reference: an unknown line-search name throws std::invalid_argument
 * ("Unknown line search method: <name>", lbfgs.cpp:69); the status messages ("Converged!",
 * "Maximum iterations reached", warnings) go to stdout; non-convergence returns the current x.
 * A HIP/RCCL failure throws std::runtime_error (the reference exit()s, L-BFGS.cu:76-92).
 * Objectives from benchmark.h are evaluated on the GPU; other callables are called on the host
 * with the trial points. Device selection: env LBFGS_DEVICE (default 0). */
#ifndef LBFGS_AMD_LBFGS_H
#define LBFGS_AMD_LBFGS_H
#include <functional>
#include <memory>
#include <string>
#include <vector>

std::vector<double> LBFGS(const std::function<double(std::vector<double>)> f,
                          const std::function<std::vector<double>(std::vector<double>)> grad,
                          const std::vector<double> x0, const std::string line_search_method,
                          const int max_iterations = 1000, const int m = 10,
                          const double tolerance = 1e-5, bool verbose = false);

std::vector<double> LBFGS_CUDA(const std::function<double(std::vector<double>)> f,
                               const std::function<std::vector<double>(std::vector<double>)> grad,
                               const std::vector<double> x0, const std::string line_search_method,
                               const int max_iterations, const int m, const double tolerance);

/* the variants' form without a method string (L-BFGS-Backtracking.cu:139-145, and the same
 * signature in L-BFGS-Interpolation.cu:105, L-BFGS-Wolfe.cu:105, L-BFGS-Backtracking_Wolfe.cu:106).
 * In the reference the line search is fixed by which .cu file was compiled (run.sh $1); here the
 * caller names its variant at compile time, -DLBFGS_CUDA_VARIANT='"wolfe"' (or "backtracking",
 * "interpolation", "backtracking_wolfe"), or at run time with the environment variable
 * LBFGS_CUDA_VARIANT; with neither it is "backtracking" (L-BFGS-Backtracking.cu). An unknown name
 * throws std::invalid_argument as the string form does. */
namespace lbfgs_amd {
/* the string-less LBFGS_CUDA of the variant file `variant` names: the string form's solve, or with
 * the environment variable LBFGS_CUDA_COMPAT=1 that file's own loop and inline line search
 * (LBFGS_FLAG_CUDA_COMPAT | LBFGS_FLAG_CUDA_VARIANT, lbfgs_hip.h) */
std::vector<double> cuda_variant(const std::function<double(std::vector<double>)>& f,
                                 const std::function<std::vector<double>(std::vector<double>)>& grad,
                                 const std::vector<double>& x0, const std::string& variant, int max_iterations,
                                 int m, double tolerance);
}  // namespace lbfgs_amd

#ifdef LBFGS_CUDA_VARIANT
static inline std::vector<double> LBFGS_CUDA(const std::function<double(std::vector<double>)> f,
                                             const std::function<std::vector<double>(std::vector<double>)> grad,
                                             const std::vector<double> x0, const int max_iterations, const int m,
                                             const double tolerance) {
    return lbfgs_amd::cuda_variant(f, grad, x0, std::string(LBFGS_CUDA_VARIANT), max_iterations, m, tolerance);
}
#else
std::vector<double> LBFGS_CUDA(const std::function<double(std::vector<double>)> f,
                               const std::function<std::vector<double>(std::vector<double>)> grad,
                               const std::vector<double> x0, const int max_iterations, const int m,
                               const double tolerance);
#endif

namespace lbfgs_amd {
/* which objective path the calling thread's last LBFGS / LBFGS_CUDA call took: 0 Rosenbrock,
 * 1 tridiagonal quadratic, 2 separable quadratic (device kernels), 3 host callbacks, 4 dense
 * quadratic (device) (LBFGS_OBJ_* of lbfgs_hip.h); -1 before the first call. Diagnostic. */
int last_objective();

/* Dense quadratic f(x) = x'Ax + b'x, grad = 2Ax + b (A symmetric, n x n row-major): the problems
 * of the reference's sequential-implementation/matrices.h (mat<n>, linear<n>). Passed to LBFGS()
 * as a pair, they are recognised and evaluated on the device (LBFGS_OBJ_DENSE_QUAD); called
 * directly they compute the same values on the host. */
struct DenseQuadF {
    std::shared_ptr<const std::vector<double>> A, b;
    double operator()(const std::vector<double>& x) const;
};
struct DenseQuadG {
    std::shared_ptr<const std::vector<double>> A, b;
    std::vector<double> operator()(const std::vector<double>& x) const;
};
std::function<double(const std::vector<double>&)> dense_quadratic_function(const std::vector<double>& A,
                                                                           const std::vector<double>& b);
std::function<std::vector<double>(const std::vector<double>&)> dense_quadratic_gradient(
    const std::vector<double>& A, const std::vector<double>& b);
}  // namespace lbfgs_amd

#endif
