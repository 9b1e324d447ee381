// A caller written the way the reference's own main.cpp / benchmark.cpp call the library
// (unqualified vector<> via the headers' `using namespace std`, std::function objectives,
// the reference header names), compiled against include/ and linked with liblbfgs_hip.so.
// Prints "KEY value" lines (doubles as %a) for tests/test_cxx_dropin.py.
#include <config.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <stdexcept>

#include <benchmark.h>
#include <lbfgs.h>
#include <line_search.h>
#include <vector_utils.h>

static void put(const char* k, double v) { std::printf("KEY %s %a\n", k, v); }
static void put_x(const char* k, const vector<double>& x) {
    uint64_t a = 0, b = 0;
    for (size_t i = 0; i < x.size(); ++i) {
        uint64_t u;
        std::memcpy(&u, &x[i], 8);
        a += u;
        b += (uint64_t)(i + 1) * u;
    }
    std::printf("KEY %s %llu %llu\n", k, (unsigned long long)a, (unsigned long long)b);
}

int main() {
    const int n = 2000;
    std::mt19937 gen(42);
    std::uniform_real_distribution<> dis(-2, 2);
    vector<double> x0(n);
    for (double& v : x0) v = dis(gen);

    // 1. benchmark objective -> device objective
    vector<double> x = LBFGS(rosenbrock, rosenbrock_grad, x0, "backtracking", 30, 5, 1e-5, false);
    put_x("x_device", x);
    // 2. a user lambda -> host-callback objective (same formulas)
    auto f = [](vector<double> X) { return rosenbrock(X); };
    auto g = [](vector<double> X) { return rosenbrock_grad(X); };
    vector<double> xh = LBFGS(f, g, x0, "backtracking", 30, 5, 1e-5, false);
    put("xh_minus_x_max", [&] { double m = 0; for (int i = 0; i < n; ++i) m = std::max(m, std::fabs(xh[i] - x[i])); return m; }());
    // 3. generate_quadratic_* -> device tridiagonal quadratic, Wolfe, to convergence
    auto qf = generate_quadratic_function(n);
    auto qg = generate_quadratic_gradient(n);
    vector<double> xq = LBFGS(qf, qg, x0, "wolfe", 1000, 20, 1e-5, false);
    put_x("x_qtri", xq);
    // 4. vector_utils
    put("dot", dotProduct(x0, x0));
    put("norm", vectorNorm(x0));
    put_x("add", add(x0, x0));
    put_x("scal", scalarProduct(0.37, x0));
    put_x("neg", negative(x0));
    try {
        dotProduct(x0, vector<double>(3));
    } catch (const logic_error& e) {
        std::printf("KEY size_error %s\n", e.what());
    }
    // 5. line searches at x0 along -grad
    vector<double> g0 = rosenbrock_grad(x0);
    vector<double> d = negative(g0);
    put("ls_backtracking", backtrackingLineSearch(x0, d, rosenbrock, g0));
    put("ls_interpolation", armijoInterpolationLineSearch(x0, d, rosenbrock, g0));
    put("ls_wolfe", wolfeInterpolationLineSearch(x0, d, rosenbrock, rosenbrock_grad, g0));
    put("ls_backtracking_wolfe", backtrackingWolfeLineSearch(x0, d, rosenbrock, rosenbrock_grad, g0));
    put("cubic", cubicInterpolate(0.0, 1.0, 2.0, -1.0, 1.5, 0.5));
    // 6. unknown method -> invalid_argument (lbfgs.cpp:69)
    try {
        LBFGS(rosenbrock, rosenbrock_grad, x0, "bogus");
    } catch (const invalid_argument& e) {
        std::printf("KEY bad_method %s\n", e.what());
    }
    // 7. LBFGS_CUDA surface (constants.h profile), both overloads
    put_x("x_cuda", LBFGS_CUDA(rosenbrock, rosenbrock_grad, x0, "wolfe", 20, 5, 1e-5));
    put_x("x_cuda_bt", LBFGS_CUDA(rosenbrock, rosenbrock_grad, x0, 20, 5, 1e-5));
    std::printf("KEY C2 %a\n", C2);
    // 8. dense quadratic (matrices.h form x'Ax + b'x) -> device dense objective
    {
        const int nd = 300;
        vector<double> A((size_t)nd * nd), bv(nd), xd0(nd);
        std::mt19937 gd(7);
        std::uniform_real_distribution<> u(-1, 1);
        for (int i = 0; i < nd; ++i)
            for (int j = 0; j <= i; ++j) A[(size_t)i * nd + j] = A[(size_t)j * nd + i] = u(gd) / nd + (i == j ? 1.0 : 0.0);
        for (double& v : bv) v = u(gd);
        for (double& v : xd0) v = 2 * u(gd);
        auto df = lbfgs_amd::dense_quadratic_function(A, bv);
        auto dg = lbfgs_amd::dense_quadratic_gradient(A, bv);
        vector<double> xd = LBFGS(df, dg, xd0, "backtracking", 5000, 5, 1e-6, false);
        std::printf("KEY dense_objective %d\n", lbfgs_amd::last_objective());
        put("dense_gnorm", vectorNorm(dg(xd)));
        put_x("dense_x", xd);
    }
    return 0;
}
