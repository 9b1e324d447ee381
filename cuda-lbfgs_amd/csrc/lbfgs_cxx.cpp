// lbfgs_cxx.cpp — C++ drop-in layer (include/lbfgs.h, include/benchmark.h) over the C ABI.
//
// LBFGS()/LBFGS_CUDA() keep the reference signatures (sequential-implementation/lbfgs.h:17-25,
// parallel-implementation/L-BFGS.cu:105-112) and run on the GPU. The benchmark objectives are
// recognised through std::function::target and evaluated by the device kernels; any other
// callable is driven through the host-callback objective.
#include <cstdint>
#include <cstdlib>
#include <limits>
#include <algorithm>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "benchmark.h"
#include "lbfgs.h"
#include "lbfgs_hip.h"

using std::vector;

// ---- benchmark objectives: the reference formulas, host-side (benchmark.cpp:16-81) ----------
namespace lbfgs_amd {
double QuadTridiagF::operator()(const vector<double>& x) const {
    double result = 0.0;
    for (int i = 0; i < n; i++) result += 1000.0 * x[i] * x[i];
    for (int i = 0; i < n - 1; i++) result += (1000.0 / 10.0) * x[i] * x[i + 1];
    return result;
}
vector<double> QuadTridiagG::operator()(const vector<double>& x) const {
    vector<double> g(n, 0.0);
    for (int i = 0; i < n; i++) g[i] = 2.0 * 1000.0 * x[i];
    for (int i = 0; i < n - 1; i++) {
        g[i] += (1000.0 / 10.0) * x[i + 1];
        g[i + 1] += (1000.0 / 10.0) * x[i];
    }
    return g;
}
}  // namespace lbfgs_amd

std::function<double(const vector<double>&)> generate_quadratic_function(int n) {
    return lbfgs_amd::QuadTridiagF{n};
}
std::function<vector<double>(const vector<double>&)> generate_quadratic_gradient(int n) {
    return lbfgs_amd::QuadTridiagG{n};
}

double rosenbrock(const vector<double>& X) {
    double sum = 0.0;
    for (size_t i = 0; i + 1 < X.size(); i++) {
        double term1 = X[i + 1] - X[i] * X[i];
        double term2 = 1 - X[i];
        sum += 100.0 * term1 * term1 + term2 * term2;
    }
    return sum;
}

vector<double> rosenbrock_grad(const vector<double>& X) {
    vector<double> grad(X.size(), 0.0);
    for (size_t i = 0; i + 1 < X.size(); i++) {
        double term1 = 2.0 * (X[i] - 1);
        double term2 = X[i + 1] - X[i] * X[i];
        grad[i] += term1 - 400.0 * X[i] * term2;
        grad[i + 1] += 200.0 * term2;
    }
    return grad;
}

double quadratic(const vector<double>& X) {
    double sum = 0.0;
    for (const double x : X) sum += (x - 1) * (x - 1);
    return sum;
}

vector<double> quadratic_grad(const vector<double>& X) {
    vector<double> g(X.size());
    for (size_t i = 0; i < X.size(); i++) g[i] = 2.0 * (X[i] - 1);
    return g;
}

// ---- LBFGS / LBFGS_CUDA ------------------------------------------------------------------
namespace {

using FnF = std::function<double(vector<double>)>;
using FnG = std::function<vector<double>(vector<double>)>;
using FnFc = std::function<double(const vector<double>&)>;
using FnGc = std::function<vector<double>(const vector<double>&)>;
typedef double (*PlainF)(const vector<double>&);
typedef vector<double> (*PlainG)(const vector<double>&);

int identify(const FnF& f, const FnG& g, int n) {
    const PlainF* pf = f.target<PlainF>();
    const PlainG* pg = g.target<PlainG>();
    if (pf && pg) {
        if (*pf == &rosenbrock && *pg == &rosenbrock_grad) return LBFGS_OBJ_ROSENBROCK;
        if (*pf == &quadratic && *pg == &quadratic_grad) return LBFGS_OBJ_QUAD_SEPARABLE;
    }
    const FnFc* wf = f.target<FnFc>();
    const FnGc* wg = g.target<FnGc>();
    const lbfgs_amd::QuadTridiagF* qf = wf ? wf->target<lbfgs_amd::QuadTridiagF>() : f.target<lbfgs_amd::QuadTridiagF>();
    const lbfgs_amd::QuadTridiagG* qg = wg ? wg->target<lbfgs_amd::QuadTridiagG>() : g.target<lbfgs_amd::QuadTridiagG>();
    if (qf && qg && qf->n == n && qg->n == n) return LBFGS_OBJ_QUAD_TRIDIAG;
    return LBFGS_OBJ_HOST;
}

int line_search_id(const std::string& s) {  // lbfgs.cpp:40-70
    if (s == "backtracking") return LBFGS_LS_BACKTRACKING;
    if (s == "interpolation") return LBFGS_LS_INTERPOLATION;
    if (s == "wolfe") return LBFGS_LS_WOLFE;
    if (s == "backtracking_wolfe") return LBFGS_LS_BACKTRACKING_WOLFE;
    throw std::invalid_argument("Unknown line search method: " + s);
}

struct HostFns {
    const FnF* f;
    const FnG* g;
    std::string error;
};

double host_f(const double* x, int64_t n, void* user) {
    HostFns* h = static_cast<HostFns*>(user);
    try {
        return (*h->f)(vector<double>(x, x + n));
    } catch (const std::exception& e) {
        h->error = e.what();
        return std::numeric_limits<double>::quiet_NaN();
    }
}

void host_g(const double* x, int64_t n, double* out, void* user) {
    HostFns* h = static_cast<HostFns*>(user);
    try {
        vector<double> g = (*h->g)(vector<double>(x, x + n));
        if ((int64_t)g.size() != n) throw std::logic_error("Vectors must be of same size");
        std::copy(g.begin(), g.end(), out);
    } catch (const std::exception& e) {
        h->error = e.what();
        std::fill(out, out + n, std::numeric_limits<double>::quiet_NaN());
    }
}

struct CtxDeleter {
    void operator()(lbfgs_ctx* c) const { lbfgs_ctx_destroy(c); }
};

// one cached context per thread, re-created when (n, m) change: device memory is allocated
// once per problem shape instead of per call (L-BFGS.cu:155-172 allocates per call)
lbfgs_ctx* context_for(int64_t n, int m) {
    thread_local std::unique_ptr<lbfgs_ctx, CtxDeleter> ctx;
    thread_local int64_t cn = -1;
    thread_local int cm = -1;
    if (!ctx || cn != n || cm != m) {
        ctx.reset();
        const char* dev = std::getenv("LBFGS_DEVICE");
        lbfgs_ctx* c = nullptr;
        int rc = lbfgs_ctx_create(&c, n, m, dev ? std::atoi(dev) : 0);
        if (rc != 0) throw std::runtime_error("lbfgs_ctx_create failed (" + std::to_string(rc) + ")");
        ctx.reset(c);
        cn = n;
        cm = m;
    }
    return ctx.get();
}

vector<double> run(const FnF& f, const FnG& grad, const vector<double>& x0, int ls, int max_iterations,
                   int m, double tolerance, bool verbose, const lbfgs_constants& k) {
    const int64_t n = (int64_t)x0.size();
    if (n < 1) throw std::invalid_argument("x0 must not be empty");
    const int obj = identify(f, grad, (int)n);
    lbfgs_ctx* c = context_for(n, m);
    HostFns hf{&f, &grad, {}};
    lbfgs_host_fn cb{host_f, host_g, &hf};
    vector<double> x(n);
    lbfgs_result res;
    int rc = lbfgs_minimize(c, obj, obj == LBFGS_OBJ_HOST ? &cb : nullptr, ls, &k, x0.data(), x.data(),
                            max_iterations, tolerance, verbose ? LBFGS_FLAG_VERBOSE : 0u, &res);
    if (!hf.error.empty()) throw std::runtime_error("objective callback failed: " + hf.error);
    if (rc < 0) throw std::runtime_error(std::string("LBFGS failed: ") + lbfgs_last_error(c));
    return x;
}

}  // namespace

vector<double> LBFGS(const FnF f, const FnG grad, const vector<double> x0, const std::string line_search_method,
                     const int max_iterations, const int m, const double tolerance, bool verbose) {
    const int ls = line_search_id(line_search_method);
    lbfgs_constants k;
    lbfgs_constants_default(&k);
    return run(f, grad, x0, ls, max_iterations, m, tolerance, verbose, k);
}

vector<double> LBFGS_CUDA(const FnF f, const FnG grad, const vector<double> x0, const std::string line_search_method,
                          const int max_iterations, const int m, const double tolerance) {
    const int ls = line_search_id(line_search_method);
    lbfgs_constants k;
    lbfgs_constants_cuda(&k);  // parallel-implementation/constants.h (C2 = 0.7)
    return run(f, grad, x0, ls, max_iterations, m, tolerance, false, k);
}

vector<double> LBFGS_CUDA(const FnF f, const FnG grad, const vector<double> x0, const int max_iterations,
                          const int m, const double tolerance) {
    return LBFGS_CUDA(f, grad, x0, std::string("backtracking"), max_iterations, m, tolerance);
}
