// san_main.cpp — sanitizer job (tests/sanitize/Makefile, run by tests/test_sanitize.py).
//
// The C driver (lbfgs_driver.c) and the C++ drop-in shim (lbfgs_cxx.cpp) built with
// -fsanitize=address,undefined on the CPU, over the host test double of the device layer
// (host_device_double.c, canonical-order reductions from the oracle). Every solve must
// reproduce the oracle's ORC_CANON trajectory bit for bit (f, |g|, alpha, x checksums, final x,
// messages, status) - so the host logic is exercised on the same paths the GPU runs - and the
// sanitizers must stay silent (any report aborts the process: -fno-sanitize-recover=all).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "benchmark.h"
#include "lbfgs.h"
#include "lbfgs_hip.h"
#include "lbfgs_oracle.h"
#include "vector_utils.h"

static int g_fail = 0;
#define EXPECT(cond, ...)                                    \
    do {                                                     \
        if (!(cond)) {                                       \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);               \
            std::fprintf(stderr, "\n");                      \
            ++g_fail;                                        \
        }                                                    \
    } while (0)

static bool same_bits(double a, double b) { return std::memcmp(&a, &b, 8) == 0 || (std::isnan(a) && std::isnan(b)); }

struct OracleRun {
    std::vector<double> x, f, gn, al;
    std::vector<uint64_t> c1, c2;
    std::string msg;
    orc_result res;
    int64_t nf = 0, ng = 0;
};

static OracleRun oracle(int obj, int ls, int64_t n, int m, int maxit, const std::vector<double>& x0,
                        double (*hf)(const double*, int64_t, void*) = nullptr,
                        void (*hg)(const double*, int64_t, double*, void*) = nullptr, void* user = nullptr,
                        int cuda = 0, double tol = 1e-5) {
    orc_opts o;
    std::memset(&o, 0, sizeof o);
    o.obj = obj;
    o.ls = ls;
    o.mode = ORC_CANON;
    o.n = n;
    o.m = m;
    o.maxit = maxit;
    o.tol = tol;
    o.c1 = 1e-4;
    o.c2 = cuda ? 0.7 : 0.9; /* parallel-implementation/constants.h for the CUDA paths */
    o.cuda = cuda;
    o.initial_step = 1.0;
    o.backtracking_alpha = 0.5;
    o.backtracking_tol = 1e-8;
    o.wolfe_interp_min = 1e-10;
    o.host_f = hf;
    o.host_g = hg;
    o.host_user = user;
    OracleRun r;
    const int cap = maxit + 2;
    r.x.resize(n);
    r.f.resize(cap);
    r.gn.resize(cap);
    r.al.resize(cap);
    r.c1.resize(cap);
    r.c2.resize(cap);
    std::vector<int64_t> nf(cap);
    std::vector<char> msg(1 << 20);
    int64_t fn = 0, gnn = 0;
    orc_lbfgs(&o, x0.data(), r.x.data(), r.f.data(), r.gn.data(), r.al.data(), r.c1.data(), r.c2.data(), nf.data(),
              cap, nullptr, 0, &fn, nullptr, 0, &gnn, msg.data(), (int)msg.size(), &r.res);
    r.msg = msg.data();
    r.f.resize(r.res.ntrace);
    r.nf = r.res.nf;
    r.ng = r.res.ng;
    return r;
}

static void compare(const char* tag, lbfgs_ctx* c, int status, const std::vector<double>& x, const lbfgs_result& res,
                    const OracleRun& o) {
    const int len = lbfgs_trace_len(c);
    EXPECT(len == o.res.ntrace, "%s: trace length %d vs %d", tag, len, o.res.ntrace);
    std::vector<double> f(len), gn(len), al(len);
    std::vector<uint64_t> c1(len), c2(len);
    lbfgs_trace_get(c, f.data(), gn.data(), al.data(), c1.data(), c2.data(), len);
    for (int k = 0; k < len && k < o.res.ntrace; ++k) {
        EXPECT(same_bits(f[k], o.f[k]) && same_bits(gn[k], o.gn[k]), "%s: iteration %d f %.17g/%.17g", tag, k, f[k],
               o.f[k]);
        EXPECT(same_bits(al[k], o.al[k]), "%s: iteration %d alpha %.17g/%.17g", tag, k, al[k], o.al[k]);
        EXPECT(c1[k] == o.c1[k] && c2[k] == o.c2[k], "%s: iteration %d x checksum", tag, k);
    }
    for (size_t i = 0; i < x.size(); ++i)
        if (!same_bits(x[i], o.x[i])) {
            EXPECT(false, "%s: x[%zu] %.17g vs %.17g", tag, i, x[i], o.x[i]);
            break;
        }
    std::vector<char> msg(1 << 20);
    lbfgs_messages(c, msg.data(), (int)msg.size());
    EXPECT(o.msg == msg.data(), "%s: messages differ", tag);
    EXPECT(status == o.res.status && res.iterations == o.res.iters, "%s: status %d/%d iterations %d/%d", tag, status,
           o.res.status, res.iterations, o.res.iters);
}

static std::vector<double> x0_for(int64_t n, uint32_t seed) {
    std::vector<double> x(n);
    orc_x0_uniform(x.data(), n, seed, -2.0, 2.0);
    return x;
}

// device objectives, every line search, default / batched-off / unfused / the small-n single
// launch per iteration with and without the speculative next iteration / the persistent two-loop
static void device_objectives() {
    const int64_t sizes[] = {1, 2, 3, 1000, 4097, 70001};
    const int objs[] = {LBFGS_OBJ_ROSENBROCK, LBFGS_OBJ_QUAD_TRIDIAG, LBFGS_OBJ_QUAD_SEPARABLE};
    int64_t adopted = 0, dropped = 0, searches[4] = {0, 0, 0, 0}, search_commits = 0;
    for (int64_t n : sizes)
        for (int obj : objs)
            for (int ls = 0; ls < 4; ++ls)
                for (int mode = 0; mode < 6; ++mode) {
                    const int m = n < 10 ? 2 : 5, maxit = n > 10000 ? 12 : 40;
                    if (obj == LBFGS_OBJ_QUAD_SEPARABLE && ls == LBFGS_LS_WOLFE) continue;  // diverges to NaN
                    setenv("LBFGS_BATCH", mode == 1 ? "0" : "1", 1);
                    setenv("LBFGS_DOUBLE_SMALL", mode == 3 || mode == 4 ? "1" : "0", 1);
                    setenv("LBFGS_SPEC", mode == 4 ? "0" : "1", 1);
                    setenv("LBFGS_DOUBLE_TWOLOOP", mode == 5 ? "1" : "0", 1);
                    const auto x0 = x0_for(n, 42 + (uint32_t)n);
                    lbfgs_ctx* c = nullptr;
                    EXPECT(lbfgs_ctx_create(&c, n, m, 0) == 0, "create n=%lld", (long long)n);
                    if (!c) continue;
                    std::vector<double> x(n);
                    lbfgs_result res;
                    const unsigned flags = LBFGS_FLAG_QUIET | LBFGS_FLAG_TRACE | (mode == 2 ? LBFGS_FLAG_UNFUSED : 0u);
                    const int st = lbfgs_minimize(c, obj, nullptr, ls, nullptr, x0.data(), x.data(), maxit, 1e-5,
                                                  flags, &res);
                    EXPECT(st >= 0, "minimize n=%lld obj %d ls %d mode %d: %d %s", (long long)n, obj, ls, mode, st,
                           lbfgs_last_error(c));
                    char tag[96];
                    std::snprintf(tag, sizeof tag, "n=%lld obj=%d ls=%d mode=%d", (long long)n, obj, ls, mode);
                    if (st >= 0) compare(tag, c, st, x, res, oracle(obj, ls, n, m, maxit, x0));
                    int64_t a = 0, d = 0;
                    lbfgs_spec_stats(c, &a, &d);
                    EXPECT(mode == 3 || a + d == 0, "%s: speculative launches outside the speculative mode", tag);
                    adopted += a;
                    dropped += d;
                    int64_t sl = 0, sc = 0;  // the device-resident line search (the double's restatement)
                    lbfgs_search_stats(c, &sl, &sc);
                    EXPECT(mode == 3 || mode == 4 || sl == 0, "%s: device searches outside the small-n forms", tag);
                    EXPECT(sc <= sl, "%s: %lld device-search commits of %lld launches", tag, (long long)sc,
                           (long long)sl);
                    searches[ls] += sl;
                    search_commits += sc;
                    lbfgs_ctx_destroy(c);
                }
    EXPECT(adopted > 100 && dropped > 10, "speculative launches: %lld taken, %lld dropped", (long long)adopted,
           (long long)dropped);
    std::printf("speculative next iteration: %lld launches taken, %lld dropped\n", (long long)adopted,
                (long long)dropped);
    for (int ls = 0; ls < 4; ++ls) EXPECT(searches[ls] > 0, "line search %d never continued on the device", ls);
    EXPECT(search_commits > 0, "no device-search commit");
    std::printf("device line searches: %lld / %lld / %lld / %lld launches (backtracking / interpolation / Wolfe / "
                "backtracking-Wolfe), %lld commits in them\n", (long long)searches[0], (long long)searches[1],
                (long long)searches[2], (long long)searches[3], (long long)search_commits);
    setenv("LBFGS_BATCH", "1", 1);
    setenv("LBFGS_DOUBLE_SMALL", "0", 1);
    setenv("LBFGS_SPEC", "1", 1);
    setenv("LBFGS_DOUBLE_TWOLOOP", "0", 1);
}

// LBFGS_FLAG_CUDA_COMPAT: L-BFGS.cu's loop with line_search.cpp's searches (cuda 1) and the four
// variant files' loops with their inline searches (cuda 2), against the oracle's restatements
static void cuda_paths() {
    const int64_t sizes[] = {1, 2, 5, 1000, 4097};
    const int objs[] = {LBFGS_OBJ_ROSENBROCK, LBFGS_OBJ_QUAD_TRIDIAG, LBFGS_OBJ_QUAD_SEPARABLE};
    lbfgs_constants k;
    lbfgs_constants_cuda(&k);
    for (int64_t n : sizes)
        for (int obj : objs)
            for (int ls = 0; ls < 4; ++ls)
                for (int cuda = 1; cuda <= 2; ++cuda) {
                    const int m = n < 10 ? 2 : 5, maxit = n > 10 ? 60 : 300;
                    const double tol = 1e-10;
                    const auto x0 = x0_for(n, 7 + (uint32_t)n);
                    lbfgs_ctx* c = nullptr;
                    EXPECT(lbfgs_ctx_create(&c, n, m, 0) == 0, "create n=%lld", (long long)n);
                    if (!c) continue;
                    std::vector<double> x(n);
                    lbfgs_result res;
                    const unsigned flags = LBFGS_FLAG_QUIET | LBFGS_FLAG_TRACE | LBFGS_FLAG_CUDA_COMPAT |
                                           (cuda == 2 ? LBFGS_FLAG_CUDA_VARIANT : 0u);
                    const int st = lbfgs_minimize(c, obj, nullptr, ls, &k, x0.data(), x.data(), maxit, tol, flags, &res);
                    EXPECT(st >= 0, "cuda %d minimize n=%lld obj %d ls %d: %d %s", cuda, (long long)n, obj, ls, st,
                           lbfgs_last_error(c));
                    char tag[96];
                    std::snprintf(tag, sizeof tag, "cuda=%d n=%lld obj=%d ls=%d", cuda, (long long)n, obj, ls);
                    if (st >= 0) compare(tag, c, st, x, res, oracle(obj, ls, n, m, maxit, x0, nullptr, nullptr, nullptr, cuda, tol));
                    lbfgs_ctx_destroy(c);
                }
}

// host callbacks: the reference call sequence call for call, and one call per point by default
struct Counter {
    int obj;
    int64_t nf = 0, ng = 0;
};
static double cb_f(const double* x, int64_t n, void* u) {
    Counter* k = static_cast<Counter*>(u);
    ++k->nf;
    return orc_f(k->obj, x, n, ORC_CANON);
}
static void cb_g(const double* x, int64_t n, double* g, void* u) {
    Counter* k = static_cast<Counter*>(u);
    ++k->ng;
    orc_grad(k->obj, x, n, g);
}

static void host_callbacks() {
    for (int ls = 0; ls < 4; ++ls)
        for (int refcalls = 0; refcalls < 2; ++refcalls) {
            const int64_t n = 1500;
            const int m = 5, maxit = 30;
            const auto x0 = x0_for(n, 7);
            Counter ko{LBFGS_OBJ_ROSENBROCK}, kg{LBFGS_OBJ_ROSENBROCK};
            const OracleRun o = oracle(ORC_OBJ_HOST, ls, n, m, maxit, x0, cb_f, cb_g, &ko);
            lbfgs_ctx* c = nullptr;
            lbfgs_ctx_create(&c, n, m, 0);
            lbfgs_host_fn cb{cb_f, cb_g, &kg};
            std::vector<double> x(n);
            lbfgs_result res;
            const unsigned flags = LBFGS_FLAG_QUIET | LBFGS_FLAG_TRACE | (refcalls ? LBFGS_FLAG_REFERENCE_CALLS : 0u);
            const int st = lbfgs_minimize(c, LBFGS_OBJ_HOST, &cb, ls, nullptr, x0.data(), x.data(), maxit, 1e-5, flags,
                                          &res);
            char tag[64];
            std::snprintf(tag, sizeof tag, "host ls=%d refcalls=%d", ls, refcalls);
            EXPECT(st >= 0, "%s: %d", tag, st);
            if (st >= 0) compare(tag, c, st, x, res, o);
            EXPECT(res.f_calls == kg.nf && res.grad_calls == kg.ng, "%s: counters", tag);
            if (refcalls)
                EXPECT(kg.nf == ko.nf && kg.ng == ko.ng, "%s: calls %lld/%lld f, %lld/%lld g", tag, (long long)kg.nf,
                       (long long)ko.nf, (long long)kg.ng, (long long)ko.ng);
            else
                EXPECT(kg.nf < ko.nf && kg.ng <= ko.ng, "%s: not fewer calls", tag);
            lbfgs_ctx_destroy(c);
        }
}

// the dense quadratic objective (matrices.h form), every line search, against the oracle
static void dense_objective() {
    const int64_t n = 97;
    std::vector<double> A((size_t)(n * n)), b(n);
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t j = 0; j <= i; ++j)
            A[(size_t)(i * n + j)] = A[(size_t)(j * n + i)] = std::sin(0.37 * (double)(i * 31 + j)) / (double)n +
                                                              (i == j ? 1.5 : 0.0);
        b[(size_t)i] = std::cos(0.11 * (double)i);
    }
    orc_dense_set(A.data(), b.data());
    const auto x0 = x0_for(n, 11);
    for (int ls = 0; ls < 4; ++ls) {
        lbfgs_ctx* c = nullptr;
        lbfgs_ctx_create(&c, n, 5, 0);
        EXPECT(lbfgs_minimize(c, LBFGS_OBJ_DENSE_QUAD, nullptr, ls, nullptr, x0.data(), nullptr, 10, 1e-5, 0,
                              nullptr) == LBFGS_ERR_STATE,
               "dense without data");
        EXPECT(lbfgs_set_dense_quadratic(c, A.data(), b.data()) == 0, "set dense");
        std::vector<double> x(n);
        lbfgs_result res;
        const int st = lbfgs_minimize(c, LBFGS_OBJ_DENSE_QUAD, nullptr, ls, nullptr, x0.data(), x.data(), 200, 1e-5,
                                      LBFGS_FLAG_QUIET | LBFGS_FLAG_TRACE, &res);
        char tag[48];
        std::snprintf(tag, sizeof tag, "dense ls=%d", ls);
        EXPECT(st == LBFGS_STATUS_CONVERGED, "%s: status %d", tag, st);
        if (st >= 0) compare(tag, c, st, x, res, oracle(ORC_OBJ_DENSE, ls, n, 5, 200, x0));
        lbfgs_ctx_destroy(c);
    }
}

// stepping API, standalone line search, primitives, error paths
static void api_surface() {
    const int64_t n = 3000;
    const auto x0 = x0_for(n, 3);
    lbfgs_ctx* c = nullptr;
    EXPECT(lbfgs_ctx_create(&c, n, 4, 0) == 0, "create");
    lbfgs_result res;
    EXPECT(lbfgs_solver_init(c, LBFGS_OBJ_ROSENBROCK, nullptr, LBFGS_LS_BACKTRACKING, nullptr, x0.data(), 1e-5,
                             LBFGS_FLAG_QUIET | LBFGS_FLAG_TRACE) == 0,
           "init");
    for (int i = 0; i < 5; ++i) EXPECT(lbfgs_solver_step(c, 3, &res) == LBFGS_STATUS_RUNNING, "step");
    EXPECT(res.h_min == 4 && res.h_max == 4, "h %d..%d", res.h_min, res.h_max);
    std::vector<double> x(n), d(n), g(n);
    EXPECT(lbfgs_get_x(c, x.data()) == 0, "get_x");
    orc_grad(ORC_OBJ_ROSENBROCK, x.data(), n, g.data());
    for (int64_t i = 0; i < n; ++i) d[i] = -g[i];
    for (int ls = 0; ls < 4; ++ls) {
        double a = 0.0;
        EXPECT(lbfgs_line_search(c, LBFGS_OBJ_ROSENBROCK, nullptr, ls, nullptr, x.data(), d.data(), g.data(), &a) == 0,
               "line search %d", ls);
        EXPECT(a > 0.0, "alpha %g", a);
    }
    double dot = 0.0, nrm = 0.0;
    EXPECT(lbfgs_dev_dot(c, x.data(), g.data(), &dot) == 0 && same_bits(dot, orc_dot(x.data(), g.data(), n, ORC_CANON)),
           "dot");
    EXPECT(lbfgs_dev_norm(c, g.data(), &nrm) == 0, "norm");
    std::vector<double> out(n);
    for (int op = 0; op < 3; ++op) EXPECT(lbfgs_dev_elementwise(c, op, x.data(), g.data(), 0.5, out.data()) == 0, "ew");
    double f = 0.0, dphi = 0.0;
    EXPECT(lbfgs_dev_objective(c, LBFGS_OBJ_QUAD_TRIDIAG, x.data(), &f, out.data()) == 0, "objective");
    EXPECT(lbfgs_dev_trial(c, LBFGS_OBJ_ROSENBROCK, x.data(), d.data(), 1e-3, &f, out.data(), &dphi) == 0, "trial");
    std::vector<std::vector<double>> S(3, std::vector<double>(n)), Y(3, std::vector<double>(n));
    for (int j = 0; j < 3; ++j)
        for (int64_t i = 0; i < n; ++i) {
            S[j][i] = std::sin(0.001 * (double)(i + 17 * j));
            Y[j][i] = S[j][i] * (1.5 + 0.1 * j);
        }
    const double* Sp[3] = {S[0].data(), S[1].data(), S[2].data()};
    const double* Yp[3] = {Y[0].data(), Y[1].data(), Y[2].data()};
    double gd = 0.0;
    EXPECT(lbfgs_dev_twoloop(c, g.data(), Sp, Yp, 3, out.data(), &gd) == 0, "twoloop");
    EXPECT(same_bits(gd, orc_twoloop(g.data(), Sp, Yp, 3, n, ORC_CANON, d.data())), "twoloop g.d");
    // error paths
    EXPECT(lbfgs_minimize(c, 99, nullptr, 0, nullptr, x0.data(), x.data(), 5, 1e-5, 0, &res) == LBFGS_ERR_BAD_ARG,
           "bad objective");
    EXPECT(lbfgs_minimize(c, LBFGS_OBJ_HOST, nullptr, 0, nullptr, x0.data(), x.data(), 5, 1e-5, 0, &res) ==
               LBFGS_ERR_BAD_ARG,
           "host without callbacks");
    EXPECT(lbfgs_minimize(c, 0, nullptr, 7, nullptr, x0.data(), x.data(), 5, 1e-5, 0, &res) == LBFGS_ERR_BAD_ARG,
           "bad line search");
    lbfgs_ctx_destroy(c);
    lbfgs_ctx* bad = nullptr;
    EXPECT(lbfgs_ctx_create(&bad, 0, 4, 0) == LBFGS_ERR_BAD_ARG && !bad, "n = 0");
    EXPECT(lbfgs_ctx_create(&bad, 10, 0, 0) == LBFGS_ERR_BAD_ARG && !bad, "m = 0");
}

// the C++ drop-in: LBFGS() with the reference's own objectives and with a caller lambda
static void cxx_dropin() {
    setenv("LBFGS_MODE", "default", 1);
    std::vector<double> x0 = x0_for(200, 42);
    const std::vector<double> a = LBFGS(rosenbrock, rosenbrock_grad, x0, "backtracking", 50, 5, 1e-5, false);
    const OracleRun o = oracle(ORC_OBJ_ROSENBROCK, ORC_LS_BACKTRACKING, 200, 5, 50, x0);
    for (size_t i = 0; i < a.size(); ++i)
        if (!same_bits(a[i], o.x[i])) {
            EXPECT(false, "LBFGS drop-in x[%zu]", i);
            break;
        }
    int calls = 0;
    auto f = [&calls](std::vector<double> x) {
        ++calls;
        double s = 0.0;
        for (double v : x) s += (v - 3.0) * (v - 3.0);
        return s;
    };
    auto g = [](std::vector<double> x) {
        for (double& v : x) v = 2.0 * (v - 3.0);
        return x;
    };
    const std::vector<double> b = LBFGS(f, g, x0, "backtracking", 100, 3, 1e-8, false);
    double err = 0.0;
    for (double v : b) err = std::isfinite(v) ? std::max(err, std::fabs(v - 3.0)) : INFINITY;
    EXPECT(err < 1e-6 && calls > 0, "lambda objective: err %g calls %d", err, calls);
    bool threw = false;
    try {
        LBFGS(f, g, x0, "no_such_search", 10, 3, 1e-8, false);
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    EXPECT(threw, "unknown line search must throw std::invalid_argument");
    const std::vector<double> v1 = {1.0, 2.0, 3.0}, v2 = {4.0, 5.0, 6.0};
    EXPECT(dotProduct(v1, v2) == 32.0, "dotProduct");
}

int main() {
    device_objectives();
    cuda_paths();
    host_callbacks();
    dense_objective();
    api_surface();
    cxx_dropin();
    if (g_fail) {
        std::fprintf(stderr, "%d failure(s)\n", g_fail);
        return 1;
    }
    std::printf("sanitizer job: all checks passed\n");
    return 0;
}
