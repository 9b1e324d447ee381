// oracle/ref_driver.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Golden-trace driver for the *reference* sequential L-BFGS. It is compiled together
// with the reference's own, unmodified sources
//   /root/reference/sequential-implementation/{lbfgs,vector_utils,line_search,benchmark}.cpp
// (and main.cpp with its main() renamed, for the separable quadratic) by oracle/Makefile,
// into oracle/_ref/ref_lbfgs. Nothing here restates the algorithm: it only wraps the
// reference's objective functions so every f / grad call made by the reference
// LBFGS() (lbfgs.cpp:17-203) is observed and logged bit-exactly.
//
// Trace files written (all little-endian binary):
//   <prefix>.f.bin   one double per f() call, in call order
//   <prefix>.g.bin   per grad() call: u64 c1, u64 c2, f64 |g| (sequential, = vectorNorm),
//                    f64 wall seconds since LBFGS() entry, u64 f-calls so far
//                    c1 = sum(bits(x_i)) mod 2^64, c2 = sum((i+1)*bits(x_i)) mod 2^64
//   <prefix>.x.bin   full x (n doubles) for grad calls 0..full_upto-1
//   <prefix>.ret.bin returned x: u64 c1, u64 c2, then (if n <= 200000) the n doubles
//
// usage: ref_lbfgs <obj> <n> <m> <method> <maxit> <tol> <seed> <lo> <hi> <prefix> <full_upto>
//   obj ∈ {rosenbrock, quad_tridiag, quad_sep, stress_tiny_sq, stress_scaled_sq, stress_quartic_well}
//   x0 ~ std::uniform_real_distribution<>(lo, hi) over std::mt19937(seed), as main.cpp:36-43.
// usage: ref_lbfgs kat <n> <seed> <prefix>       (objective known-answer vectors)
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include <lbfgs.h>  // reference declaration, lbfgs.h:17-25

using std::vector;

// Reference objectives (declared in benchmark.h:12-16 / defined in benchmark.cpp, main.cpp).
// Declared here instead of including benchmark.h, which pulls matrices.h (non-inline
// global definitions) into a second translation unit.
std::function<double(const std::vector<double>&)> generate_quadratic_function(int n);
std::function<std::vector<double>(const std::vector<double>&)> generate_quadratic_gradient(int n);
double rosenbrock(const vector<double>& X);
vector<double> rosenbrock_grad(const vector<double>& X);
double quadratic(const vector<double>& X);           // main.cpp:7-13
vector<double> quadratic_grad(const vector<double>& X);  // main.cpp:15-21

static void checksum(const vector<double>& x, uint64_t* c1, uint64_t* c2) {
    uint64_t a = 0, b = 0;
    for (size_t i = 0; i < x.size(); ++i) {
        uint64_t u;
        std::memcpy(&u, &x[i], 8);
        a += u;
        b += (uint64_t)(i + 1) * u;
    }
    *c1 = a;
    *c2 = b;
}

static double seq_norm(const vector<double>& v) {  // same loop as vectorNorm (vector_utils.cpp:78-86)
    double r = 0.;
    for (double e : v) r += e * e;
    return __builtin_sqrt(r);
}

static vector<double> make_x0(int n, unsigned seed, double lo, double hi) {
    std::mt19937 gen(seed);
    std::uniform_real_distribution<> dis(lo, hi);
    vector<double> x0(n);
    for (double& v : x0) v = dis(gen);
    return x0;
}

static void write_all(FILE* fp, const void* p, size_t bytes) {
    if (fwrite(p, 1, bytes, fp) != bytes) {
        std::perror("fwrite");
        std::exit(2);
    }
}

static int run_kat(int n, unsigned seed, const std::string& prefix) {
    // x ~ U(-2, 2); write x, rosenbrock(x), rosenbrock_grad(x), tridiagonal quadratic f/g,
    // separable quadratic f/g — all computed by the reference's own functions.
    vector<double> x = make_x0(n, seed, -2.0, 2.0);
    FILE* fp = std::fopen((prefix + ".kat.bin").c_str(), "wb");
    if (!fp) return 2;
    double fr = rosenbrock(x);
    vector<double> gr = rosenbrock_grad(x);
    auto qf = generate_quadratic_function(n);
    auto qg = generate_quadratic_gradient(n);
    double fq = qf(x);
    vector<double> gq = qg(x);
    double fs = quadratic(x);
    vector<double> gs = quadratic_grad(x);
    write_all(fp, x.data(), 8 * (size_t)n);
    write_all(fp, &fr, 8);
    write_all(fp, gr.data(), 8 * (size_t)n);
    write_all(fp, &fq, 8);
    write_all(fp, gq.data(), 8 * (size_t)n);
    write_all(fp, &fs, 8);
    write_all(fp, gs.data(), 8 * (size_t)n);
    std::fclose(fp);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 5 && std::string(argv[1]) == "kat") {
        return run_kat(std::atoi(argv[2]), (unsigned)std::strtoul(argv[3], nullptr, 10), argv[4]);
    }
    if (argc < 12) {
        std::fprintf(stderr,
                     "usage: %s <obj> <n> <m> <method> <maxit> <tol> <seed> <lo> <hi> <prefix> "
                     "<full_upto>\n",
                     argv[0]);
        return 2;
    }
    const std::string obj = argv[1];
    const int n = std::atoi(argv[2]);
    const int m = std::atoi(argv[3]);
    const std::string method = argv[4];
    const int maxit = std::atoi(argv[5]);
    const double tol = std::strtod(argv[6], nullptr);
    const unsigned seed = (unsigned)std::strtoul(argv[7], nullptr, 10);
    const double lo = std::strtod(argv[8], nullptr);
    const double hi = std::strtod(argv[9], nullptr);
    const std::string prefix = argv[10];
    const long full_upto = std::atol(argv[11]);

    std::function<double(const vector<double>&)> base_f;
    std::function<vector<double>(const vector<double>&)> base_g;
    if (obj == "rosenbrock") {
        base_f = rosenbrock;
        base_g = rosenbrock_grad;
    } else if (obj == "quad_tridiag") {
        base_f = generate_quadratic_function(n);
        base_g = generate_quadratic_gradient(n);
    } else if (obj == "quad_sep") {
        base_f = quadratic;
        base_g = quadratic_grad;
    } else if (obj == "stress_tiny_sq" || obj == "stress_scaled_sq" || obj == "stress_quartic_well") {
        // Stress objectives (ours, not the reference's) that drive the reference LBFGS() down
        // its guard paths (lbfgs.cpp:102-124 invalid rho / gamma, :148-153 non-descent,
        // :164-168 line-search failure). Written term by term, summed left to right, with the
        // operand order tests/oracle_lib.py stress_objective() uses, so both sides agree bit
        // for bit.
        if (obj == "stress_tiny_sq") {  // x ~ 1e-155: s.y subnormal -> 1/(s.y) = inf
            base_f = [](const vector<double>& x) {
                double s = 0.0;
                for (double v : x) s += v * v;
                return s;
            };
            base_g = [](const vector<double>& x) {
                vector<double> g(x.size());
                for (size_t i = 0; i < x.size(); ++i) g[i] = 2.0 * x[i];
                return g;
            };
        } else if (obj == "stress_scaled_sq") {  // gradients ~1e100: y.y overflows -> gamma = 0
            base_f = [](const vector<double>& x) {
                double s = 0.0;
                for (double v : x) s += 1e100 * v * v;
                return s;
            };
            base_g = [](const vector<double>& x) {
                vector<double> g(x.size());
                for (size_t i = 0; i < x.size(); ++i) g[i] = 2.0 * 1e100 * x[i];
                return g;
            };
        } else {  // double well: the Wolfe search's quirky cubic leaves a negative step
            base_f = [](const vector<double>& x) {
                double s = 0.0;
                for (double v : x) s += -0.2 * v * v + 0.0016 * v * v * v * v;
                return s;
            };
            base_g = [](const vector<double>& x) {
                vector<double> g(x.size());
                for (size_t i = 0; i < x.size(); ++i) g[i] = 2.0 * -0.2 * x[i] + 4.0 * 0.0016 * x[i] * x[i] * x[i];
                return g;
            };
        }
    } else {
        std::fprintf(stderr, "unknown objective %s\n", obj.c_str());
        return 2;
    }

    FILE* ff = std::fopen((prefix + ".f.bin").c_str(), "wb");
    FILE* fg = std::fopen((prefix + ".g.bin").c_str(), "wb");
    FILE* fx = std::fopen((prefix + ".x.bin").c_str(), "wb");
    if (!ff || !fg || !fx) {
        std::perror("fopen");
        return 2;
    }

    vector<double> x0 = make_x0(n, seed, lo, hi);
    uint64_t nf = 0, ng = 0;
    auto t0 = std::chrono::steady_clock::now();

    std::function<double(vector<double>)> f = [&](vector<double> x) {
        double v = base_f(x);
        write_all(ff, &v, 8);
        ++nf;
        return v;
    };
    std::function<vector<double>(vector<double>)> grad = [&](vector<double> x) {
        vector<double> g = base_g(x);
        double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        uint64_t c1, c2;
        checksum(x, &c1, &c2);
        double gn = seq_norm(g);
        write_all(fg, &c1, 8);
        write_all(fg, &c2, 8);
        write_all(fg, &gn, 8);
        write_all(fg, &t, 8);
        write_all(fg, &nf, 8);
        if ((long)ng < full_upto) write_all(fx, x.data(), 8 * (size_t)n);
        ++ng;
        return g;
    };

    t0 = std::chrono::steady_clock::now();
    vector<double> xr = LBFGS(f, grad, x0, method, maxit, m, tol, false);
    std::fclose(ff);
    std::fclose(fg);
    std::fclose(fx);

    FILE* fr = std::fopen((prefix + ".ret.bin").c_str(), "wb");
    uint64_t c1, c2;
    checksum(xr, &c1, &c2);
    write_all(fr, &c1, 8);
    write_all(fr, &c2, 8);
    if (n <= 200000) write_all(fr, xr.data(), 8 * (size_t)n);
    std::fclose(fr);
    std::fflush(stdout);
    return 0;
}
