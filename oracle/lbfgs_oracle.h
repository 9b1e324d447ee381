/* oracle/lbfgs_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference sequential L-BFGS
 * (/root/reference/sequential-implementation/lbfgs.cpp:17-203, line_search.cpp:8-189,
 *  vector_utils.cpp:32-86, benchmark.cpp:16-81, main.cpp:7-21) used as the CHECKER for the
 * HIP product. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it. Parity of this restatement is pinned against traces of the reference itself
 * (oracle/_ref, tests/golden/), see tests/test_oracle_golden.py.
 *
 * Two reduction orders:
 *   ORC_SEQ   : strictly left-to-right sums, exactly as the reference (bit-exact vs reference)
 *   ORC_CANON : the product's canonical device tree order, so that the HIP
 *               path can be checked bit-exactly over a whole run.
 */
#ifndef LBFGS_ORACLE_H
#define LBFGS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ORC_OBJ_HOST: the caller's f/grad callbacks (the reference's LBFGS takes any
 * std::function objective, lbfgs.h:9-10); used with the dense quadratics of matrices.h */
enum { ORC_OBJ_ROSENBROCK = 0, ORC_OBJ_QUAD_TRIDIAG = 1, ORC_OBJ_QUAD_SEPARABLE = 2, ORC_OBJ_HOST = 3,
       ORC_OBJ_DENSE = 4 /* x'Ax + b'x, the matrices.h problems (orc_dense_set) */ };
enum { ORC_LS_BACKTRACKING = 0, ORC_LS_INTERPOLATION = 1, ORC_LS_WOLFE = 2, ORC_LS_BACKTRACKING_WOLFE = 3 };
enum { ORC_SEQ = 0, ORC_CANON = 1, ORC_CANON_VF = 2 /* contiguous rows per wave */,
       ORC_PAIR = 3 /* pairwise sums */, ORC_REV = 4 /* right-to-left sums */,
       ORC_FMA = 5 /* left-to-right, products fused */ };
enum { ORC_CONVERGED = 0, ORC_MAX_ITER = 1, ORC_LS_FAILED = 2 };

/* the canonical geometry's size bounds (restating lbfgs_device.h LBK_MIDL*, LBK_VFL_LO): segments
 * are at least ORC_MIDL long for ORC_MIDL_LO <= n <= ORC_MIDL_HI (512 elsewhere); the vector-free
 * commit keeps the 512-minimum base length below ORC_VFL_LO */
#define ORC_MIDL 2048
#define ORC_MIDL_LO 65536
#define ORC_MIDL_HI 2097152
#define ORC_VFL_LO 262144

typedef struct {
    int obj, ls, mode, verbose;
    int64_t n;
    int m, maxit;
    double tol;
    /* config.h:5-17 */
    double c1, c2, initial_step, backtracking_alpha, backtracking_tol, wolfe_interp_min;
    /* ORC_OBJ_HOST only */
    double (*host_f)(const double* x, int64_t n, void* user);
    void (*host_g)(const double* x, int64_t n, double* g, void* user);
    void* host_user;
    /* 1: vector-free (Gram-matrix) variant of the product's LBFGS_FLAG_VECTOR_FREE mode,
     * restated in ORC_CANON order (not a reference algorithm; its own parity contract) */
    int vf;
    /* 1: the CUDA path - LBFGS_CUDA of parallel-implementation/L-BFGS.cu:105-380 with the line
     * searches of parallel-implementation/line_search.cpp (the product's LBFGS_FLAG_CUDA_COMPAT) */
    int cuda; /* 1: the CUDA path, L-BFGS.cu (orc_lbfgs_cuda); 2: the variant files' loops (their inline searches) */
} orc_opts;

typedef struct {
    int iters, status, ntrace;
    int64_t nf, ng;
    int64_t skips; /* the CUDA path: first-loop pairs skipped for s.y <= 1e-10 (L-BFGS.cu:222-223) */
} orc_result;

/* x0 exactly as std::mt19937(seed) + std::uniform_real_distribution<double>(lo, hi)
 * (libstdc++ generate_canonical<double,53>, two 32-bit draws per value; main.cpp:36-43). */
void orc_x0_uniform(double* x, int64_t n, uint32_t seed, double lo, double hi);

/* Reductions. */
double orc_dot(const double* a, const double* b, int64_t n, int mode);
double orc_sum(const double* t, int64_t n, int64_t limit, int mode); /* terms t[e], e < limit */
void orc_canon_geometry(int64_t n, int64_t* seg_len, int64_t* nseg);
int orc_vf_factor(int64_t n); /* vector-free commit segment, in canonical segments */
/* group partials Q_0..Q_7 of the canonical order (total = sequential sum of the 8). */
void orc_canon_dot_groups(const double* a, const double* b, int64_t n, double* q8);

/* Dense quadratic data for ORC_OBJ_DENSE (A n x n row-major, b; kept by pointer). Row i of Ax is
 * formed as the product's k_dense_rows does in every mode: 64 lane sums over j = l, l+64, ...
 * (fma, ascending), then the butterfly v_l + v_{l^m}, m = 1, 2, ..., 32; grad_i = 2 r_i + b_i,
 * f = sum of x_i r_i + b_i x_i in the mode's order. */
void orc_dense_set(const double* A, const double* b);

/* Objectives (benchmark.cpp:16-81, main.cpp:7-21). */
double orc_f(int obj, const double* x, int64_t n, int mode);
void orc_grad(int obj, const double* x, int64_t n, double* g);

/* Full L-BFGS run. Trace entry k = state at the top of iteration k (plus the final state);
 * tr_alpha[k] = step taken in iteration k (NaN for the last entry). flog/glog record every
 * objective call in the reference's call order (reference-faithful evaluation). */
int orc_lbfgs(const orc_opts* o, const double* x0, double* x_out,
              double* tr_f, double* tr_gnorm, double* tr_alpha, uint64_t* tr_c1, uint64_t* tr_c2,
              int64_t* tr_nf, int trace_cap,
              double* flog, int64_t flog_cap, int64_t* flog_n,
              uint64_t* glog, int64_t glog_cap, int64_t* glog_n,
              char* msg, int msg_cap, orc_result* res);

void orc_checksum(const double* x, int64_t n, uint64_t* c1, uint64_t* c2);

/* one line search of parallel-implementation/line_search.cpp (orc_opts.ls, constants in o; the
 * CUDA path's searches) from x along d with gradient g; f / grad calls logged as in orc_lbfgs */
int orc_cuda_line_search(const orc_opts* o, const double* x, const double* d, const double* g, double* alpha,
                         double* flog, int64_t flog_cap, int64_t* flog_n, uint64_t* glog, int64_t glog_cap,
                         int64_t* glog_n);

/* two-loop recursion alone for history S/Y[0..h-1] (oldest first); writes d, returns g.d */
double orc_twoloop(const double* g, const double* const* S, const double* const* Y, int h,
                   int64_t n, int mode, double* d);

#ifdef __cplusplus
}
#endif
#endif
