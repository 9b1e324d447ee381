/* oracle/lbfgs_oracle.c — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * A plain-C restatement of the reference algorithm, used as the checker for the HIP path.
 * Each function cites the reference lines it restates. Compiled with -ffp-contract=off so that
 * every a*b+c below is two roundings, exactly like the reference binary (x86-64, no FMA).
 * The only FMA is the explicit fma() of the canonical dot (ORC_CANON), which mirrors the
 * device kernels' v_fma_f64 accumulation.
 */
#include "lbfgs_oracle.h"

#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* Vector loops run over OpenMP threads where n is large: every parallel loop below writes
 * disjoint elements (or canonical segment partials, or exact integer sums), so the results are
 * the sequential program's bit for bit; only the time changes (configs[4]'s n = 1e9 restated on
 * a 16-core host, tests/golden/make_fullsize.py). Without -fopenmp the pragmas are ignored. */
#define ORC_PAR_MIN 65536
#define ORC_STR(x) #x
#define ORC_PAR(n) _Pragma(ORC_STR(omp parallel for schedule(static) if ((n) > ORC_PAR_MIN)))

/* ------------------------------------------------------------------------------------------
 * x0: std::mt19937 + std::uniform_real_distribution<double> (libstdc++ 11)
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    uint32_t mt[624];
    int idx;
} mt19937;

static void mt_seed(mt19937* s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; ++i)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->idx = 624;
}

static uint32_t mt_next(mt19937* s) {
    if (s->idx >= 624) {
        for (int i = 0; i < 624; ++i) {
            uint32_t y = (s->mt[i] & 0x80000000u) | (s->mt[(i + 1) % 624] & 0x7fffffffu);
            s->mt[i] = s->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        s->idx = 0;
    }
    uint32_t y = s->mt[s->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

void orc_x0_uniform(double* x, int64_t n, uint32_t seed, double lo, double hi) {
    mt19937* s = (mt19937*)malloc(sizeof(mt19937));
    mt_seed(s, seed);
    for (int64_t i = 0; i < n; ++i) {
        /* generate_canonical<double,53>: sum = g1 + g2 * 2^32 (rounded), / 2^64 */
        double sum = 0.0, tmp = 1.0;
        for (int k = 0; k < 2; ++k) {
            sum += (double)mt_next(s) * tmp;
            tmp *= 4294967296.0;
        }
        double u = sum / tmp;
        if (u >= 1.0) u = nextafter(1.0, 0.0);
        x[i] = u * (hi - lo) + lo; /* uniform_real_distribution::operator() */
    }
    free(s);
}

void orc_checksum(const double* x, int64_t n, uint64_t* c1, uint64_t* c2) {
    uint64_t a = 0, b = 0; /* modular integer sums: exact in any order */
#pragma omp parallel for schedule(static) reduction(+ : a, b) if (n > ORC_PAR_MIN)
    for (int64_t i = 0; i < n; ++i) {
        uint64_t u;
        memcpy(&u, &x[i], 8);
        a += u;
        b += (uint64_t)(i + 1) * u;
    }
    *c1 = a;
    *c2 = b;
}

/* ------------------------------------------------------------------------------------------
 * Reductions.
 * ORC_SEQ  : vector_utils.cpp:32-41 (dotProduct), :78-86 (vectorNorm) — left to right.
 * ORC_CANON: the device order:
 *   seg_len L = max(Lmin, roundup(ceil(n/8192), 128)), Lmin = 2048 for 65536 <= n <= 2097152
 *   (lbfgs_kernels.hip lbk_geometry_plan: n that cannot shard), 512 otherwise;
 *   segment s = [sL, min((s+1)L, n));
 *   thread t = 64w + lane (256 per segment); thread t visits, for u = 0.., row r = 4u + w,
 *   elements sL + 128r + 2 lane + v (v = 0,1) that are < segment end and < limit;
 *   dot: acc = fma(a, b, acc); sum: acc = acc + t.
 *   segment partial = balanced pairwise tree over the 256 thread accumulators;
 *   group g partial  = balanced pairwise tree over segment partials 1024g..1024g+1023
 *                      (0.0 for segments >= nseg);
 *   total = ((((((Q0+Q1)+Q2)+Q3)+Q4)+Q5)+Q6)+Q7.
 * ---------------------------------------------------------------------------------------- */
#define CANON_SEGS 8192
#define CANON_GROUPS 8
#define CANON_SEG_PER_GROUP 1024

void orc_canon_geometry(int64_t n, int64_t* seg_len, int64_t* nseg) {
    int64_t per = (n + CANON_SEGS - 1) / CANON_SEGS;
    int64_t L = ((per + 127) / 128) * 128;
    const int64_t lmin = (n >= ORC_MIDL_LO && n <= ORC_MIDL_HI) ? ORC_MIDL : 512;
    if (L < lmin) L = lmin;
    *seg_len = L;
    *nseg = (n + L - 1) / L;
}

/* The vector-free commit's segments (lbfgs_kernels.hip vgeo / lbk_vf_factor): F canonical
 * segments each, F the largest of {1, 2, 4, 8} with 2 F L0 <= 8192 and
 * ceil(n / (2 F L0)) >= 1024 while doubling, L0 = max(512, roundup(ceil(n/8192), 128)) (the
 * canonical length without the mid-n minimum); 1024 / F of them per group, placed first in the
 * group's 1024-entry tree (0.0 behind). */
int orc_vf_factor(int64_t n) {
    int64_t per = (n + CANON_SEGS - 1) / CANON_SEGS;
    int64_t L = ((per + 127) / 128) * 128;
    if (L < 512) L = 512;
    int F = 1;
    while (F < 8 && 2 * F * L <= 8192 && (n + 2 * F * L - 1) / (2 * F * L) >= 1024) F *= 2;
    return F;
}

static double tree_sum(double* a, int count) { /* balanced, natural order, in place */
    for (int w = count; w > 1; w >>= 1)
        for (int j = 0; j < w / 2; ++j) a[j] = a[2 * j] + a[2 * j + 1];
    return a[0];
}

/* kind 0: dot of (a,b) with fma; kind 1: sum of a[].
 * Row-to-wave assignment within a segment: rows r = 4u + w (the default order), or, for
 * ORC_CANON_VF (the vector-free commit, lbfgs_kernels.hip stream_vf), contiguous runs: wave w
 * takes rows [wR, min((w+1)R, nrow)), R = ceil(nrow / 4), nrow = rows of the segment's
 * elements. Each lane accumulates its rows in ascending order either way. */
static void canon_groups_mode(const double* a, const double* b, int64_t n, int64_t limit, int kind, int contig,
                              double* q8) {
    int64_t L, nseg;
    orc_canon_geometry(n, &L, &nseg);
    int64_t spg = CANON_SEG_PER_GROUP;
    if (contig) {
        /* base length: the canonical L, except ORC_MIDL_LO <= n < ORC_VFL_LO where the
         * vector-free commit keeps the 512-minimum length (lbfgs_kernels.hip vf_base_len) */
        const int F = orc_vf_factor(n);
        if (n >= ORC_MIDL_LO && n < ORC_VFL_LO) {
            const int64_t per = (n + CANON_SEGS - 1) / CANON_SEGS;
            L = ((per + 127) / 128) * 128;
            if (L < 512) L = 512;
        }
        L *= F;
        nseg = (n + L - 1) / L;
        spg /= F;
    }
    double* segp = (double*)calloc(CANON_SEGS, sizeof(double));
#pragma omp parallel for schedule(dynamic, 4) if (n > ORC_PAR_MIN)
    for (int64_t s = 0; s < nseg; ++s) {
        double acc[256];
        int64_t sbeg = s * L;
        int64_t send = sbeg + L < n ? sbeg + L : n;
        const int64_t nrow = (send - sbeg + 127) / 128, R = (nrow + 3) / 4;
        if (send > limit) send = limit > sbeg ? limit : sbeg;
        for (int t = 0; t < 256; ++t) {
            int w = t >> 6, lane = t & 63;
            double v = 0.0;
            for (int64_t u = 0;; ++u) {
                int64_t row;
                if (contig) {
                    row = w * R + u;
                    if (u >= R || row >= nrow) break;
                } else {
                    row = 4 * u + w; /* rows r = 4u + w of the segment */
                    if (128 * row >= L) break;
                }
                int64_t base = sbeg + 128 * row + 2 * lane;
                for (int k = 0; k < 2; ++k) {
                    int64_t e = base + k;
                    if (e < send) v = kind == 0 ? fma(a[e], b[e], v) : v + a[e];
                }
            }
            acc[t] = v;
        }
        segp[(s / spg) * CANON_SEG_PER_GROUP + s % spg] = tree_sum(acc, 256);
    }
    for (int g = 0; g < CANON_GROUPS; ++g) q8[g] = tree_sum(segp + g * CANON_SEG_PER_GROUP, CANON_SEG_PER_GROUP);
    free(segp);
}

static void canon_groups(const double* a, const double* b, int64_t n, int64_t limit, int kind, double* q8) {
    canon_groups_mode(a, b, n, limit, kind, 0, q8);
}

static double canon_total(const double* q8) {
    double t = q8[0];
    for (int g = 1; g < CANON_GROUPS; ++g) t = t + q8[g];
    return t;
}

void orc_canon_dot_groups(const double* a, const double* b, int64_t n, double* q8) {
    canon_groups(a, b, n, n, 0, q8);
}

/* ORC_PAIR / ORC_REV / ORC_FMA: other legitimate summation orders of the same products / terms
 * (recursive pairwise halving with 8-term sequential leaves; strictly right to left; left to
 * right with the products fused into the additions, as an FMA-contracting build). Not a
 * device order: they measure how long the reference agrees with ITSELF when only the order of
 * its sums changes (tests/test_oracle_horizons.py), the yardstick for the canonical order's
 * horizon against the reference. */
static double pair_sum(const double* a, const double* b, int64_t lo, int64_t hi) {
    if (hi - lo <= 8) {
        double s = 0.0;
        for (int64_t i = lo; i < hi; ++i) s += b ? a[i] * b[i] : a[i];
        return s;
    }
    const int64_t mid = lo + (hi - lo) / 2;
    return pair_sum(a, b, lo, mid) + pair_sum(a, b, mid, hi);
}

static double alt_sum(const double* a, const double* b, int64_t limit, int mode) {
    if (mode == ORC_PAIR) return pair_sum(a, b, 0, limit);
    if (mode == ORC_FMA) { /* left to right, products contracted (the reference built with FMA) */
        double s = 0.0;
        for (int64_t i = 0; i < limit; ++i) s = b ? fma(a[i], b[i], s) : s + a[i];
        return s;
    }
    double s = 0.0;
    for (int64_t i = limit - 1; i >= 0; --i) s += b ? a[i] * b[i] : a[i];
    return s;
}

double orc_dot(const double* a, const double* b, int64_t n, int mode) {
    if (mode == ORC_PAIR || mode == ORC_REV || mode == ORC_FMA) return alt_sum(a, b, n, mode);
    if (mode == ORC_CANON || mode == ORC_CANON_VF) {
        double q8[CANON_GROUPS];
        canon_groups_mode(a, b, n, n, 0, mode == ORC_CANON_VF, q8);
        return canon_total(q8);
    }
    double sum = 0.; /* vector_utils.cpp:36-38 */
    for (int64_t i = 0; i < n; ++i) sum += a[i] * b[i];
    return sum;
}

double orc_sum(const double* t, int64_t n, int64_t limit, int mode) {
    if (mode == ORC_PAIR || mode == ORC_REV || mode == ORC_FMA) return alt_sum(t, NULL, limit, mode);
    if (mode == ORC_CANON || mode == ORC_CANON_VF) {
        double q8[CANON_GROUPS];
        canon_groups_mode(t, NULL, n, limit, 1, mode == ORC_CANON_VF, q8);
        return canon_total(q8);
    }
    double sum = 0.0;
    for (int64_t i = 0; i < limit; ++i) sum += t[i];
    return sum;
}

static double orc_norm(const double* v, int64_t n, int mode) {
    if (mode == ORC_CANON || mode == ORC_PAIR || mode == ORC_REV || mode == ORC_FMA) return sqrt(orc_dot(v, v, n, mode));
    double r = 0.; /* vector_utils.cpp:80-85 */
    for (int64_t i = 0; i < n; ++i) r += v[i] * v[i];
    return sqrt(r);
}

/* ------------------------------------------------------------------------------------------
 * Objectives.
 * ---------------------------------------------------------------------------------------- */
static double* g_terms = NULL; /* scratch for canonical f */
static int64_t g_terms_n = 0;

static double* terms_buf(int64_t n) {
    if (g_terms_n < n) {
        free(g_terms);
        g_terms = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
        g_terms_n = n;
    }
    return g_terms;
}

static const double* g_dense_A;
static const double* g_dense_b;

void orc_dense_set(const double* A, const double* b) {
    g_dense_A = A;
    g_dense_b = b;
}

/* row of A x in the device's order (lbfgs_kernels.hip k_dense_rows) */
static double dense_row(const double* a, const double* x, int64_t n) {
    double v[64], w[64];
    for (int l = 0; l < 64; ++l) {
        v[l] = 0.0;
        for (int64_t j = l; j < n; j += 64) v[l] = fma(a[j], x[j], v[l]);
    }
    for (int m = 1; m < 64; m <<= 1) {
        for (int l = 0; l < 64; ++l) w[l] = v[l] + v[l ^ m];
        memcpy(v, w, sizeof v);
    }
    return v[0];
}

double orc_f(int obj, const double* x, int64_t n, int mode) {
    if (obj == ORC_OBJ_DENSE) {
        double* t = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
        for (int64_t i = 0; i < n; ++i) {
            const double r = dense_row(g_dense_A + i * n, x, n);
            t[i] = x[i] * r + g_dense_b[i] * x[i];
        }
        double f;
        if (mode == ORC_SEQ) {
            f = 0.0;
            for (int64_t i = 0; i < n; ++i) f += t[i];
        } else {
            f = orc_sum(t, n, n, mode);
        }
        free(t);
        return f;
    }
    if (mode == ORC_SEQ) {
        double sum = 0.0;
        if (obj == ORC_OBJ_ROSENBROCK) { /* benchmark.cpp:58-68 */
            for (int64_t i = 0; i + 1 < n; i++) {
                double term1 = x[i + 1] - x[i] * x[i];
                double term2 = 1 - x[i];
                sum += 100.0 * term1 * term1 + term2 * term2;
            }
        } else if (obj == ORC_OBJ_QUAD_TRIDIAG) { /* benchmark.cpp:17-33 */
            for (int64_t i = 0; i < n; i++) sum += 1000.0 * x[i] * x[i];
            for (int64_t i = 0; i < n - 1; i++) sum += (1000.0 / 10.0) * x[i] * x[i + 1];
        } else { /* main.cpp:7-13 */
            for (int64_t i = 0; i < n; i++) sum += (x[i] - 1) * (x[i] - 1);
        }
        return sum;
    }
    /* canonical: the same per-element terms, summed in the device order */
    double* t = terms_buf(n);
    int64_t limit = n;
    if (obj == ORC_OBJ_ROSENBROCK) {
        ORC_PAR(n)
        for (int64_t i = 0; i < n - 1; i++) {
            double term1 = x[i + 1] - x[i] * x[i];
            double term2 = 1 - x[i];
            t[i] = 100.0 * term1 * term1 + term2 * term2;
        }
        limit = n - 1;
    } else if (obj == ORC_OBJ_QUAD_TRIDIAG) {
        ORC_PAR(n)
        for (int64_t i = 0; i < n; i++) {
            double dterm = 1000.0 * x[i] * x[i];
            t[i] = (i + 1 < n) ? dterm + 100.0 * x[i] * x[i + 1] : dterm;
        }
    } else {
        ORC_PAR(n)
        for (int64_t i = 0; i < n; i++) t[i] = (x[i] - 1) * (x[i] - 1);
    }
    return orc_sum(t, n, limit, mode);
}

void orc_grad(int obj, const double* x, int64_t n, double* g) {
    if (obj == ORC_OBJ_DENSE) {
        for (int64_t i = 0; i < n; ++i) g[i] = 2.0 * dense_row(g_dense_A + i * n, x, n) + g_dense_b[i];
        return;
    }
    /* benchmark.cpp's loops add into grad[i] and grad[i + 1] from iteration i; per element that is
     * grad[i] = (0.0 + 200 term2_{i-1}) + (term1_i - 400 x_i term2_i) (Rosenbrock, :70-81) and
     * grad[i] = (2000 x_i + 100 x_{i-1}) + 100 x_{i+1} (tridiagonal, :37-56): the same additions in
     * the same order, written element by element so that the elements can run in parallel */
    if (obj == ORC_OBJ_ROSENBROCK) { /* benchmark.cpp:70-81 */
        ORC_PAR(n)
        for (int64_t i = 0; i < n; ++i) {
            double v = 0.0;
            if (i > 0) {
                double term2 = x[i] - x[i - 1] * x[i - 1];
                v += 200.0 * term2; /* grad[i + 1] += 200 term2 of iteration i - 1 */
            }
            if (i + 1 < n) {
                double term1 = 2.0 * (x[i] - 1);
                double term2 = x[i + 1] - x[i] * x[i];
                v += term1 - 400.0 * x[i] * term2; /* grad[i] += ... of iteration i */
            }
            g[i] = v;
        }
    } else if (obj == ORC_OBJ_QUAD_TRIDIAG) { /* benchmark.cpp:37-56 */
        ORC_PAR(n)
        for (int64_t i = 0; i < n; i++) {
            double v = 2.0 * 1000.0 * x[i];
            if (i > 0) v += (1000.0 / 10.0) * x[i - 1];     /* grad[i + 1] += ... of iteration i - 1 */
            if (i + 1 < n) v += (1000.0 / 10.0) * x[i + 1]; /* grad[i] += ... of iteration i */
            g[i] = v;
        }
    } else { /* main.cpp:15-21 */
        ORC_PAR(n)
        for (int64_t i = 0; i < n; i++) g[i] = 2.0 * (x[i] - 1);
    }
}

/* ------------------------------------------------------------------------------------------
 * Driver state, call logging.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    const orc_opts* o;
    int64_t n;
    double* flog;
    int64_t flog_cap, flog_n;
    uint64_t* glog;
    int64_t glog_cap, glog_n;
    int64_t nf, ng;
    char* msg;
    int msg_cap, msg_len;
    double* tmp; /* trial point scratch */
} ctx_t;

static void say(ctx_t* c, const char* fmt, ...) {
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    int k = vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c->o->verbose) fputs(buf, stdout);
    if (c->msg && k > 0 && c->msg_len + k < c->msg_cap) {
        memcpy(c->msg + c->msg_len, buf, (size_t)k);
        c->msg_len += k;
        c->msg[c->msg_len] = 0;
    }
}

static double F(ctx_t* c, const double* x) {
    double v = c->o->obj == ORC_OBJ_HOST ? c->o->host_f(x, c->n, c->o->host_user)
                                          : orc_f(c->o->obj, x, c->n, c->o->mode);
    if (c->flog && c->flog_n < c->flog_cap) c->flog[c->flog_n++] = v;
    c->nf++;
    return v;
}

static void G(ctx_t* c, const double* x, double* g) {
    if (c->o->obj == ORC_OBJ_HOST)
        c->o->host_g(x, c->n, g, c->o->host_user);
    else
        orc_grad(c->o->obj, x, c->n, g);
    if (c->glog && c->glog_n + 3 <= c->glog_cap) {
        uint64_t c1, c2, gb;
        double gn = orc_norm(g, c->n, ORC_SEQ); /* the trace driver logs the sequential norm */
        orc_checksum(x, c->n, &c1, &c2);
        memcpy(&gb, &gn, 8);
        c->glog[c->glog_n++] = c1;
        c->glog[c->glog_n++] = c2;
        c->glog[c->glog_n++] = gb;
    }
    c->ng++;
}

static void trial_point(const double* x, const double* d, double alpha, int64_t n, double* out) {
    ORC_PAR(n)
    for (int64_t i = 0; i < n; ++i) out[i] = x[i] + alpha * d[i]; /* add(x, scalarProduct(alpha, d)) */
}

/* ------------------------------------------------------------------------------------------
 * Line searches — line_search.cpp:8-189.
 * ---------------------------------------------------------------------------------------- */
static double cubic_interp(double a0, double a1, double p0, double dp0, double p1, double dp1) {
    double d1 = dp0 + dp1 - 3 * (p1 - p0) / (a1 - a0); /* line_search.cpp:9-11 */
    double d2 = copysign(sqrt(d1 * d1 - dp0 * dp1), a1 - a0);
    return a0 + (a1 - a0) * (dp0 + d2 - d1) / (dp0 - dp1 + 2 * d2);
}

static double quad_interp(double a0, double a1, double p0, double dp0, double p1) {
    (void)a1; /* line_search.cpp:14-16 */
    return a0 - 0.5 * dp0 * a0 * a0 / (p1 - p0 - dp0 * a0);
}

static double ls_backtracking(ctx_t* c, const double* x, const double* d, const double* g) {
    const orc_opts* o = c->o; /* line_search.cpp:19-30 */
    double alpha = o->initial_step;
    for (;;) {
        double fx = F(c, x);
        trial_point(x, d, alpha, c->n, c->tmp);
        double ft = F(c, c->tmp);
        double gd = orc_dot(g, d, c->n, o->mode);
        if (!(fx - ft < o->c1 * alpha * gd)) break;
        alpha *= o->backtracking_alpha;
        if (alpha < o->backtracking_tol) break;
    }
    return alpha;
}

static double ls_backtracking_wolfe(ctx_t* c, const double* x, const double* d, const double* g,
                                    double* gnew) {
    const orc_opts* o = c->o; /* line_search.cpp:33-55 */
    double alpha = o->initial_step;
    for (;;) {
        trial_point(x, d, alpha, c->n, c->tmp);
        G(c, c->tmp, gnew);
        double fn = F(c, c->tmp);
        double fx = F(c, x);
        double gd = orc_dot(g, d, c->n, o->mode);
        if (fn > fx + o->c1 * alpha * gd) {
            alpha *= o->backtracking_alpha;
        } else if (orc_dot(gnew, d, c->n, o->mode) < o->c2 * gd) {
            alpha *= 1.1;
        } else {
            break;
        }
        if (alpha < o->backtracking_tol) break;
    }
    return alpha;
}

static double ls_interpolation(ctx_t* c, const double* x, const double* d, const double* g) {
    const orc_opts* o = c->o; /* line_search.cpp:57-121 */
    const double f_x = F(c, x);
    const double gd = orc_dot(g, d, c->n, o->mode);
    double alpha = o->initial_step, alpha_prev = 0.0, f_prev = f_x;
    int it = 0;
    while (it++ < 20) {
        trial_point(x, d, alpha, c->n, c->tmp);
        double f_new = F(c, c->tmp);
        if (f_new <= f_x + o->c1 * alpha * gd) return alpha;
        if (alpha < o->wolfe_interp_min) return o->wolfe_interp_min;
        if (alpha_prev > 0) {
            double delta = alpha - alpha_prev;
            if (fabs(delta) < 1e-10) {
                alpha *= 0.5;
            } else {
                double ga = (f_new - f_x - gd * alpha) / (alpha * alpha);
                alpha = cubic_interp(alpha_prev, alpha, f_prev, gd, f_new, ga);
                if (alpha < 0.1 * alpha_prev || alpha > 0.9 * alpha_prev) alpha = alpha_prev * 0.5;
            }
        } else {
            alpha = quad_interp(alpha, 0.0, f_new, gd, f_x);
            if (alpha < 0.1 * o->initial_step || alpha > 0.9 * o->initial_step)
                alpha = o->initial_step * 0.5;
        }
        alpha_prev = alpha;
        f_prev = f_new;
    }
    return alpha;
}

static double ls_wolfe(ctx_t* c, const double* x, const double* d, const double* g, double* gnew) {
    const orc_opts* o = c->o; /* line_search.cpp:125-189 */
    const double f_x = F(c, x);
    const double gd = orc_dot(g, d, c->n, o->mode);
    double alpha = o->initial_step;
    double alpha_lo = 0.0, alpha_hi = INFINITY, f_lo = f_x, dphi_lo = gd;
    for (int iter = 0; iter < 20; ++iter) {
        trial_point(x, d, alpha, c->n, c->tmp);
        double f_new = F(c, c->tmp);
        if (f_new > f_x + o->c1 * alpha * gd || (f_new >= f_lo && iter > 0)) {
            alpha_hi = alpha;
            alpha = cubic_interp(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new,
                                 (f_new - f_x - gd * alpha) / (alpha * alpha));
            continue;
        }
        G(c, c->tmp, gnew);
        double dphi_new = orc_dot(gnew, d, c->n, o->mode);
        if (fabs(dphi_new) <= -o->c2 * gd) return alpha;
        if (dphi_new >= 0) {
            alpha_hi = alpha;
            alpha = cubic_interp(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        } else {
            alpha_lo = alpha;
            f_lo = f_new;
            dphi_lo = dphi_new;
            if (alpha_hi == INFINITY)
                alpha *= 2;
            else
                alpha = cubic_interp(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        }
        if (alpha < o->wolfe_interp_min) return o->wolfe_interp_min;
    }
    return alpha;
}


/* ------------------------------------------------------------------------------------------
 * Vector-free variant (orc_opts.vf), restating cuda-lbfgs_amd/csrc/lbfgs_driver.c's
 * iterate_vf and k_vf_commit in the canonical order. The two-loop recursion of lbfgs.cpp:94-143
 * runs over the Gram matrix of the basis [s_0..s_{h-1}, y_0..y_{h-1}, g]; d is the combination
 * c_0 b_0 + c_1 b_1 + ... + cg g (left to right, each product rounded); g.d comes from the Gram
 * row of g; the new Gram rows of y_new and g_new are canonical dots, the row of s_new is
 * derived as alpha (d . v). Every host sum runs s terms, y terms, then g, from 0.0. The line
 * searches are those of line_search.cpp with f(x) and g.d evaluated once (identical values).
 * ---------------------------------------------------------------------------------------- */
#define VF_NA 1 /* backtracking candidates reduced by the first commit pass */
typedef struct {
    ctx_t* C;
    const double *x, *d;
    double* gt;    /* trial gradient scratch */
    double a0, f0, dphi0; /* the fused first trial */
    double cand[VF_NA], fc[VF_NA]; /* f at a0 beta^j, j = 1, 2, in the ORC_CANON_VF order */
} vf_ls_t;

static double vf_trial(vf_ls_t* L, double alpha, int need_g, double* dphi) {
    ctx_t* c = L->C;
    if (alpha == L->a0) {
        if (dphi) *dphi = L->dphi0;
        return L->f0;
    }
    if (!need_g)
        for (int j = 0; j < VF_NA; ++j)
            if (alpha == L->cand[j]) return L->fc[j];
    trial_point(L->x, L->d, alpha, c->n, c->tmp);
    double f = F(c, c->tmp);
    if (need_g) {
        G(c, c->tmp, L->gt);
        *dphi = orc_dot(L->gt, L->d, c->n, ORC_CANON);
    }
    return f;
}

static double vf_ls(vf_ls_t* L, double f_x, double gd) {
    const orc_opts* o = L->C->o;
    double alpha = o->initial_step;
    if (o->ls == ORC_LS_BACKTRACKING) {
        for (;;) {
            double ft = vf_trial(L, alpha, 0, NULL);
            if (!(f_x - ft < o->c1 * alpha * gd)) break;
            alpha *= o->backtracking_alpha;
            if (alpha < o->backtracking_tol) break;
        }
        return alpha;
    }
    if (o->ls == ORC_LS_BACKTRACKING_WOLFE) {
        for (;;) {
            double dphi;
            double fn = vf_trial(L, alpha, 1, &dphi);
            if (fn > f_x + o->c1 * alpha * gd) {
                alpha *= o->backtracking_alpha;
            } else if (dphi < o->c2 * gd) {
                alpha *= 1.1;
            } else {
                break;
            }
            if (alpha < o->backtracking_tol) break;
        }
        return alpha;
    }
    if (o->ls == ORC_LS_INTERPOLATION) {
        double alpha_prev = 0.0, f_prev = f_x;
        int it = 0;
        while (it++ < 20) {
            double f_new = vf_trial(L, alpha, 0, NULL);
            if (f_new <= f_x + o->c1 * alpha * gd) return alpha;
            if (alpha < o->wolfe_interp_min) return o->wolfe_interp_min;
            if (alpha_prev > 0) {
                double delta = alpha - alpha_prev;
                if (fabs(delta) < 1e-10) {
                    alpha *= 0.5;
                } else {
                    double ga = (f_new - f_x - gd * alpha) / (alpha * alpha);
                    alpha = cubic_interp(alpha_prev, alpha, f_prev, gd, f_new, ga);
                    if (alpha < 0.1 * alpha_prev || alpha > 0.9 * alpha_prev) alpha = alpha_prev * 0.5;
                }
            } else {
                alpha = quad_interp(alpha, 0.0, f_new, gd, f_x);
                if (alpha < 0.1 * o->initial_step || alpha > 0.9 * o->initial_step) alpha = o->initial_step * 0.5;
            }
            alpha_prev = alpha;
            f_prev = f_new;
        }
        return alpha;
    }
    /* Wolfe */
    double alpha_lo = 0.0, alpha_hi = INFINITY, f_lo = f_x, dphi_lo = gd;
    for (int iter = 0; iter < 20; ++iter) {
        double f_new = vf_trial(L, alpha, 0, NULL);
        if (f_new > f_x + o->c1 * alpha * gd || (f_new >= f_lo && iter > 0)) {
            alpha_hi = alpha;
            alpha = cubic_interp(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, (f_new - f_x - gd * alpha) / (alpha * alpha));
            continue;
        }
        double dphi_new;
        f_new = vf_trial(L, alpha, 1, &dphi_new);
        if (fabs(dphi_new) <= -o->c2 * gd) return alpha;
        if (dphi_new >= 0) {
            alpha_hi = alpha;
            alpha = cubic_interp(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        } else {
            alpha_lo = alpha;
            f_lo = f_new;
            dphi_lo = dphi_new;
            if (alpha_hi == INFINITY)
                alpha *= 2;
            else
                alpha = cubic_interp(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        }
        if (alpha < o->wolfe_interp_min) return o->wolfe_interp_min;
    }
    return alpha;
}

/* d = c_0 b_0 + ... + c_{2h-1} b_{2h-1} + cg g (h == 0: cg g) */
static void vf_direction(int h, double* const* B, const double* cb, double cg, const double* g, int64_t n, double* d) {
    for (int64_t i = 0; i < n; ++i) {
        double v = 0.0;
        for (int l = 0; l < 2 * h; ++l) v = (l == 0) ? cb[0] * B[0][i] : v + cb[l] * B[l][i];
        d[i] = h == 0 ? cg * g[i] : v + cg * g[i];
    }
}

#define VGI(p, q) ((p) * (m + 1) + (q))

static int orc_lbfgs_vf(const orc_opts* o, const double* x0, double* x_out, double* tr_f, double* tr_gnorm,
                        double* tr_alpha, uint64_t* tr_c1, uint64_t* tr_c2, int64_t* tr_nf, int trace_cap,
                        ctx_t* Cp, orc_result* res) {
    ctx_t* C = Cp;
    const int64_t n = o->n;
    const int m = o->m;
    const size_t vb = sizeof(double) * (size_t)n;
    double *x = malloc(vb), *g = malloc(vb), *d = malloc(vb), *xn = malloc(vb), *gn = malloc(vb), *gt = malloc(vb);
    C->tmp = malloc(vb);
    double *S[65], *Y[65];
    for (int i = 0; i <= m; ++i) {
        S[i] = malloc(vb);
        Y[i] = malloc(vb);
    }
    const size_t P = (size_t)m + 1;
    double *Gss = calloc(P * P, sizeof(double)), *Gsy = calloc(P * P, sizeof(double)),
           *Gyy = calloc(P * P, sizeof(double)), *Gsg = calloc(P, sizeof(double)), *Gyg = calloc(P, sizeof(double));
    int ring[65], h = 0, free_pair = 0;
    double cs[64], cy[64], cg, YB[128], GB[128];
    double* B[128];

    memcpy(x, x0, vb);
    double f_cur = F(C, x);
    G(C, x, g);
    double gg = orc_dot(g, g, n, ORC_CANON);
    int status = ORC_MAX_ITER, ntr = 0, k;
    for (k = 0; k < o->maxit; ++k) {
        const double gnorm = sqrt(gg);
        if (ntr < trace_cap) {
            tr_f[ntr] = f_cur;
            tr_gnorm[ntr] = gnorm;
            tr_alpha[ntr] = NAN;
            orc_checksum(x, n, &tr_c1[ntr], &tr_c2[ntr]);
            tr_nf[ntr] = C->nf;
        }
        if (o->verbose) printf("Iteration %d, f = %g, |grad| = %g\n", k, f_cur, gnorm);
        if (gnorm < o->tol) {
            say(C, "Converged!\n");
            status = ORC_CONVERGED;
            ntr++;
            goto done;
        }
        for (int j = 0; j < h; ++j) cs[j] = cy[j] = 0.0;
        cg = -1.0;
        if (!(k == 0 || h == 0)) {
            int bad = 0;
            for (int i = h - 1; i >= 0; --i)
                if (!isfinite(1.0 / Gsy[VGI(ring[i], ring[i])])) bad = 1;
            const int top = ring[h - 1];
            if (bad) {
                say(C, "Warning: Invalid rho at iteration %d\n", k);
            } else {
                const double gamma = Gsy[VGI(top, top)] / Gyy[VGI(top, top)];
                if (gamma <= 0 || !isfinite(gamma)) {
                    say(C, "Warning: Invalid gamma at iteration %d\n", k);
                } else {
                    double ds[64], dy[64], a[64], dg = 1.0;
                    for (int j = 0; j < h; ++j) ds[j] = dy[j] = 0.0;
                    for (int i = h - 1; i >= 0; --i) {
                        const int ri = ring[i];
                        const double rho = 1.0 / Gsy[VGI(ri, ri)];
                        double t = 0.0;
                        for (int j = 0; j < h; ++j) t = t + ds[j] * Gss[VGI(ri, ring[j])];
                        for (int j = 0; j < h; ++j) t = t + dy[j] * Gsy[VGI(ri, ring[j])];
                        t = t + dg * Gsg[ri];
                        a[i] = rho * t;
                        dy[i] = dy[i] - a[i];
                    }
                    for (int j = 0; j < h; ++j) {
                        ds[j] = ds[j] * gamma;
                        dy[j] = dy[j] * gamma;
                    }
                    dg = dg * gamma;
                    for (int i = 0; i < h; ++i) {
                        const int ri = ring[i];
                        const double rho = 1.0 / Gsy[VGI(ri, ri)];
                        double t = 0.0;
                        for (int j = 0; j < h; ++j) t = t + ds[j] * Gsy[VGI(ring[j], ri)];
                        for (int j = 0; j < h; ++j) t = t + dy[j] * Gyy[VGI(ri, ring[j])];
                        t = t + dg * Gyg[ri];
                        const double beta = rho * t;
                        ds[i] = ds[i] + (a[i] - beta);
                    }
                    for (int j = 0; j < h; ++j) {
                        cs[j] = -ds[j];
                        cy[j] = -dy[j];
                    }
                    cg = -dg;
                }
            }
        }
        double gd = 0.0;
        for (int j = 0; j < h; ++j) gd = gd + cs[j] * Gsg[ring[j]];
        for (int j = 0; j < h; ++j) gd = gd + cy[j] * Gyg[ring[j]];
        gd = gd + cg * gg;
        if (gd >= 0) {
            say(C, "Warning: Not a descent direction, using gradient\n");
            for (int j = 0; j < h; ++j) cs[j] = cy[j] = 0.0;
            cg = -1.0;
            gd = 0.0;
            for (int j = 0; j < h; ++j) gd = gd + cs[j] * Gsg[ring[j]];
            for (int j = 0; j < h; ++j) gd = gd + cy[j] * Gyg[ring[j]];
            gd = gd + cg * gg;
        }
        double cb[128];
        for (int j = 0; j < h; ++j) {
            B[j] = S[ring[j]];
            B[h + j] = Y[ring[j]];
            cb[j] = cs[j];
            cb[h + j] = cy[j];
        }
        vf_direction(h, B, cb, cg, g, n, d);

        /* commit at alpha: x_new, f, g_new, s, y into the free pair, and the dots */
        double alpha = 0.0;
        double fN = 0.0, sy = 0.0, yy = 0.0, ggN = 0.0, yg = 0.0, ggo = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            /* pass 0: the fused first trial at a0; pass 1: the commit at the accepted step */
            const double at = pass == 0 ? o->initial_step : alpha;
            if (pass == 1 && at == o->initial_step) break;
            trial_point(x, d, at, n, xn);
            fN = orc_f(o->obj, xn, n, ORC_CANON_VF);
            C->nf++;
            G(C, xn, gn);
            double* sk = S[free_pair];
            double* yk = Y[free_pair];
            for (int64_t i = 0; i < n; ++i) {
                sk[i] = xn[i] - x[i];
                yk[i] = gn[i] - g[i];
            }
            sy = orc_dot(sk, yk, n, ORC_CANON_VF);
            yy = orc_dot(yk, yk, n, ORC_CANON_VF);
            ggN = orc_dot(gn, gn, n, ORC_CANON_VF);
            yg = orc_dot(yk, gn, n, ORC_CANON_VF);
            ggo = orc_dot(gn, g, n, ORC_CANON_VF);
            for (int l = 0; l < 2 * h; ++l) {
                YB[l] = orc_dot(yk, B[l], n, ORC_CANON_VF);
                GB[l] = orc_dot(gn, B[l], n, ORC_CANON_VF);
            }
            if (pass == 0) {
                double dgn = 0.0;
                for (int j = 0; j < h; ++j) dgn = dgn + cs[j] * GB[j];
                for (int j = 0; j < h; ++j) dgn = dgn + cy[j] * GB[h + j];
                dgn = dgn + cg * ggo;
                vf_ls_t L = {C, x, d, gt, o->initial_step, fN, dgn, {0.0}, {0.0}};
                L.cand[0] = o->initial_step * o->backtracking_alpha;
                for (int j = 1; j < VF_NA; ++j) L.cand[j] = L.cand[j - 1] * o->backtracking_alpha;
                for (int j = 0; j < VF_NA; ++j) {
                    trial_point(x, d, L.cand[j], n, C->tmp);
                    L.fc[j] = orc_f(o->obj, C->tmp, n, ORC_CANON_VF);
                }
                alpha = vf_ls(&L, f_cur, gd);
                if (ntr < trace_cap) tr_alpha[ntr] = alpha;
                ntr++;
            }
        }
        double dgn = 0.0;
        for (int j = 0; j < h; ++j) dgn = dgn + cs[j] * GB[j];
        for (int j = 0; j < h; ++j) dgn = dgn + cy[j] * GB[h + j];
        dgn = dgn + cg * ggo;
        f_cur = fN;
        if (alpha < 1e-10) {
            say(C, "Warning: Line search failed at iteration %d\n", k);
            status = ORC_LS_FAILED;
            goto done;
        }
        if (sy > 0) {
            const int p = free_pair;
            double dS[64], dY[64];
            for (int q = 0; q < h; ++q) {
                const int rq = ring[q];
                double a = 0.0, b = 0.0;
                for (int j = 0; j < h; ++j) a = a + cs[j] * Gss[VGI(ring[j], rq)];
                for (int j = 0; j < h; ++j) a = a + cy[j] * Gsy[VGI(rq, ring[j])];
                dS[q] = a + cg * Gsg[rq];
                for (int j = 0; j < h; ++j) b = b + cs[j] * Gsy[VGI(ring[j], rq)];
                for (int j = 0; j < h; ++j) b = b + cy[j] * Gyy[VGI(ring[j], rq)];
                dY[q] = b + cg * Gyg[rq];
            }
            double dd = 0.0;
            for (int j = 0; j < h; ++j) dd = dd + cs[j] * dS[j];
            for (int j = 0; j < h; ++j) dd = dd + cy[j] * dY[j];
            dd = dd + cg * gd;
            for (int q = 0; q < h; ++q) {
                const int rq = ring[q];
                Gss[VGI(p, rq)] = Gss[VGI(rq, p)] = alpha * dS[q];
                Gsy[VGI(p, rq)] = alpha * dY[q];
                Gsy[VGI(rq, p)] = YB[q];
                Gyy[VGI(p, rq)] = Gyy[VGI(rq, p)] = YB[h + q];
                Gsg[rq] = GB[q];
                Gyg[rq] = GB[h + q];
            }
            Gss[VGI(p, p)] = (alpha * alpha) * dd;
            Gsy[VGI(p, p)] = sy;
            Gyy[VGI(p, p)] = yy;
            Gsg[p] = alpha * dgn;
            Gyg[p] = yg;
            if (h >= m) {
                const int oldest = ring[0];
                for (int i = 0; i + 1 < m; ++i) ring[i] = ring[i + 1];
                ring[m - 1] = p;
                free_pair = oldest;
            } else {
                ring[h++] = p;
                free_pair = h;
            }
        } else {
            say(C, "Warning: Skipping update, sy = %g\n", sy);
            for (int q = 0; q < h; ++q) {
                Gsg[ring[q]] = GB[q];
                Gyg[ring[q]] = GB[h + q];
            }
        }
        double* t = x;
        x = xn;
        xn = t;
        t = g;
        g = gn;
        gn = t;
        gg = ggN;
    }
    if (ntr < trace_cap) {
        tr_f[ntr] = f_cur;
        tr_gnorm[ntr] = sqrt(gg);
        tr_alpha[ntr] = NAN;
        orc_checksum(x, n, &tr_c1[ntr], &tr_c2[ntr]);
        tr_nf[ntr] = C->nf;
    }
    ntr++;
    say(C, "Maximum iterations reached\n");
done:
    if (x_out) memcpy(x_out, x, vb);
    if (res) {
        res->iters = k;
        res->status = status;
        res->ntrace = ntr;
        res->nf = C->nf;
        res->ng = C->ng;
    }
    free(x); free(g); free(d); free(xn); free(gn); free(gt); free(C->tmp);
    for (int i = 0; i <= m; ++i) {
        free(S[i]);
        free(Y[i]);
    }
    free(Gss); free(Gsy); free(Gyy); free(Gsg); free(Gyg);
    return 0;
}
#undef VGI

/* ------------------------------------------------------------------------------------------
 * The CUDA path (orc_opts.cuda = 1): LBFGS_CUDA of parallel-implementation/L-BFGS.cu:105-380 with
 * the host line searches of parallel-implementation/line_search.cpp (its own versions: floors,
 * a cached bisection Wolfe search, a safeguarded cubic). The line searches are pinned call for
 * call against that file compiled here (oracle/ref_cuda_ls.cpp); the loop's cuBLAS dots and axpys
 * cannot run here, so the loop is restated only ("parity unpinned": their summation order is
 * cuBLAS's; ORC_SEQ sums left to right, ORC_CANON in the product's order).
 * ---------------------------------------------------------------------------------------- */
static double pls_dot(ctx_t* c, const double* a, const double* b) { return orc_dot(a, b, c->n, c->o->mode); }

static double pls_backtracking(ctx_t* c, const double* x, const double* d, const double* g) {
    const orc_opts* o = c->o; /* parallel line_search.cpp:21-40 (the sequential search plus a floor) */
    double alpha = o->initial_step;
    for (;;) {
        double fx = F(c, x);
        trial_point(x, d, alpha, c->n, c->tmp);
        double ft = F(c, c->tmp);
        double gd = pls_dot(c, g, d);
        if (!(fx - ft < o->c1 * alpha * gd)) break;
        alpha *= o->backtracking_alpha;
        if (alpha < o->backtracking_tol) break;
    }
    if (alpha < 1e-4) return 0.5; /* :36-39 */
    return alpha;
}

/* :42-147: constants of its own (C1 1e-4, C2 0.9, tolerance 1e-10); bisection between alpha_lo
 * and alpha_hi, doubling while alpha_hi is unset; f values cached by alpha (a repeated alpha is
 * not evaluated again) */
#define PLS_CACHE 24
static double pls_backtracking_wolfe(ctx_t* c, const double* x, const double* d, const double* g, double* gnew) {
    const double C1 = 1e-4, C2 = 0.9, TOL = 1e-10;
    double alpha = 1.0;
    int iter = 0;
    const double f_current = F(c, x);
    const double gd = pls_dot(c, g, d);
    double ca[PLS_CACHE], cf[PLS_CACHE];
    int nc = 0;
    double alpha_lo = 0.0, alpha_hi = DBL_MAX;
    while (iter++ < 20) {
        int hit = -1;
        for (int j = 0; j < nc; ++j)
            if (ca[j] == alpha) hit = j;
        double f_new;
        trial_point(x, d, alpha, c->n, c->tmp); /* x_new (the cached point has the same bits) */
        if (hit >= 0) {
            f_new = cf[hit];
        } else {
            f_new = F(c, c->tmp);
            if (nc < PLS_CACHE) {
                ca[nc] = alpha;
                cf[nc++] = f_new;
            }
        }
        if (f_new <= f_current + C1 * alpha * gd) {
            G(c, c->tmp, gnew);
            const double gnd = pls_dot(c, gnew, d);
            if (gnd >= C2 * gd) break;
            alpha_lo = alpha;
        } else {
            alpha_hi = alpha;
        }
        if (alpha_hi < DBL_MAX)
            alpha = (alpha_lo + alpha_hi) / 2.0;
        else
            alpha = 2.0 * alpha_lo;
        if (alpha < TOL) break;
    }
    return alpha;
}

static double pls_interpolation(ctx_t* c, const double* x, const double* d, const double* g) {
    const orc_opts* o = c->o; /* :149-213 (the sequential search plus a floor after 20 trials) */
    const double f_x = F(c, x);
    const double gd = pls_dot(c, g, d);
    double alpha = o->initial_step, alpha_prev = 0.0, f_prev = f_x;
    int it = 0;
    while (it++ < 20) {
        trial_point(x, d, alpha, c->n, c->tmp);
        double f_new = F(c, c->tmp);
        if (f_new <= f_x + o->c1 * alpha * gd) return alpha;
        if (alpha < o->wolfe_interp_min) return o->wolfe_interp_min;
        if (alpha_prev > 0) {
            double delta = alpha - alpha_prev;
            if (fabs(delta) < 1e-10) {
                alpha *= 0.5;
            } else {
                double ga = (f_new - f_x - gd * alpha) / (alpha * alpha);
                alpha = cubic_interp(alpha_prev, alpha, f_prev, gd, f_new, ga);
                if (alpha < 0.1 * alpha_prev || alpha > 0.9 * alpha_prev) alpha = alpha_prev * 0.5;
            }
        } else {
            alpha = quad_interp(alpha, 0.0, f_new, gd, f_x);
            if (alpha < 0.1 * o->initial_step || alpha > 0.9 * o->initial_step) alpha = o->initial_step * 0.5;
        }
        alpha_prev = alpha;
        f_prev = f_new;
    }
    if (alpha < 1e-4) return 0.5; /* :209-212 */
    return alpha;
}

/* :216-275 safeCubicInterpolate: sorted endpoints, the midpoint whenever a step is not finite
 * or the cubic has no real minimiser, and the result kept 10 % inside the bracket */
static double pls_safe_cubic(double a0, double a1, double p0, double dp0, double p1, double dp1) {
    if (a0 > a1) {
        double t = a0; a0 = a1; a1 = t;
        t = p0; p0 = p1; p1 = t;
        t = dp0; dp0 = dp1; dp1 = t;
    }
    const double d1 = dp0 + dp1 - 3 * (p1 - p0) / (a1 - a0);
    if (isnan(d1) || isinf(d1)) return 0.5 * (a0 + a1);
    const double disc = d1 * d1 - dp0 * dp1;
    if (disc < 0) return 0.5 * (a0 + a1);
    const double d2 = copysign(sqrt(disc), a1 - a0);
    const double den = dp0 - dp1 + 2 * d2;
    if (fabs(den) < 1e-10) return 0.5 * (a0 + a1);
    const double r = a0 + (a1 - a0) * (dp0 + d2 - d1) / den;
    if (isnan(r) || isinf(r)) return 0.5 * (a0 + a1);
    const double lo = a0 + 0.1 * (a1 - a0), hi = a1 - 0.1 * (a1 - a0);
    const double mn = (r < hi) ? r : hi;   /* std::min(hi, r) */
    return (lo < mn) ? mn : lo;            /* std::max(lo, min) */
}

static double pls_wolfe(ctx_t* c, const double* x, const double* d, const double* g, double* gnew) {
    const orc_opts* o = c->o; /* :277-368 */
    const double f_x = F(c, x);
    const double gd = pls_dot(c, g, d);
    double alpha = o->initial_step;
    double alpha_lo = 0.0, alpha_hi = INFINITY, f_lo = f_x, dphi_lo = gd;
    for (int iter = 0; iter < 20; ++iter) {
        trial_point(x, d, alpha, c->n, c->tmp);
        double f_new = F(c, c->tmp);
        if (f_new > f_x + o->c1 * alpha * gd || (f_new >= f_lo && iter > 0)) {
            alpha_hi = alpha;
            alpha = pls_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new,
                                   (f_new - f_x - gd * alpha) / (alpha * alpha));
            continue;
        }
        G(c, c->tmp, gnew);
        double dphi_new = pls_dot(c, gnew, d);
        if (fabs(dphi_new) <= -o->c2 * gd) return alpha;
        if (dphi_new >= 0) {
            alpha_hi = alpha;
            alpha = pls_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        } else {
            alpha_lo = alpha;
            f_lo = f_new;
            dphi_lo = dphi_new;
            if (alpha_hi == INFINITY)
                alpha *= 2;
            else
                alpha = pls_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        }
        if (alpha < o->wolfe_interp_min) return o->wolfe_interp_min;
    }
    return alpha;
}

static double pls_run(ctx_t* c, int ls, const double* x, const double* d, const double* g, double* gnew) {
    switch (ls) {
        case ORC_LS_BACKTRACKING: return pls_backtracking(c, x, d, g);
        case ORC_LS_INTERPOLATION: return pls_interpolation(c, x, d, g);
        case ORC_LS_WOLFE: return pls_wolfe(c, x, d, g, gnew);
        default: return pls_backtracking_wolfe(c, x, d, g, gnew);
    }
}

int orc_cuda_line_search(const orc_opts* o, const double* x, const double* d, const double* g, double* alpha,
                         double* flog, int64_t flog_cap, int64_t* flog_n, uint64_t* glog, int64_t glog_cap,
                         int64_t* glog_n) {
    ctx_t C;
    memset(&C, 0, sizeof C);
    C.o = o;
    C.n = o->n;
    C.flog = flog;
    C.flog_cap = flog_cap;
    C.glog = glog;
    C.glog_cap = glog_cap;
    C.tmp = (double*)malloc(sizeof(double) * (size_t)o->n);
    double* gnew = (double*)malloc(sizeof(double) * (size_t)o->n);
    if (!C.tmp || !gnew) return -1;
    *alpha = pls_run(&C, o->ls, x, d, g, gnew);
    if (flog_n) *flog_n = C.flog_n;
    if (glog_n) *glog_n = C.glog_n;
    free(C.tmp);
    free(gnew);
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * The variant files (orc_opts.cuda = 2): the string-less LBFGS_CUDA of L-BFGS-Backtracking.cu,
 * -Interpolation.cu, -Wolfe.cu and -Backtracking_Wolfe.cu, the same loop as L-BFGS.cu around an
 * inline search of each file's own. Their searches get the current gradient (d_g); all but the
 * backtracking file take f(x) as f(x_host), the host copy of the LAST trial point the previous
 * search transferred (x0 at k = 0), and start f_prev / f_lo from f(x0) (initial_f) every time.
 * vs->fhost is that f, vs->f0 = f(x0). ok = the file's line_search_success. Parity unpinned: the
 * searches live in .cu files that cannot be built here.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    double f0, fhost;
} vstate_t;

static double vls_backtracking(ctx_t* c, const double* x, const double* d, double gd) {
    const double C1 = 1e-4, TOL = 1e-10; /* L-BFGS-Backtracking.cu:153-156 */
    const double fx = F(c, x);            /* :304-309, x_host copied from d_x */
    double step = 1.0;
    for (;;) { /* :311-340 */
        trial_point(x, d, step, c->n, c->tmp);
        const double ft = F(c, c->tmp);
        if (ft <= fx + C1 * step * gd) break;
        step *= 0.5;
        if (step < TOL) {
            step = 0.5;
            break;
        }
    }
    return step;
}

static double vls_interpolation(ctx_t* c, vstate_t* vs, const double* x, const double* d, double gd, int* ok) {
    const orc_opts* o = c->o; /* L-BFGS-Interpolation.cu:259-342 */
    const double f_x = vs->fhost;
    double alpha = o->initial_step, alpha_prev = 0.0, f_prev = vs->f0;
    *ok = 0;
    for (int iter = 0; iter < 20; ++iter) {
        trial_point(x, d, alpha, c->n, c->tmp);
        const double f_new = F(c, c->tmp);
        vs->fhost = f_new;
        if (f_new <= f_x + o->c1 * alpha * gd) {
            *ok = 1;
            break;
        }
        if (alpha < o->wolfe_interp_min) {
            alpha = o->wolfe_interp_min;
            break;
        }
        if (alpha_prev > 0) {
            const double delta = alpha - alpha_prev;
            if (fabs(delta) < 1e-10) {
                alpha *= 0.5;
            } else {
                const double ga = (f_new - f_x - gd * alpha) / (alpha * alpha);
                double next = cubic_interp(alpha_prev, alpha, f_prev, gd, f_new, ga);
                if (next < 0.1 * alpha_prev || next > 0.9 * alpha_prev) next = alpha_prev * 0.5;
                alpha = next;
            }
        } else {
            double next = quad_interp(alpha, 0.0, f_new, gd, f_x);
            if (next < 0.1 * o->initial_step || next > 0.9 * o->initial_step) next = o->initial_step * 0.5;
            alpha = next;
        }
        alpha_prev = alpha; /* :335, after the update */
        f_prev = f_new;
    }
    if (alpha < 1e-4) alpha = 0.5; /* :339-342 */
    return alpha;
}

static double vls_wolfe(ctx_t* c, vstate_t* vs, const double* x, const double* d, double gd, double* gnew, int* ok) {
    const orc_opts* o = c->o; /* L-BFGS-Wolfe.cu:259-349 */
    const double f_x = vs->fhost;
    double alpha = o->initial_step, alpha_lo = 0.0, alpha_hi = INFINITY, f_lo = vs->f0, dphi_lo = gd;
    *ok = 0;
    for (int iter = 0; iter < 20; ++iter) {
        trial_point(x, d, alpha, c->n, c->tmp);
        const double f_new = F(c, c->tmp);
        vs->fhost = f_new;
        if (f_new > f_x + o->c1 * alpha * gd || (f_new >= f_lo && iter > 0)) {
            alpha_hi = alpha;
            alpha = pls_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, (f_new - f_x - gd * alpha) / (alpha * alpha));
            continue;
        }
        G(c, c->tmp, gnew);
        const double dphi_new = pls_dot(c, gnew, d);
        if (fabs(dphi_new) <= -o->c2 * gd) {
            *ok = 1;
            break;
        }
        if (dphi_new >= 0) {
            alpha_hi = alpha;
            alpha = pls_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        } else {
            alpha_lo = alpha;
            f_lo = f_new;
            dphi_lo = dphi_new;
            if (alpha_hi == INFINITY)
                alpha *= 2;
            else
                alpha = pls_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        }
        if (alpha < o->wolfe_interp_min) {
            alpha = o->wolfe_interp_min;
            break;
        }
    }
    return alpha;
}

static double vls_backtracking_wolfe(ctx_t* c, vstate_t* vs, const double* x, const double* d, double gd,
                                     double* gnew, int* ok) {
    const double C1 = 1e-4, C2 = 0.9, TOL = 1e-10; /* L-BFGS-Backtracking_Wolfe.cu:261-264 */
    const double f_x = vs->fhost;
    double alpha = 1.0, alpha_lo = 0.0, alpha_hi = DBL_MAX;
    double ca[PLS_CACHE], cf[PLS_CACHE], cgd[PLS_CACHE]; /* cache / grad_cache by alpha */
    int cg[PLS_CACHE], nc = 0;
    *ok = 0;
    for (int iter = 0; iter < 20; ++iter) { /* :279-397 */
        int hit = -1;
        for (int j = 0; j < nc; ++j)
            if (ca[j] == alpha) hit = j;
        if (hit < 0) {
            trial_point(x, d, alpha, c->n, c->tmp);
            hit = nc++;
            ca[hit] = alpha;
            cf[hit] = F(c, c->tmp);
            cg[hit] = 0;
            vs->fhost = cf[hit];
        }
        if (cf[hit] <= f_x + C1 * alpha * gd) {
            if (!cg[hit]) { /* the point transferred again, its gradient evaluated and cached */
                trial_point(x, d, alpha, c->n, c->tmp);
                vs->fhost = cf[hit];
                G(c, c->tmp, gnew);
                cgd[hit] = pls_dot(c, gnew, d);
                cg[hit] = 1;
            }
            if (cgd[hit] >= C2 * gd) {
                *ok = 1;
                break;
            }
            alpha_lo = alpha;
        } else {
            alpha_hi = alpha;
        }
        if (alpha_hi < DBL_MAX)
            alpha = (alpha_lo + alpha_hi) / 2.0;
        else
            alpha = 2.0 * alpha_lo;
        if (alpha < TOL) {
            alpha = TOL;
            trial_point(x, d, alpha, c->n, c->tmp);
            vs->fhost = F(c, c->tmp);
            break;
        }
    }
    return alpha;
}

/* L-BFGS.cu:195-358. Trace entry k is the state the iteration prints after its step: f(x_{k+1})
 * ("Optimum value"), |g_{k+1}| ("norm_g"), alpha_k, the x_{k+1} checksums. */
static int orc_lbfgs_cuda(const orc_opts* o, const double* x0, double* x_out, double* tr_f, double* tr_gnorm,
                          double* tr_alpha, uint64_t* tr_c1, uint64_t* tr_c2, int64_t* tr_nf, int trace_cap,
                          ctx_t* C, orc_result* res) {
    const int64_t n = o->n;
    const int m = o->m, mode = o->mode;
    const size_t vb = sizeof(double) * (size_t)n;
    double *x = malloc(vb), *g = malloc(vb), *d = malloc(vb), *q = malloc(vb), *r = malloc(vb), *xn = malloc(vb),
           *gn = malloc(vb), *g0 = malloc(vb), *gt = malloc(vb);
    C->tmp = malloc(vb);
    double** S = calloc((size_t)m, sizeof(double*));
    double** Y = calloc((size_t)m, sizeof(double*));
    double* alpha = calloc((size_t)m, sizeof(double)); /* vector<double> alpha(m), rho(m): zeros */
    double* rho = calloc((size_t)m, sizeof(double));
    for (int i = 0; i < m; ++i) {
        S[i] = calloc((size_t)n, sizeof(double));
        Y[i] = calloc((size_t)n, sizeof(double));
    }
    say(C, "Starting\n"); /* :115 */
    memcpy(x, x0, vb);
    G(C, x0, g0); /* :199 - the host gradient, never updated: every line search gets it */
    memcpy(g, g0, vb);
    vstate_t vs;
    vs.f0 = vs.fhost = o->cuda == 2 ? F(C, x0) : 0.0; /* the variants' initial_f = f(x_host), :172-173 */
    int status = ORC_MAX_ITER, ntr = 0, k;
    int64_t skips = 0;
    for (k = 0; k < o->maxit; ++k) {
        if (k == 0) {
            for (int64_t i = 0; i < n; ++i) d[i] = -g[i]; /* :208 */
        } else {
            memcpy(q, g, vb); /* :212 */
            const int lo = k - m > 0 ? k - m : 0;
            for (int i = k - 1; i >= lo; --i) { /* :216-235 */
                const int sl = i % m;
                const double sy = orc_dot(S[sl], Y[sl], n, mode);
                if (sy <= 1e-10) { /* alpha[sl], rho[sl] keep their last values */
                    skips++;
                    continue;
                }
                rho[sl] = 1.0 / sy;
                const double sq = orc_dot(S[sl], q, n, mode);
                alpha[sl] = rho[sl] * sq;
                const double na = -alpha[sl];
                for (int64_t j = 0; j < n; ++j) q[j] = q[j] + na * Y[sl][j]; /* cublasDaxpy */
            }
            {
                const int last = (k - 1) % m; /* :237-262 */
                const double ys = orc_dot(S[last], Y[last], n, mode);
                const double yy = orc_dot(Y[last], Y[last], n, mode);
                const double gamma = (yy > 0 && ys > 1e-10) ? ys / yy : 1.0;
                for (int64_t j = 0; j < n; ++j) r[j] = q[j] * gamma; /* scaleByRho */
            }
            for (int i = lo; i < k; ++i) { /* :264-274 */
                const int sl = i % m;
                const double yr = orc_dot(Y[sl], r, n, mode);
                const double beta = rho[sl] * yr;
                const double diff = alpha[sl] - beta;
                for (int64_t j = 0; j < n; ++j) r[j] = r[j] + diff * S[sl][j];
            }
            for (int64_t j = 0; j < n; ++j) d[j] = -r[j]; /* :276 */
        }
        double step;
        if (o->cuda == 2) { /* a variant file's own search, on the current gradient */
            const double gd = pls_dot(C, g, d);
            int ok = 1;
            switch (o->ls) {
                case ORC_LS_BACKTRACKING: step = vls_backtracking(C, x, d, gd); break;
                case ORC_LS_INTERPOLATION: step = vls_interpolation(C, &vs, x, d, gd, &ok); break;
                case ORC_LS_WOLFE: step = vls_wolfe(C, &vs, x, d, gd, gt, &ok); break;
                default: step = vls_backtracking_wolfe(C, &vs, x, d, gd, gt, &ok); break;
            }
            say(C, "alpha: %g\n", step);
            if (o->ls == ORC_LS_BACKTRACKING) {
                if (step < 1e-4) /* L-BFGS-Backtracking.cu:345-348 */
                    say(C, "Warning: Line search resulted in very small step size at iteration %d\n", k);
            } else if (!ok && step < 1e-10) { /* e.g. L-BFGS-Wolfe.cu:353-366 */
                say(C, "Warning: Line search failed at iteration %d\n", k);
                status = ORC_LS_FAILED;
                goto done;
            }
        } else {
            step = pls_run(C, o->ls, x, d, g0, gt); /* :293, the stale gradient */
            if (step < 1e-10) { /* :295-306 */
                say(C, "Warning: Line search failed at iteration %d\n", k);
                status = ORC_LS_FAILED;
                goto done;
            }
            say(C, "alpha: %g\n", step); /* :308 */
        }
        for (int64_t j = 0; j < n; ++j) xn[j] = x[j] + step * d[j]; /* updateSolution :310 */
        G(C, xn, gn); /* :323 */
        {
            const int sl = k % m; /* updateVectors :332, unconditionally */
            for (int64_t j = 0; j < n; ++j) {
                S[sl][j] = xn[j] - x[j];
                Y[sl][j] = gn[j] - g[j];
            }
        }
        memcpy(x, xn, vb); /* :335-340 */
        memcpy(g, gn, vb);
        const double norm_g = sqrt(orc_dot(g, g, n, mode)); /* :342-345 */
        const double fv = F(C, xn);                          /* :348 */
        say(C, "Iteration %d: norm_g = %g\n", k, norm_g);
        say(C, "Optimum value: %g\n", fv);
        if (ntr < trace_cap) {
            tr_f[ntr] = fv;
            tr_gnorm[ntr] = norm_g;
            tr_alpha[ntr] = step;
            orc_checksum(x, n, &tr_c1[ntr], &tr_c2[ntr]);
            tr_nf[ntr] = C->nf;
        }
        ntr++;
        if (norm_g <= o->tol) { /* :353-357 */
            say(C, "Convergence achieved at iteration %d\n", k);
            status = ORC_CONVERGED;
            k++;
            goto done;
        }
    }
done:
    if (x_out) memcpy(x_out, x, vb);
    if (res) {
        res->iters = k;
        res->status = status;
        res->ntrace = ntr;
        res->nf = C->nf;
        res->ng = C->ng;
        res->skips = skips;
    }
    free(x); free(g); free(d); free(q); free(r); free(xn); free(gn); free(g0); free(gt); free(C->tmp);
    for (int i = 0; i < m; ++i) {
        free(S[i]);
        free(Y[i]);
    }
    free(S); free(Y); free(alpha); free(rho);
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * LBFGS — lbfgs.cpp:17-203.
 * ---------------------------------------------------------------------------------------- */
int orc_lbfgs(const orc_opts* o, const double* x0, double* x_out,
              double* tr_f, double* tr_gnorm, double* tr_alpha, uint64_t* tr_c1, uint64_t* tr_c2,
              int64_t* tr_nf, int trace_cap,
              double* flog, int64_t flog_cap, int64_t* flog_n,
              uint64_t* glog, int64_t glog_cap, int64_t* glog_n,
              char* msg, int msg_cap, orc_result* res) {
    const int64_t n = o->n;
    const int m = o->m;
    if (n < 1 || m < 1 || o->ls < 0 || o->ls > 3) return -1;
    ctx_t C;
    memset(&C, 0, sizeof C);
    C.o = o;
    C.n = n;
    C.flog = flog;
    C.flog_cap = flog_cap;
    C.glog = glog;
    C.glog_cap = glog_cap;
    C.msg = msg;
    C.msg_cap = msg_cap;
    if (msg && msg_cap > 0) msg[0] = 0;
    if (o->cuda) {
        int rc = orc_lbfgs_cuda(o, x0, x_out, tr_f, tr_gnorm, tr_alpha, tr_c1, tr_c2, tr_nf, trace_cap, &C, res);
        if (flog_n) *flog_n = C.flog_n;
        if (glog_n) *glog_n = C.glog_n;
        return rc;
    }
    if (o->vf) {
        if (m > 64) return -1;
        int rc = orc_lbfgs_vf(o, x0, x_out, tr_f, tr_gnorm, tr_alpha, tr_c1, tr_c2, tr_nf, trace_cap, &C, res);
        if (flog_n) *flog_n = C.flog_n;
        if (glog_n) *glog_n = C.glog_n;
        return rc;
    }

    size_t vb = sizeof(double) * (size_t)n;
    double* x = (double*)malloc(vb);
    double* g = (double*)malloc(vb);
    double* d = (double*)malloc(vb);
    double* q = (double*)malloc(vb);
    double* r = (double*)malloc(vb);
    double* xn = (double*)malloc(vb);
    double* gn = (double*)malloc(vb);
    C.tmp = (double*)malloc(vb);
    double* alpha_i = (double*)malloc(sizeof(double) * (size_t)m);
    /* history deque: hs[0] oldest .. hs[h-1] newest; storage pool of m+1 pairs */
    double** hs = (double**)malloc(sizeof(double*) * (size_t)(m + 1));
    double** hy = (double**)malloc(sizeof(double*) * (size_t)(m + 1));
    for (int i = 0; i <= m; ++i) {
        hs[i] = (double*)malloc(vb);
        hy[i] = (double*)malloc(vb);
    }
    int h = 0;

    memcpy(x, x0, vb);
    double f_current = F(&C, x0); /* :29 */
    G(&C, x, g);                  /* :30 */
    int status = ORC_MAX_ITER, ntr = 0, k;
    const int mode = o->mode;

    for (k = 0; k < o->maxit; ++k) {
        double gnorm = orc_norm(g, n, mode);
        if (ntr < trace_cap) {
            tr_f[ntr] = f_current;
            tr_gnorm[ntr] = gnorm;
            tr_alpha[ntr] = NAN;
            orc_checksum(x, n, &tr_c1[ntr], &tr_c2[ntr]);
            tr_nf[ntr] = C.nf;
        }
        if (o->verbose) printf("Iteration %d, f = %g, |grad| = %g\n", k, f_current, gnorm); /* :76-78 */
        if (gnorm < o->tol) {                                                               /* :80 */
            say(&C, "Converged!\n");
            status = ORC_CONVERGED;
            ntr++;
            goto done;
        }
        if (k == 0 || h == 0) { /* :87-91 */
            ORC_PAR(n)
            for (int64_t i = 0; i < n; ++i) d[i] = -g[i];
        } else { /* two-loop :94-143 */
            memcpy(q, g, vb);
            for (int i = h - 1; i >= 0; --i) {
                double rho = 1.0 / orc_dot(hy[i], hs[i], n, mode);
                if (!isfinite(rho)) {
                    say(&C, "Warning: Invalid rho at iteration %d\n", k);
                    ORC_PAR(n)
                    for (int64_t j = 0; j < n; ++j) d[j] = -g[j];
                    goto perform_line_search;
                }
                alpha_i[i] = rho * orc_dot(hs[i], q, n, mode);
                ORC_PAR(n)
                for (int64_t j = 0; j < n; ++j) q[j] -= alpha_i[i] * hy[i][j];
            }
            {
                double gamma = orc_dot(hs[h - 1], hy[h - 1], n, mode) / orc_dot(hy[h - 1], hy[h - 1], n, mode);
                if (gamma <= 0 || !isfinite(gamma)) {
                    say(&C, "Warning: Invalid gamma at iteration %d\n", k);
                    ORC_PAR(n)
                    for (int64_t j = 0; j < n; ++j) d[j] = -g[j];
                    goto perform_line_search;
                }
                ORC_PAR(n)
                for (int64_t i = 0; i < n; ++i) r[i] = q[i] * gamma;
            }
            for (int i = 0; i < h; ++i) {
                double rho = 1.0 / orc_dot(hy[i], hs[i], n, mode);
                double beta = rho * orc_dot(hy[i], r, n, mode);
                ORC_PAR(n)
                for (int64_t j = 0; j < n; ++j) r[j] += hs[i][j] * (alpha_i[i] - beta);
            }
            ORC_PAR(n)
            for (int64_t j = 0; j < n; ++j) d[j] = -r[j];
        }
    perform_line_search:; /* :146-156 */
        double gd = orc_dot(g, d, n, mode);
        if (gd >= 0) {
            say(&C, "Warning: Not a descent direction, using gradient\n");
            ORC_PAR(n)
            for (int64_t j = 0; j < n; ++j) d[j] = -g[j];
            gd = orc_dot(g, d, n, mode);
        }
        (void)gd;
        double alpha;
        switch (o->ls) {
            case ORC_LS_BACKTRACKING: alpha = ls_backtracking(&C, x, d, g); break;
            case ORC_LS_INTERPOLATION: alpha = ls_interpolation(&C, x, d, g); break;
            case ORC_LS_WOLFE: alpha = ls_wolfe(&C, x, d, g, gn); break;
            default: alpha = ls_backtracking_wolfe(&C, x, d, g, gn); break;
        }
        if (ntr < trace_cap) tr_alpha[ntr] = alpha;
        ntr++;
        trial_point(x, d, alpha, n, xn); /* :159 */
        f_current = F(&C, xn);           /* :160-161 */
        if (alpha < 1e-10) {             /* :164-168 */
            say(&C, "Warning: Line search failed at iteration %d\n", k);
            status = ORC_LS_FAILED;
            goto done;
        }
        G(&C, xn, gn); /* :171 */
        {
            /* :174-195 — the new pair is written to the spare pool slot hs[h] (h <= m) */
            double* sk = hs[h];
            double* yk = hy[h];
            ORC_PAR(n)
            for (int64_t i = 0; i < n; ++i) {
                sk[i] = xn[i] - x[i];
                yk[i] = gn[i] - g[i];
            }
            double sy = orc_dot(sk, yk, n, mode);
            if (sy > 0) {
                if (h >= m) { /* pop_front: rotate the oldest into the spare slot */
                    double* s0 = hs[0];
                    double* y0 = hy[0];
                    for (int i = 0; i < m; ++i) {
                        hs[i] = hs[i + 1];
                        hy[i] = hy[i + 1];
                    }
                    hs[m] = s0;
                    hy[m] = y0;
                } else {
                    h++;
                }
            } else {
                say(&C, "Warning: Skipping update, sy = %g\n", sy);
            }
        }
        { /* :197-198 */
            double* t = x;
            x = xn;
            xn = t;
            t = g;
            g = gn;
            gn = t;
        }
    }
    /* maximum iterations: final state entry */
    if (ntr < trace_cap) {
        tr_f[ntr] = f_current;
        tr_gnorm[ntr] = orc_norm(g, n, mode);
        tr_alpha[ntr] = NAN;
        orc_checksum(x, n, &tr_c1[ntr], &tr_c2[ntr]);
        tr_nf[ntr] = C.nf;
    }
    ntr++;
    say(&C, "Maximum iterations reached\n");

done:
    if (x_out) memcpy(x_out, x, vb);
    if (res) {
        res->iters = k;
        res->status = status;
        res->ntrace = ntr;
        res->nf = C.nf;
        res->ng = C.ng;
    }
    if (flog_n) *flog_n = C.flog_n;
    if (glog_n) *glog_n = C.glog_n;
    free(x); free(g); free(d); free(q); free(r); free(xn); free(gn); free(C.tmp); free(alpha_i);
    for (int i = 0; i <= m; ++i) {
        free(hs[i]);
        free(hy[i]);
    }
    free(hs);
    free(hy);
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * Two-loop recursion alone (lbfgs.cpp:94-143) for a given history S[0..h-1] (oldest first),
 * used to check the device two-loop primitive. Returns g.d.
 * ---------------------------------------------------------------------------------------- */
double orc_twoloop(const double* g, const double* const* S, const double* const* Y, int h,
                   int64_t n, int mode, double* d) {
    double* q = (double*)malloc(sizeof(double) * (size_t)n);
    double* r = (double*)malloc(sizeof(double) * (size_t)n);
    double* al = (double*)malloc(sizeof(double) * (size_t)h);
    memcpy(q, g, sizeof(double) * (size_t)n);
    for (int i = h - 1; i >= 0; --i) {
        double rho = 1.0 / orc_dot(Y[i], S[i], n, mode);
        al[i] = rho * orc_dot(S[i], q, n, mode);
        for (int64_t j = 0; j < n; ++j) q[j] -= al[i] * Y[i][j];
    }
    double gamma = orc_dot(S[h - 1], Y[h - 1], n, mode) / orc_dot(Y[h - 1], Y[h - 1], n, mode);
    for (int64_t i = 0; i < n; ++i) r[i] = q[i] * gamma;
    for (int i = 0; i < h; ++i) {
        double rho = 1.0 / orc_dot(Y[i], S[i], n, mode);
        double beta = rho * orc_dot(Y[i], r, n, mode);
        for (int64_t j = 0; j < n; ++j) r[j] += S[i][j] * (al[i] - beta);
    }
    for (int64_t j = 0; j < n; ++j) d[j] = -r[j];
    double gd = orc_dot(g, d, n, mode);
    free(q);
    free(r);
    free(al);
    return gd;
}
