/* lbfgs_driver.c — C host driver of the MI355X L-BFGS solver (public ABI: include/lbfgs_hip.h).
 *
 * The control flow is the reference's LBFGS() (sequential-implementation/lbfgs.cpp:17-203) and
 * its line searches (line_search.cpp:8-189), restated over scalars only: every n-vector lives
 * on the GPU and every vector operation is a fused device pass (lbfgs_kernels.hip). The host
 * sees, per iteration, one 512-byte read-back of the commit's reductions (g.d, f, s.y, y.y,
 * |g|^2, s.g, g.d_phi), plus one per extra line-search trial.
 *
 * Per-iteration device schedule (h stored pairs, reference line numbers):
 *   [P0]  s_{h-1}.g         fused into the previous commit (SG), or lbk_dot if that pair
 *                           was not pushed                                     (:133)
 *   h-1 x k_axpy_dot        q -= alpha_{i+1} y_{i+1};  s_i.q                    (:124-138)
 *   k_mid                   r = (q - alpha_0 y_0) gamma;  y_0.r                 (:141-154,:160)
 *   h-1 x k_axpy2_dot       r += s_i (alpha_i - beta_i);  y_{i+1}.r             (:157-165)
 *   k_commit (TWOLOOP)      d = -(r + s(alpha-beta)), g.d, x+a0 d, f, grad, s, y, dots
 *                           — the last second-loop pass, the first line-search trial at
 *                           a0 = INITIAL_STEP_SIZE and the commit, in one pass  (:163-198)
 * If the line search accepts a0 (the common case) the iteration is complete; otherwise d is
 * materialised (k_last), the remaining trials run as k_trial passes and the commit is redone
 * at the accepted step. Results are bit-identical to running the reference's steps
 * separately in the canonical reduction order (oracle/lbfgs_oracle.c, ORC_CANON).
 */
#define _POSIX_C_SOURCE 199309L
#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lbfgs_device.h"
#include "lbfgs_hip.h"

/* roctx ranges (SURVEY §5 tracing): "lbfgs iteration" around every iteration and "line search"
 * around its trials, visible under rocprofv3 --marker-trace; no-ops without a tool attached.
 * The product build defines LBFGS_ROCTX (cuda-lbfgs_amd/Makefile); other host builds of this
 * file (the sanitizer job) compile them out. */
#ifdef LBFGS_ROCTX
struct hsa_agent_s; /* named in roctx.h's prototypes (C: declare before use) */
struct ihipStream_t;
#include <rocprofiler-sdk-roctx/roctx.h>
#define TRACE_PUSH(name) roctxRangePushA(name)
#define TRACE_POP() roctxRangePop()
#else
#define TRACE_PUSH(name) ((void)0)
#define TRACE_POP() ((void)0)
#endif

#define MMAX 64

/* result slots */
#define SLOT_INIT 0
#define SLOT_COMMIT0 1 /* commits alternate 1 / 2 so SG survives into the next iteration */
#define SLOT_P0 3
#define SLOT_A0 4 /* + i  : s_i . q          */
#define SLOT_B0(m) (4 + (m)) /* + i : y_i . r   */
#define SLOT_LAST(m) (4 + 2 * (m))
#define SLOT_TRIAL(m) (5 + 2 * (m))
#define SLOT_MISC(m) (6 + 2 * (m))
#define REF(slot, comp) ((slot) * LBK_KMAX + (comp))
#define D_VF 3 /* direction as a combination of the basis (vector-free mode) */

struct lbfgs_ctx {
    lbk_ctx* dev;
    const lbk_geo* geo;
    int64_t n;
    int m;
    /* device vectors */
    double *x, *g, *xn, *gn, *d, *q, *r, *gt;
    const double* rc;   /* the r the last two-loop pass wrote */
    double* S[MMAX + 1];
    double* Y[MMAX + 1];
    /* history: ring[0] oldest .. ring[h-1] newest, indices into the m+1 pair pool */
    int h, ring[MMAX + 1], free_pair;
    double sy[MMAX + 1], yy[MMAX + 1];
    /* solver state */
    int inited, obj, ls, k, status, finished;
    lbfgs_constants K;
    double tol;
    unsigned flags;
    double f_cur, gg;
    int sg_valid, sg_ref;
    lbfgs_host_fn cb;
    /* host-callback objective (LBFGS_OBJ_HOST), pinned buffers: hx the trial point z, hxx the
     * iterate x (reference call order only), hg[2] the gradient double buffer (a callback fills
     * one while the other's upload may still be in flight) */
    double *hx, *hxx, *hg[2];
    int hg_cur;
    int hz_valid, hz_pending; /* hx holds (or is receiving) z = x + hz_alpha d of this iteration */
    double hz_alpha;
    int hxx_valid, hxx_pending;
    int hf_valid; /* f(z) at hf_alpha, this iteration */
    double hf_alpha, hf_val;
    int refcalls; /* LBFGS_FLAG_REFERENCE_CALLS */
    int dense_set; /* lbfgs_set_dense_quadratic called */
    int64_t cb_f, cb_g;
    /* per-iteration working state */
    int dmode, d_ready;
    double rho_last, a0;
    int ref_b_last, ref_a_last, s_last_pair;
    int spec_valid;
    double spec_f, spec_dphi, spec_tot[LBK_KMAX];
    int gt_valid;
    double gt_alpha;
    int unfused; /* LBFGS_FLAG_UNFUSED */
    /* batched line-search trials (LBFGS_BATCH, default on): the first commit also reduces f at
     * the backtracking search's next step; a trial pass evaluates the next LBK_TRIALS_NC steps of
     * a halving chain, or f and g.d together for the Wolfe searches; d stays unmaterialised for
     * the first two trial passes and the commit */
    int batch;
    int cand_valid;
    double cand_alpha, cand_f;
    int tc_n, tc_dphi_ok;
    double tc_a[LBK_TRIALS_NC], tc_f[LBK_TRIALS_NC], tc_dphi;
    int trial_passes;
    /* small n: the device-resident line search (lbk_search_dev) commits at the step it finds into
     * this slot (-1: no commit requested); committed: it did, this iteration; recommit_a0: a
     * launch that timed out may have left the first commit's outputs partly rewritten, so the
     * commit is repeated even at the first trial's step */
    int search_cslot, search_committed, recommit_a0;
    int64_t search_launches, search_commits; /* since solver init (lbfgs_search_stats) */
    /* vector-free mode (LBFGS_FLAG_VECTOR_FREE): Gram matrix over the pair pool, indexed by
     * pool slot (P = m + 1): Gss[p][q] = s_p.s_q, Gsy[p][q] = s_p.y_q, Gyy[p][q] = y_p.y_q,
     * Gsg[p] = s_p.g, Gyg[p] = y_p.g (g = current gradient; |g|^2 is gg) */
    int vf;
    double *Gss, *Gsy, *Gyy, *Gsg, *Gyg;
    int vf_h;                            /* basis size of this iteration's direction */
    const double* vf_S[MMAX];            /* basis, ring order */
    const double* vf_Y[MMAX];
    double vf_cs[MMAX], vf_cy[MMAX], vf_cg; /* d = sum cs s + sum cy y + cg g */
    double vf_tot[LBK_KW], vf_spec[LBK_KW];
    int vf_hb;
    /* f at the backtracking candidates a0 beta, a0 beta^2, reduced by the first commit pass */
    double vf_cand[LBK_VF_NA], vf_cand_f[LBK_VF_NA];
    int vf_cand_valid;
    /* speculative next iteration (small n, cooperative form): the launch of
     * iteration sp_k queued behind iteration sp_k - 1's before the host has read that one's
     * results, with the arguments the host will pass if the first trial is taken and the pair
     * stored (the kernel checks exactly that, see lbk_spec) */
    int spec_on;                  /* LBFGS_SPEC (default 1) */
    int steps_left;               /* iterations still to run in this lbfgs_solver_step call */
    unsigned long long cur_epoch; /* this iteration's cooperative launch (0: none) */
    int cur_spec;                 /* ... which was a speculative one, adopted */
    double cur_rho, cur_gamma;    /* the host's rho of the newest pair and gamma, this iteration */
    int cur_p0;
    int sp_pend, sp_k, sp_h, sp_free, sp_p0, sp_cslot, sp_hostgo;
    double sp_alpha; /* the step the queued launch assumes iteration sp_k - 1 commits */
    int sp_ring[MMAX + 1];
    double *sp_x, *sp_xn, *sp_g, *sp_gn;
    double sp_rho[MMAX];
    unsigned long long sp_epoch;
    int64_t sp_adopted, sp_dropped;
    /* counters */
    int64_t trials_f, trials_fg, commits, passes;
    int h_min, h_max; /* pairs stored at the top of the iterations of the current call */
    /* LBFGS_FLAG_CUDA_COMPAT: the CUDA path's per-ring-slot alpha and rho (kept across iterations
     * as L-BFGS.cu's vector<double> alpha(m), rho(m)), its stale line-search gradient g0 */
    int cuda;          /* 1: LBFGS_FLAG_CUDA_COMPAT (L-BFGS.cu), 2: with LBFGS_FLAG_CUDA_VARIANT */
    double cv_f0;      /* the variants' initial_f = f(x0) */
    double cv_fhost;   /* f at their host copy x_host: the last trial point a search transferred */
    double cu_alpha[MMAX], cu_rho[MMAX];
    double* g0c;
    /* messages / trace */
    char* msg;
    int msg_len, msg_cap;
    double *tr_f, *tr_gn, *tr_a;
    uint64_t *tr_c1, *tr_c2;
    int tr_len, tr_cap;
    char err[256];
};

/* ------------------------------------------------------------------------------------------ */
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void say(lbfgs_ctx* c, const char* fmt, ...) {
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    int k = vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (k < 0) return;
    if (!(c->flags & LBFGS_FLAG_QUIET)) {
        fputs(buf, stdout);
        fflush(stdout);
    }
    if (c->msg_len + k + 1 > c->msg_cap) {
        int cap = c->msg_cap ? c->msg_cap * 2 : 4096;
        while (cap < c->msg_len + k + 1) cap *= 2;
        char* p = (char*)realloc(c->msg, (size_t)cap);
        if (!p) return;
        c->msg = p;
        c->msg_cap = cap;
    }
    memcpy(c->msg + c->msg_len, buf, (size_t)k);
    c->msg_len += k;
    c->msg[c->msg_len] = 0;
}

static int dev_err(lbfgs_ctx* c, int rc) {
    if (rc < 0) snprintf(c->err, sizeof c->err, "%s", lbk_last_error(c->dev));
    return rc < -6 ? LBFGS_ERR_HIP : rc;
}
#define DEV(call)                                 \
    do {                                          \
        int rc_ = (call);                         \
        if (rc_ != 0) return dev_err(c, rc_);     \
        c->passes++;                              \
    } while (0)
#define DEVNC(call)                               \
    do {                                          \
        int rc_ = (call);                         \
        if (rc_ != 0) return dev_err(c, rc_);     \
    } while (0)

static int trace_push(lbfgs_ctx* c, double f, double gn, int with_ck) {
    if (!(c->flags & LBFGS_FLAG_TRACE)) return 0;
    if (c->tr_len == c->tr_cap) {
        int cap = c->tr_cap ? 2 * c->tr_cap : 1024;
        double* a = (double*)realloc(c->tr_f, sizeof(double) * cap);
        if (a) c->tr_f = a;
        a = (double*)realloc(c->tr_gn, sizeof(double) * cap);
        if (a) c->tr_gn = a;
        a = (double*)realloc(c->tr_a, sizeof(double) * cap);
        if (a) c->tr_a = a;
        uint64_t* u = (uint64_t*)realloc(c->tr_c1, sizeof(uint64_t) * cap);
        if (u) c->tr_c1 = u;
        u = (uint64_t*)realloc(c->tr_c2, sizeof(uint64_t) * cap);
        if (u) c->tr_c2 = u;
        if (!c->tr_f || !c->tr_gn || !c->tr_a || !c->tr_c1 || !c->tr_c2) return LBFGS_ERR_NOMEM;
        c->tr_cap = cap;
    }
    int i = c->tr_len++;
    c->tr_f[i] = f;
    c->tr_gn[i] = gn;
    c->tr_a[i] = NAN;
    c->tr_c1[i] = c->tr_c2[i] = 0;
    if (with_ck) DEVNC(lbk_checksum(c->dev, c->x, &c->tr_c1[i], &c->tr_c2[i]));
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
void lbfgs_constants_default(lbfgs_constants* k) { /* sequential-implementation/config.h:5-17 */
    k->c1 = 1e-4;
    k->c2 = 0.9;
    k->initial_step = 1.0;
    k->backtracking_alpha = 0.5;
    k->backtracking_tol = 1e-8;
    k->wolfe_interp_min = 1e-10;
    k->wolfe_interp_max = 10.0;
}

void lbfgs_constants_cuda(lbfgs_constants* k) { /* parallel-implementation/constants.h:5-17 */
    lbfgs_constants_default(k);
    k->c2 = 0.7;
}

#ifndef LBFGS_SRC_HASH
#define LBFGS_SRC_HASH "unknown"
#endif
int lbfgs_spec_stats(const lbfgs_ctx* c, int64_t* adopted, int64_t* dropped) {
    if (!c) return LBFGS_ERR_BAD_ARG;
    if (adopted) *adopted = c->sp_adopted;
    if (dropped) *dropped = c->sp_dropped;
    return 0;
}

int lbfgs_search_stats(const lbfgs_ctx* c, int64_t* launches, int64_t* commits) {
    if (!c) return LBFGS_ERR_BAD_ARG;
    if (launches) *launches = c->search_launches;
    if (commits) *commits = c->search_commits;
    return 0;
}

#ifndef LBFGS_ARCH
#define LBFGS_ARCH "unknown"
#endif
const char* lbfgs_build_info(void) {
    return "src=" LBFGS_SRC_HASH " built=" __DATE__ " " __TIME__ " arch=" LBFGS_ARCH;
}

int lbfgs_unique_id(void* out128) { return lbk_unique_id(out128) == 0 ? 0 : LBFGS_ERR_RCCL; }

int lbfgs_device_count(void) { return lbk_device_count(); }

static void free_vectors(lbfgs_ctx* c) {
    double** v[] = {&c->x, &c->g, &c->xn, &c->gn, &c->d, &c->q, &c->r, &c->gt, &c->g0c};
    for (size_t i = 0; i < sizeof v / sizeof v[0]; ++i) {
        lbk_vec_free(c->dev, *v[i]);
        *v[i] = NULL;
    }
    for (int i = 0; i <= MMAX; ++i) {
        lbk_vec_free(c->dev, c->S[i]);
        lbk_vec_free(c->dev, c->Y[i]);
        c->S[i] = c->Y[i] = NULL;
    }
}

struct lbfgs_host_group {
    lbk_group* g;
    int world;
};

int lbfgs_host_group_create(lbfgs_host_group** out, int world) {
    if (!out || world < 1 || world > 8 || (8 % world) != 0) return LBFGS_ERR_BAD_ARG;
    lbfgs_host_group* h = (lbfgs_host_group*)calloc(1, sizeof *h);
    if (!h) return LBFGS_ERR_NOMEM;
    h->g = lbk_group_create(world);
    h->world = world;
    if (!h->g) {
        free(h);
        return LBFGS_ERR_NOMEM;
    }
    *out = h;
    return 0;
}

void lbfgs_host_group_destroy(lbfgs_host_group* h) {
    if (!h) return;
    lbk_group_destroy(h->g);
    free(h);
}

static int ctx_create(lbfgs_ctx** out, int64_t n, int m, int device, int rank, int world,
                      const void* unique_id, lbk_group* grp) {
    if (!out) return LBFGS_ERR_BAD_ARG;
    *out = NULL;
    if (n < 1 || m < 1 || m > MMAX || world < 1 || (8 % world) != 0 || rank < 0 || rank >= world)
        return LBFGS_ERR_BAD_ARG;
    lbfgs_ctx* c = (lbfgs_ctx*)calloc(1, sizeof(lbfgs_ctx));
    if (!c) return LBFGS_ERR_NOMEM;
    c->n = n;
    c->m = m;
    int rc = lbk_create(&c->dev, device, n, rank, world, unique_id, grp);
    if (rc != 0) {
        if (c->dev) {
            snprintf(c->err, sizeof c->err, "%s", lbk_last_error(c->dev));
            fprintf(stderr, "lbfgs_ctx_create: %s\n", c->err);
            lbk_destroy(c->dev);
        }
        free(c);
        return rc == -3 ? LBFGS_ERR_RCCL : rc == -1 ? LBFGS_ERR_BAD_ARG : LBFGS_ERR_HIP;
    }
    c->geo = lbk_geometry(c->dev);
    double** v[] = {&c->x, &c->g, &c->xn, &c->gn, &c->d, &c->q, &c->r, &c->gt};
    int ok = 1;
    for (size_t i = 0; i < sizeof v / sizeof v[0]; ++i) ok &= (*v[i] = lbk_vec_alloc(c->dev)) != NULL;
    for (int i = 0; i <= m; ++i) {
        ok &= (c->S[i] = lbk_vec_alloc(c->dev)) != NULL;
        ok &= (c->Y[i] = lbk_vec_alloc(c->dev)) != NULL;
    }
    if (!ok) {
        fprintf(stderr, "lbfgs_ctx_create: %s\n", lbk_last_error(c->dev));
        free_vectors(c);
        lbk_destroy(c->dev);
        free(c);
        return LBFGS_ERR_NOMEM;
    }
    lbk_sync(c->dev);
    *out = c;
    return 0;
}

int lbfgs_ctx_create_sharded(lbfgs_ctx** out, int64_t n, int m, int device, int rank, int world,
                             const void* unique_id) {
    return ctx_create(out, n, m, device, rank, world, unique_id, NULL);
}

int lbfgs_ctx_create_emulated(lbfgs_ctx** out, int64_t n, int m, int device, int rank,
                              lbfgs_host_group* grp) {
    if (!grp) return LBFGS_ERR_BAD_ARG;
    return ctx_create(out, n, m, device, rank, grp->world, NULL, grp->g);
}

int lbfgs_ctx_create(lbfgs_ctx** out, int64_t n, int m, int device) {
    return ctx_create(out, n, m, device, 0, 1, NULL, NULL);
}

void lbfgs_ctx_destroy(lbfgs_ctx* c) {
    if (!c) return;
    free_vectors(c);
    lbk_destroy(c->dev);
    lbk_host_free(c->hx);
    lbk_host_free(c->hxx);
    lbk_host_free(c->hg[0]);
    lbk_host_free(c->hg[1]);
    free(c->msg);
    free(c->tr_f);
    free(c->tr_gn);
    free(c->tr_a);
    free(c->tr_c1);
    free(c->tr_c2);
    free(c->Gss);
    free(c->Gsy);
    free(c->Gyy);
    free(c->Gsg);
    free(c->Gyg);
    free(c);
}

const char* lbfgs_last_error(const lbfgs_ctx* c) { return c ? c->err : "null context"; }

int lbfgs_shard_range(int64_t n, int rank, int world, int64_t* elem_lo, int64_t* n_loc) {
    lbk_geo g;
    if (lbk_geometry_plan(n, rank, world, &g) != 0) return LBFGS_ERR_BAD_ARG;
    if (elem_lo) *elem_lo = g.elem_lo;
    if (n_loc) *n_loc = g.n_loc;
    return 0;
}

int lbfgs_local_range(const lbfgs_ctx* c, int64_t* elem_lo, int64_t* n_loc) {
    if (!c) return LBFGS_ERR_BAD_ARG;
    if (elem_lo) *elem_lo = c->geo->elem_lo;
    if (n_loc) *n_loc = c->geo->n_loc;
    return 0;
}

int lbfgs_sync(lbfgs_ctx* c) { return lbk_sync(c->dev) == 0 ? 0 : LBFGS_ERR_HIP; }

int lbfgs_peer_handle(lbfgs_ctx* c, void* out) {
    if (!c || !out || lbk_peer_handle(c->dev, out) != 0) return LBFGS_ERR_BAD_ARG;
    return 0;
}

int lbfgs_peer_connect(lbfgs_ctx* c, const void* handles) {
    if (!c || !handles || c->geo->world <= 1) return LBFGS_ERR_BAD_ARG;
    const int rc = lbk_peer_connect(c->dev, handles);
    if (rc != 0) {
        snprintf(c->err, sizeof c->err, "%s", lbk_last_error(c->dev));
        return rc == -1 ? LBFGS_ERR_BAD_ARG : rc == -3 ? LBFGS_ERR_RCCL : LBFGS_ERR_HIP;
    }
    return 0;
}

int lbfgs_peer_enable(lbfgs_ctx* c, int on) {
    if (!c || c->geo->world <= 1) return LBFGS_ERR_BAD_ARG;
    return lbk_peer_enable(c->dev, on) == 0 ? 0 : LBFGS_ERR_STATE;
}

int lbfgs_rccl_attach(lbfgs_ctx* c, const void* unique_id) {
    if (!c || !unique_id || c->geo->world <= 1) return LBFGS_ERR_BAD_ARG;
    const int rc = lbk_rccl_attach(c->dev, unique_id);
    if (rc != 0) {
        snprintf(c->err, sizeof c->err, "%s", lbk_last_error(c->dev));
        return rc == -1 ? LBFGS_ERR_BAD_ARG : rc == -3 ? LBFGS_ERR_RCCL : LBFGS_ERR_HIP;
    }
    return 0;
}

int lbfgs_set_dense_quadratic(lbfgs_ctx* c, const double* A, const double* b) {
    if (!c || !A || !b || c->geo->world != 1) return LBFGS_ERR_BAD_ARG;
    const int rc = lbk_dense_set(c->dev, A, b);
    if (rc != 0) {
        snprintf(c->err, sizeof c->err, "%s", lbk_last_error(c->dev));
        return rc == -1 ? LBFGS_ERR_BAD_ARG : LBFGS_ERR_HIP;
    }
    c->inited = 0;
    c->dense_set = 1;
    return 0;
}

int lbfgs_exchange_backend(const lbfgs_ctx* c) { return c ? lbk_exchange_backend(c->dev) : LBFGS_ERR_BAD_ARG; }
int lbfgs_exchange_fold(const lbfgs_ctx* c) { return c ? lbk_exchange_fold(c->dev) : LBFGS_ERR_BAD_ARG; }

int lbfgs_exchange_latency(lbfgs_ctx* c, int backend, int components, int iters, double* us) {
    if (!c || !us) return LBFGS_ERR_BAD_ARG;
    const int rc = lbk_exchange_bench(c->dev, backend, components, iters, us);
    if (rc == 0) return 0;
    snprintf(c->err, sizeof c->err, "%s", lbk_last_error(c->dev));
    return rc == -1 ? LBFGS_ERR_BAD_ARG : rc == -5 ? LBFGS_ERR_STATE : rc == -3 ? LBFGS_ERR_RCCL : LBFGS_ERR_HIP;
}

int lbfgs_cu_partition(const lbfgs_ctx* c) { return c ? lbk_cu_partition(c->dev) : LBFGS_ERR_BAD_ARG; }

int lbfgs_vector_fallbacks(const lbfgs_ctx* c) { return c ? lbk_vec_fallbacks(c->dev) : LBFGS_ERR_BAD_ARG; }

int lbfgs_vector_pool(const lbfgs_ctx* c, int* pooled, double* held_gb) {
    return c ? lbk_vec_pool_stats(c->dev, pooled, held_gb) : LBFGS_ERR_BAD_ARG;
}

int lbfgs_wait_stats(const lbfgs_ctx* c, double* slept_s, uint64_t* waits, int* adaptive) {
    if (!c) return LBFGS_ERR_BAD_ARG;
    unsigned long long w = 0;
    const int rc = lbk_wait_stats(c->dev, slept_s, &w, adaptive);
    if (waits) *waits = (uint64_t)w;
    return rc;
}

int lbfgs_coop_info(const lbfgs_ctx* c, int* coop_max, int* search_max, int* fallbacks) {
    return c ? lbk_coop_info(c->dev, coop_max, search_max, fallbacks) : LBFGS_ERR_BAD_ARG;
}

int lbfgs_stream_probe(lbfgs_ctx* c, int launches, double* us, double* bytes) {
    /* the work vector holds a copy of y_0 (random doubles, as the passes' q): a zero-filled one
     * streamed ~3 % faster in the same process (profiles/r06/gap/), which overstated the box */
    return lbfgs_stream_probe_variant(c, 16, launches, us, bytes);
}

int lbfgs_stream_probe_variant(lbfgs_ctx* c, int variant, int launches, double* us, double* bytes) {
    if (!c || !us || launches < 1 || variant < 0 || (variant & 7) > 6 || variant > 31) return LBFGS_ERR_BAD_ARG;
    if (!c->inited) return LBFGS_ERR_STATE;
    /* + 8: the work vector is the solver's own q (variants 0-5), which the next iteration's first
     * two-loop pass rewrites from g before anything reads it (gap analysis: the same buffer as the
     * in-solve passes) */
    const int own_q = (variant & 8) != 0 && (variant & 7) <= 5;
    const int fill = (variant & 16) != 0; /* + 16: the scratch vector starts as a copy of y_0, not zeros */
    variant &= 7;
    /* the written operand is a scratch vector, not the solver's q: nothing of the solve is touched
     * (q - 0 * y is q only while y is finite) */
    double* scratch = lbk_vec_alloc(c->dev);
    if (!scratch) return dev_err(c, -2);
    double* outs[4] = {NULL, NULL, NULL, NULL}; /* variant 6: the commit's four written vectors */
    int rc = 0;
    for (int k = 0; variant == 6 && k < 4 && rc == 0; ++k)
        if (!(outs[k] = lbk_vec_alloc(c->dev))) rc = -2;
    if (rc == 0 && fill && !own_q) rc = lbk_copy(c->dev, scratch, c->Y[0]);
    if (rc == 0)
        rc = lbk_stream_probe(c->dev, own_q ? c->q : scratch, (const double* const*)c->Y, (const double* const*)c->S,
                              c->m + 1, launches, us, variant, outs);
    for (int k = 0; k < 4; ++k) lbk_vec_free(c->dev, outs[k]);
    lbk_vec_free(c->dev, scratch);
    if (rc != 0) return dev_err(c, rc);
    if (bytes) *bytes = (variant == 6 ? 64.0 : 32.0) * (double)c->geo->n_loc;
    return 0;
}

/* the context's vectors in allocation order (lbfgs_ctx_create): x, g, xn, gn, d, q, r, gt, then
 * S_0, Y_0, S_1, Y_1, ...; index 8 + 2 (m + 1) = a scratch vector allocated for the call */
static double* vec_by_index(lbfgs_ctx* c, int k, double* scratch) {
    double* w[] = {c->x, c->g, c->xn, c->gn, c->d, c->q, c->r, c->gt};
    if (k >= 0 && k < 8) return w[k];
    k -= 8;
    if (k >= 0 && k < 2 * (c->m + 1)) return (k & 1) ? c->Y[k >> 1] : c->S[k >> 1];
    return k == 2 * (c->m + 1) ? scratch : NULL;
}

int lbfgs_vector_address(lbfgs_ctx* c, int k, uint64_t* addr) {
    if (!c || !addr) return LBFGS_ERR_BAD_ARG;
    double* v = vec_by_index(c, k, NULL);
    if (!v) return LBFGS_ERR_BAD_ARG;
    *addr = (uint64_t)(uintptr_t)v;
    return 0;
}

int lbfgs_stream_probe_vectors(lbfgs_ctx* c, int qk, int yk, int sk, int launches, double* us) {
    if (!c || !us || launches < 1) return LBFGS_ERR_BAD_ARG;
    if (!c->inited) return LBFGS_ERR_STATE;
    double* scratch = lbk_vec_alloc(c->dev);
    if (!scratch) return dev_err(c, -2);
    double* q = vec_by_index(c, qk, scratch);
    const double* y = vec_by_index(c, yk, scratch);
    const double* s = vec_by_index(c, sk, scratch);
    int rc = (q && y && s) ? 0 : -1;
    /* alpha = 0: q is written back unchanged (the vectors are finite at any step of a solve) */
    if (rc == 0) rc = lbk_stream_probe(c->dev, q, &y, &s, 1, launches, us, 0, NULL);
    lbk_vec_free(c->dev, scratch);
    return rc == 0 ? 0 : rc == -1 ? LBFGS_ERR_BAD_ARG : dev_err(c, rc);
}

/* ------------------------------------------------------------------------------------------
 * Host-callback objective (LBFGS_OBJ_HOST; single rank). The device forms every point the
 * objective is called at (z = x + alpha d, as the commit will form x_new) and the host calls
 * f / grad on a pinned copy of it.
 *   default: one f and at most one grad call per distinct point: z, f(z) and grad(z) are
 *            cached for the iteration, so a Wolfe trial's gradient (line_search.cpp:160) reuses
 *            its f call (:146), and the commit (lbfgs.cpp:160,171) reuses both;
 *   LBFGS_FLAG_REFERENCE_CALLS: the reference's own call sequence, call for call, including its
 *            re-evaluations of f(x) inside the line searches (line_search.cpp:24,42,65,133) and
 *            of f, grad at x_new after them (lbfgs.cpp:160,171); values returned by those calls
 *            are the ones used, as in the reference.
 * Transfers are asynchronous on the solver stream: the gradient upload runs from one of two
 * pinned buffers while the host goes on (e.g. into the f call that follows a grad call,
 * line_search.cpp:39-42), and in the reference order z's download overlaps the f(x) call.
 * ---------------------------------------------------------------------------------------- */
#define XF_Z 0
#define XF_X 1
#define XF_G0 2 /* + buffer */

/* objectives evaluated outside the fused stencil passes: host callbacks, and the dense quadratic
 * (a matrix-vector product needs the whole trial point first). Both run the same driver path:
 * z = x + alpha d formed on the device, f / grad at z, the commit with the gradient supplied. */
static int ext_obj(const lbfgs_ctx* c) { return c->obj == LBFGS_OBJ_HOST || c->obj == LBFGS_OBJ_DENSE_QUAD; }

static int host_bufs(lbfgs_ctx* c) {
    const size_t b = sizeof(double) * (size_t)c->n;
    if (!c->hx) c->hx = (double*)lbk_host_alloc(b);
    if (!c->hg[0]) c->hg[0] = (double*)lbk_host_alloc(b);
    if (!c->hg[1]) c->hg[1] = (double*)lbk_host_alloc(b);
    if (c->refcalls && !c->hxx) c->hxx = (double*)lbk_host_alloc(b);
    return (c->hx && c->hg[0] && c->hg[1] && (!c->refcalls || c->hxx)) ? 0 : LBFGS_ERR_NOMEM;
}

/* x or d changed: nothing cached refers to the current iteration */
static void host_invalidate(lbfgs_ctx* c) {
    c->hz_valid = 0;
    c->hf_valid = 0;
    c->gt_valid = 0;
}

/* issue z = x + alpha d and its download (no wait) */
static int host_point_issue(lbfgs_ctx* c, double alpha) {
    if (c->hz_valid && c->hz_alpha == alpha) return 0;
    if (c->hz_pending) DEVNC(lbk_xfer_wait(c->dev, XF_Z)); /* hx is still being written */
    DEV(lbk_point(c->dev, c->xn, c->x, c->d, alpha));
    if (c->obj == LBFGS_OBJ_DENSE_QUAD) { /* z stays on the device (xn) */
        c->hz_valid = 1;
        c->hz_pending = 0;
        c->hz_alpha = alpha;
        c->hf_valid = 0;
        return 0;
    }
    DEVNC(lbk_download_local_async(c->dev, c->hx, c->xn, XF_Z));
    c->hz_valid = c->hz_pending = 1;
    c->hz_alpha = alpha;
    c->hf_valid = 0;
    return 0;
}

static int host_point(lbfgs_ctx* c, double alpha) {
    int rc = host_point_issue(c, alpha);
    if (rc) return rc;
    if (c->hz_pending) {
        DEVNC(lbk_xfer_wait(c->dev, XF_Z));
        c->hz_pending = 0;
    }
    return 0;
}

/* f(z(alpha)); fresh = 1 calls f even if it was evaluated at this point before */
static int host_f_at(lbfgs_ctx* c, double alpha, int fresh, double* f) {
    if (!fresh && c->hf_valid && c->hf_alpha == alpha && c->hz_valid && c->hz_alpha == alpha) {
        *f = c->hf_val;
        return 0;
    }
    int rc = host_point(c, alpha);
    if (rc) return rc;
    if (c->obj == LBFGS_OBJ_DENSE_QUAD) { /* f and, for free, grad into gt */
        DEV(lbk_dense_eval(c->dev, c->xn, c->gt, SLOT_TRIAL(c->m)));
        DEVNC(lbk_fetch(c->dev, SLOT_TRIAL(c->m), 1, f));
        c->gt_valid = 1;
        c->gt_alpha = alpha;
    } else {
        *f = c->cb.f(c->hx, c->n, c->cb.user);
        c->cb_f++;
    }
    c->hf_valid = 1;
    c->hf_alpha = alpha;
    c->hf_val = *f;
    return 0;
}

/* grad(z(alpha)) into the device vector dst (the upload is left in flight) */
static int host_g_at(lbfgs_ctx* c, double alpha, int fresh, double* dst) {
    if (!fresh && c->gt_valid && c->gt_alpha == alpha) {
        if (dst != c->gt) DEVNC(lbk_copy(c->dev, dst, c->gt));
        return 0;
    }
    int rc = host_point(c, alpha);
    if (rc) return rc;
    if (c->obj == LBFGS_OBJ_DENSE_QUAD) {
        double f;
        DEV(lbk_dense_eval(c->dev, c->xn, dst, SLOT_TRIAL(c->m)));
        DEVNC(lbk_fetch(c->dev, SLOT_TRIAL(c->m), 1, &f));
        c->hf_valid = 1;
        c->hf_alpha = alpha;
        c->hf_val = f;
        if (dst == c->gt) {
            c->gt_valid = 1;
            c->gt_alpha = alpha;
        } else if (c->gt_valid && c->gt_alpha == alpha) {
            c->gt_valid = 0;
        }
        return 0;
    }
    const int b = c->hg_cur;
    c->hg_cur ^= 1;
    DEVNC(lbk_xfer_wait(c->dev, XF_G0 + b)); /* the upload that last read this buffer */
    c->cb.grad(c->hx, c->n, c->hg[b], c->cb.user);
    c->cb_g++;
    DEVNC(lbk_upload_local_async(c->dev, dst, c->hg[b], XF_G0 + b));
    if (dst == c->gt) {
        c->gt_valid = 1;
        c->gt_alpha = alpha;
    } else if (c->gt_valid && c->gt_alpha == alpha) {
        c->gt_valid = 0;
    }
    return 0;
}

/* reference call order: f at the iterate x itself (line_search.cpp:24,42,65,133) */
static int host_fx_issue(lbfgs_ctx* c) {
    if (c->hxx_valid) return 0;
    DEVNC(lbk_download_local_async(c->dev, c->hxx, c->x, XF_X));
    c->hxx_valid = c->hxx_pending = 1;
    return 0;
}

static int host_fx(lbfgs_ctx* c, double* f) {
    int rc = host_fx_issue(c);
    if (rc) return rc;
    if (c->hxx_pending) {
        DEVNC(lbk_xfer_wait(c->dev, XF_X));
        c->hxx_pending = 0;
    }
    *f = c->cb.f(c->hxx, c->n, c->cb.user);
    c->cb_f++;
    return 0;
}

/* f(x) as a line search sees it: the reference's fresh call in its order (the next trial
 * point's download issued first, so it overlaps the call), else the iteration's f_current */
static int ls_fx(lbfgs_ctx* c, double next_alpha, double* fx) {
    if (!(c->obj == LBFGS_OBJ_HOST && c->refcalls)) {
        *fx = c->f_cur;
        return 0;
    }
    int rc = host_fx_issue(c);
    if (!rc && next_alpha > 0) rc = host_point_issue(c, next_alpha);
    if (!rc) rc = host_fx(c, fx);
    return rc;
}

/* ------------------------------------------------------------------------------------------
 * Line-search trial evaluation. The fused speculative commit already evaluated f and
 * g_new.d at a0; every other step runs one k_trial pass over materialised x, d.
 * ---------------------------------------------------------------------------------------- */
static int materialize_d(lbfgs_ctx* c) {
    if (c->d_ready) return 0;
    const int m = c->m;
    if (c->dmode == LBK_D_TWOLOOP) {
        DEV(lbk_last(c->dev, c->d, c->rc, c->S[c->s_last_pair], c->g, c->rho_last, c->ref_b_last,
                     c->ref_a_last, SLOT_LAST(m)));
    } else if (c->dmode == D_VF) {
        DEV(lbk_vf_dir(c->dev, c->vf_h, c->d, c->g, c->vf_S, c->vf_Y, c->vf_cs, c->vf_cy, c->vf_cg));
    } else if (c->dmode == LBK_D_NEG_G && c->unfused) {
        DEV(lbk_update(c->dev, LBK_U_NEG, c->d, c->g, NULL, 0.0, -1, -1, 0.0));
        DEV(lbk_dot(c->dev, c->g, c->d, SLOT_LAST(m)));
    } else if (c->dmode == LBK_D_NEG_G) {
        DEV(lbk_negdot(c->dev, c->d, c->g, SLOT_LAST(m)));
    }
    /* sharded: neighbours' edge d rides this slot (vector-free: d's ghost cells hold it) */
    lbk_set_ghost_slot(c->dev, c->dmode == D_VF ? -1 : SLOT_LAST(m));
    c->dmode = LBK_D_BUF;
    c->d_ready = 1;
    return 0;
}

/* Device objectives, batched (c->batch). The steps a search tries after a rejection are known in
 * advance on its halving chains - backtracking alpha * beta (line_search.cpp:26), interpolation
 * alpha * 0.5 once alpha_prev == alpha (:92-97, the reference's alpha_prev quirk) - so one pass
 * evaluates LBK_TRIALS_NC of them, formed by the same repeated multiplication as the search. The
 * Wolfe searches' next step depends on the f just computed, so their pass takes one step, with
 * g.d (:160) in the same read (the gradient is recomputed by the commit, never stored). Results
 * are those of separate single-step passes, bit for bit. */
static int trial_batched(lbfgs_ctx* c, double alpha, int need_g, double* f, double* dphi) {
    if (!need_g && c->cand_valid && alpha == c->cand_alpha) { /* reduced by the first commit */
        *f = c->cand_f;
        return 0;
    }
    for (int j = 0; j < c->tc_n; ++j)
        if (alpha == c->tc_a[j] && (!need_g || (j == 0 && c->tc_dphi_ok))) {
            *f = c->tc_f[j];
            if (need_g && dphi) *dphi = c->tc_dphi;
            return 0;
        }
    const int want_dphi = need_g || c->ls == LBFGS_LS_WOLFE || c->ls == LBFGS_LS_BACKTRACKING_WOLFE;
    double a[LBK_TRIALS_NC];
    int nc = 1;
    a[0] = alpha;
    if (!want_dphi) {
        const double ratio = c->ls == LBFGS_LS_BACKTRACKING ? c->K.backtracking_alpha : 0.5;
        nc = LBK_TRIALS_NC;
        for (int j = 1; j < nc; ++j) a[j] = a[j - 1] * ratio;
    }
    /* d: the buffer once materialised; -g formed on the fly (one rank); the last second-loop
     * update formed on the fly for this iteration's first two trial passes, then materialised
     * (3 vector reads per pass against 4 once for k_last + 2 per pass) */
    int dm = LBK_D_BUF;
    if (!c->d_ready) {
        if (c->dmode == LBK_D_NEG_G && c->geo->world == 1) {
            dm = LBK_D_NEG_G;
        } else if (c->dmode == LBK_D_TWOLOOP && c->trial_passes < 2) {
            dm = LBK_D_TWOLOOP;
        } else {
            int rc = materialize_d(c);
            if (rc) return rc;
        }
    }
    const double* dsrc = dm == LBK_D_BUF ? c->d : dm == LBK_D_TWOLOOP ? c->rc : NULL;
    const double* s_last = dm == LBK_D_TWOLOOP ? c->S[c->s_last_pair] : NULL;
    DEV(lbk_trials(c->dev, c->obj, dm, c->x, dsrc, s_last, c->g, c->rho_last, c->ref_b_last, c->ref_a_last, a, nc,
                   want_dphi, SLOT_TRIAL(c->m)));
    double t[LBK_TRIALS_NC + 1];
    DEVNC(lbk_fetch(c->dev, SLOT_TRIAL(c->m), nc + (want_dphi ? 1 : 0), t));
    c->trial_passes++;
    c->tc_n = nc;
    for (int j = 0; j < nc; ++j) {
        c->tc_a[j] = a[j];
        c->tc_f[j] = t[j];
    }
    c->tc_dphi_ok = want_dphi;
    c->tc_dphi = want_dphi ? t[nc] : 0.0;
    *f = t[0];
    if (need_g && dphi) *dphi = c->tc_dphi;
    if (want_dphi)
        c->trials_fg++;
    else
        c->trials_f++;
    return 0;
}

static int trial(lbfgs_ctx* c, double alpha, int need_g, double* f, double* dphi) {
    if (c->spec_valid && alpha == c->a0) {
        *f = c->spec_f;
        if (dphi) *dphi = c->spec_dphi;
        return 0;
    }
    if (c->vf && c->vf_cand_valid && !need_g) { /* f already reduced by the first commit pass */
        for (int j = 0; j < LBK_VF_NA; ++j)
            if (alpha == c->vf_cand[j]) {
                *f = c->vf_cand_f[j];
                return 0;
            }
    }
    if (c->batch && !c->unfused && !ext_obj(c)) return trial_batched(c, alpha, need_g, f, dphi);
    int rc = materialize_d(c);
    if (rc) return rc;
    if (c->unfused) {
        /* x_new = x + alpha d materialised, then f (and grad, g_new . d) on it */
        double t[2];
        DEV(lbk_update(c->dev, LBK_U_POINT, c->xn, c->x, c->d, 0.0, -1, -1, alpha));
        DEV(lbk_eval(c->dev, c->obj, c->xn, need_g ? c->gt : NULL, SLOT_TRIAL(c->m)));
        DEVNC(lbk_fetch(c->dev, SLOT_TRIAL(c->m), 1, t));
        *f = t[0];
        if (need_g) {
            DEV(lbk_dot(c->dev, c->gt, c->d, SLOT_MISC(c->m) + 3));
            DEVNC(lbk_fetch(c->dev, SLOT_MISC(c->m) + 3, 1, &t[1]));
            if (dphi) *dphi = t[1];
        }
    } else if (ext_obj(c)) {
        /* reference order: the backtracking-Wolfe search takes grad(x_new) before f(x_new)
         * (line_search.cpp:39-42); the Wolfe search's gradient follows its own f call at the
         * same point (:146,160), never a second f */
        const int rf = c->refcalls && !(need_g && c->ls == LBFGS_LS_WOLFE);
        if (need_g && c->ls == LBFGS_LS_BACKTRACKING_WOLFE) {
            rc = host_g_at(c, alpha, c->refcalls, c->gt);
            if (!rc) rc = host_f_at(c, alpha, rf, f);
        } else {
            rc = host_f_at(c, alpha, rf, f);
            if (!rc && need_g) rc = host_g_at(c, alpha, c->refcalls, c->gt);
        }
        if (rc) return rc;
        if (need_g) {
            double t;
            DEV(lbk_dot(c->dev, c->gt, c->d, SLOT_TRIAL(c->m)));
            DEVNC(lbk_fetch(c->dev, SLOT_TRIAL(c->m), 1, &t));
            if (dphi) *dphi = t;
        }
    } else {
        double t[2];
        DEV(lbk_trial(c->dev, c->obj, c->x, c->d, alpha, need_g ? c->gt : NULL, SLOT_TRIAL(c->m)));
        DEVNC(lbk_fetch(c->dev, SLOT_TRIAL(c->m), 2, t));
        *f = t[0];
        if (need_g && dphi) *dphi = t[1];
    }
    if (need_g)
        c->trials_fg++;
    else
        c->trials_f++;
    return 0;
}

static double cubic_interp(double a0, double a1, double p0, double dp0, double p1, double dp1) {
    double d1 = dp0 + dp1 - 3 * (p1 - p0) / (a1 - a0); /* line_search.cpp:8-12 */
    double d2 = copysign(sqrt(d1 * d1 - dp0 * dp1), a1 - a0);
    return a0 + (a1 - a0) * (dp0 + d2 - d1) / (dp0 - dp1 + 2 * d2);
}

static double quad_interp(double a0, double p0, double dp0, double p1) { /* :14-16 */
    return a0 - 0.5 * dp0 * a0 * a0 / (p1 - p0 - dp0 * a0);
}

static int search_here(const lbfgs_ctx* c, double alpha, int need_g);
static int search_device(lbfgs_ctx* c, double gd, lbk_search* st);

/* line_search.cpp:19-30 (f(x) == f_current, g.d == gd: identical values, evaluated once) */
static int ls_backtracking(lbfgs_ctx* c, double gd, double* out) {
    const lbfgs_constants* K = &c->K;
    double alpha = K->initial_step;
    for (;;) {
        if (search_here(c, alpha, 0)) {
            lbk_search st = {0};
            st.alpha = alpha;
            const int rc = search_device(c, gd, &st);
            if (rc < 0) return rc;
            if (rc == 0 && st.done) {
                *out = st.step;
                return 0;
            }
            if (rc == 0) alpha = st.alpha; /* its pass budget spent: on from there */
        }
        double fx, ft;
        int rc = ls_fx(c, alpha, &fx); /* f(x) - f(x + alpha d), left operand first */
        if (!rc) rc = trial(c, alpha, 0, &ft, NULL);
        if (rc) return rc;
        if (!(fx - ft < K->c1 * alpha * gd)) break;
        alpha *= K->backtracking_alpha;
        if (alpha < K->backtracking_tol) break;
    }
    *out = alpha;
    return 0;
}

/* line_search.cpp:33-55 */
static int ls_backtracking_wolfe(lbfgs_ctx* c, double gd, double* out) {
    const lbfgs_constants* K = &c->K;
    double alpha = K->initial_step;
    for (;;) {
        if (search_here(c, alpha, 1)) {
            lbk_search st = {0};
            st.alpha = alpha;
            const int rd = search_device(c, gd, &st);
            if (rd < 0) return rd;
            if (rd == 0 && st.done) {
                *out = st.step;
                return 0;
            }
            if (rd == 0) alpha = st.alpha;
        }
        double fn, dphi, fx;
        int rc = trial(c, alpha, 1, &fn, &dphi);
        if (!rc) rc = ls_fx(c, 0.0, &fx);
        if (rc) return rc;
        if (fn > fx + K->c1 * alpha * gd) {
            alpha *= K->backtracking_alpha;
        } else if (dphi < K->c2 * gd) {
            alpha *= 1.1;
        } else {
            break;
        }
        if (alpha < K->backtracking_tol) break;
    }
    *out = alpha;
    return 0;
}

/* line_search.cpp:57-121 */
static int ls_interpolation(lbfgs_ctx* c, double gd, double* out) {
    const lbfgs_constants* K = &c->K;
    double f_x;
    int rc0 = ls_fx(c, K->initial_step, &f_x);
    if (rc0) return rc0;
    double alpha = K->initial_step, alpha_prev = 0.0, f_prev = f_x;
    int it = 0;
    for (;;) {
        if (search_here(c, alpha, 0)) { /* it: the counter before the loop's `it++ < 20` test */
            lbk_search st = {0};
            st.alpha = alpha;
            st.alpha_prev = alpha_prev;
            st.f_prev = f_prev;
            st.iter = it;
            const int rd = search_device(c, gd, &st);
            if (rd < 0) return rd;
            if (rd == 0 && st.done) {
                *out = st.step;
                return 0;
            }
            if (rd == 0) {
                alpha = st.alpha;
                alpha_prev = st.alpha_prev;
                f_prev = st.f_prev;
                it = st.iter;
            }
        }
        if (!(it++ < 20)) break;
        double f_new;
        int rc = trial(c, alpha, 0, &f_new, NULL);
        if (rc) return rc;
        if (f_new <= f_x + K->c1 * alpha * gd) {
            *out = alpha;
            return 0;
        }
        if (alpha < K->wolfe_interp_min) {
            *out = K->wolfe_interp_min;
            return 0;
        }
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
            alpha = quad_interp(alpha, f_new, gd, f_x);
            if (alpha < 0.1 * K->initial_step || alpha > 0.9 * K->initial_step)
                alpha = K->initial_step * 0.5;
        }
        alpha_prev = alpha;
        f_prev = f_new;
    }
    *out = alpha;
    return 0;
}

/* Small n (single rank, a cooperative size, device objective): once a line search needs a trial
 * pass, the rest of the search runs on the device in one launch (lbk_search_dev: the same loop,
 * the same expressions, the same passes and caches) instead of a launch and a host
 * round trip per trial pass, and the commit at the step it finds follows in the same launch.
 * search_here: trial(alpha, need_g) would launch a pass, and the device form applies. */
static int search_here(const lbfgs_ctx* c, double alpha, int need_g) {
    if (ext_obj(c) || c->unfused || !c->batch || c->vf || !lbk_search_dev_ok(c->dev, c->obj)) return 0;
    if (c->spec_valid && alpha == c->a0) return 0; /* the commit's first trial: no pass */
    if (!need_g && c->cand_valid && alpha == c->cand_alpha) return 0;
    for (int j = 0; j < c->tc_n; ++j) /* the last trial pass */
        if (alpha == c->tc_a[j] && (!need_g || (j == 0 && c->tc_dphi_ok))) return 0;
    return 1;
}

/* st: the caller's loop variables at the top of an iteration (alpha, and the search's own); the
 * constants and the host's caches are filled in here, and the caches come back as the host loop
 * would leave them. Returns 0 (st->done: the step; else the loop variables to go on from), 1 when
 * the launch's grid barrier timed out (nothing usable came back: the host loop goes on from the
 * same state, and the device form is off for the context), or < 0. */
static int search_device(lbfgs_ctx* c, double gd, lbk_search* st) {
    const lbfgs_constants* K = &c->K;
    int rc = materialize_d(c);
    if (rc) return rc;
    st->f_x = c->f_cur; /* ls_fx for a device objective */
    st->gd = gd;
    st->c1 = K->c1;
    st->c2 = K->c2;
    st->amin = K->wolfe_interp_min;
    st->init = K->initial_step;
    st->beta = K->backtracking_alpha;
    st->tol = K->backtracking_tol;
    st->have_spec = c->spec_valid;
    st->spec_a = c->a0;
    st->spec_f = c->spec_f;
    st->spec_dphi = c->spec_dphi;
    st->have_cand = c->cand_valid;
    st->cand_a = c->cand_alpha;
    st->cand_f = c->cand_f;
    st->tc_n = c->tc_n;
    st->tc_dphi_ok = c->tc_dphi_ok;
    st->tc_dphi = c->tc_dphi;
    for (int j = 0; j < LBK_TRIALS_NC; ++j) {
        st->tc_a[j] = c->tc_a[j];
        st->tc_f[j] = c->tc_f[j];
    }
    lbk_search_commit cm = {c->g, c->xn, c->gn, c->S[c->free_pair], c->Y[c->free_pair], c->search_cslot};
    rc = lbk_search_dev(c->dev, c->obj, c->ls, c->x, c->d, st, &cm);
    if (rc == -6) { /* barrier time-out: the host loop takes over */
        if (cm.slot >= 0) c->recommit_a0 = 1;
        return 1;
    }
    if (rc) return dev_err(c, rc);
    const int passes = st->passes_f + st->passes_fg;
    c->trials_f += st->passes_f;
    c->trials_fg += st->passes_fg;
    c->trial_passes += passes;
    c->passes += passes;
    c->tc_n = st->tc_n;
    c->tc_dphi_ok = st->tc_dphi_ok;
    c->tc_dphi = st->tc_dphi;
    for (int j = 0; j < LBK_TRIALS_NC; ++j) {
        c->tc_a[j] = st->tc_a[j];
        c->tc_f[j] = st->tc_f[j];
    }
    c->search_launches++;
    if (st->committed) {
        c->search_committed = 1;
        c->search_commits++;
        c->passes++;
    }
    return 0;
}

/* line_search.cpp:125-189 */
static int ls_wolfe(lbfgs_ctx* c, double gd, double* out) {
    const lbfgs_constants* K = &c->K;
    double f_x;
    int rc0 = ls_fx(c, K->initial_step, &f_x);
    if (rc0) return rc0;
    double alpha = K->initial_step;
    double alpha_lo = 0.0, alpha_hi = INFINITY, f_lo = f_x, dphi_lo = gd;
    for (int iter = 0; iter < 20; ++iter) {
        if (search_here(c, alpha, 0)) {
            lbk_search st = {0};
            st.alpha = alpha;
            st.alpha_lo = alpha_lo;
            st.alpha_hi = alpha_hi;
            st.f_lo = f_lo;
            st.dphi_lo = dphi_lo;
            st.iter = iter;
            const int rd = search_device(c, gd, &st);
            if (rd < 0) return rd;
            if (rd == 0 && st.done) {
                *out = st.step;
                return 0;
            }
            /* rd == 1: the device search gave up (a grid barrier timed out) having changed nothing;
             * it is off for this context now, and this iteration of the host loop runs as it
             * would have. rd == 0, not done (its pass budget spent; 20 passes cover the 20
             * iterations, so not expected): on from its state */
            if (rd == 0) {
                alpha = st.alpha;
                alpha_lo = st.alpha_lo;
                alpha_hi = st.alpha_hi;
                f_lo = st.f_lo;
                dphi_lo = st.dphi_lo;
                iter = st.iter;
            }
        }
        double f_new, dphi_new;
        /* f first; the gradient only if the sufficient-decrease tests pass (:144-153) */
        int rc = trial(c, alpha, 0, &f_new, NULL);
        if (rc) return rc;
        if (f_new > f_x + K->c1 * alpha * gd || (f_new >= f_lo && iter > 0)) {
            alpha_hi = alpha;
            alpha = cubic_interp(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new,
                                 (f_new - f_x - gd * alpha) / (alpha * alpha));
            continue;
        }
        rc = trial(c, alpha, 1, &f_new, &dphi_new);
        if (rc) return rc;
        if (fabs(dphi_new) <= -K->c2 * gd) {
            *out = alpha;
            return 0;
        }
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
        if (alpha < K->wolfe_interp_min) {
            *out = K->wolfe_interp_min;
            return 0;
        }
    }
    *out = alpha;
    return 0;
}

static int run_line_search(lbfgs_ctx* c, double gd, double* alpha) {
    TRACE_PUSH("line search");
    int rc;
    switch (c->ls) {
        case LBFGS_LS_BACKTRACKING: rc = ls_backtracking(c, gd, alpha); break;
        case LBFGS_LS_INTERPOLATION: rc = ls_interpolation(c, gd, alpha); break;
        case LBFGS_LS_WOLFE: rc = ls_wolfe(c, gd, alpha); break;
        default: rc = ls_backtracking_wolfe(c, gd, alpha); break;
    }
    TRACE_POP();
    return rc;
}

/* ------------------------------------------------------------------------------------------
 * Commit at step alpha: x_new, g_new, s, y and their reductions into tot[].
 * ---------------------------------------------------------------------------------------- */
/* unfused commit (LBFGS_FLAG_UNFUSED): lbfgs.cpp:159-181 one operation per launch */
static int commit_unfused(lbfgs_ctx* c, double alpha, double* tot) {
    const int pair = c->free_pair, sm = SLOT_MISC(c->m);
    double t[2];
    DEV(lbk_update(c->dev, LBK_U_POINT, c->xn, c->x, c->d, 0.0, -1, -1, alpha));
    DEV(lbk_eval(c->dev, c->obj, c->xn, c->gn, sm)); /* f(x_new), g_new, g_new . g_new */
    DEV(lbk_update(c->dev, LBK_U_SUB, c->S[pair], c->xn, c->x, 0.0, -1, -1, 0.0));
    DEV(lbk_update(c->dev, LBK_U_SUB, c->Y[pair], c->gn, c->g, 0.0, -1, -1, 0.0));
    DEV(lbk_dot(c->dev, c->S[pair], c->Y[pair], sm + 1));
    DEV(lbk_dot(c->dev, c->Y[pair], c->Y[pair], sm + 2));
    DEVNC(lbk_fetch(c->dev, sm, 2, t));
    tot[LBK_C_F] = t[0];
    tot[LBK_C_GG] = t[1];
    DEVNC(lbk_fetch(c->dev, sm + 1, 1, &tot[LBK_C_SY]));
    DEVNC(lbk_fetch(c->dev, sm + 2, 1, &tot[LBK_C_YY]));
    c->commits++;
    return 0;
}

/* unfused two-loop (lbfgs.cpp:127-171): a dot launch and an update launch per pair and
 * loop, gamma scaling and d = -r as launches of their own; leaves d and g.d (SLOT_LAST) */
static int twoloop_unfused(lbfgs_ctx* c, const double* rho, double gamma) {
    const int h = c->h, m = c->m;
    const double* qsrc = c->g;
    for (int i = h - 1; i >= 0; --i) {
        const int sa = i == h - 1 ? SLOT_P0 : SLOT_A0 + i;
        DEV(lbk_dot(c->dev, c->S[c->ring[i]], qsrc, sa));
        DEV(lbk_update(c->dev, LBK_U_AXPY_Q, c->q, qsrc, c->Y[c->ring[i]], rho[i], sa, -1, 0.0));
        qsrc = c->q;
    }
    DEV(lbk_update(c->dev, LBK_U_SCALE, c->r, c->q, NULL, 0.0, -1, -1, gamma));
    for (int i = 0; i < h; ++i) {
        const int sa = i == h - 1 ? SLOT_P0 : SLOT_A0 + i, sb = SLOT_B0(m) + i;
        DEV(lbk_dot(c->dev, c->Y[c->ring[i]], c->r, sb));
        DEV(lbk_update(c->dev, LBK_U_AXPY_R, c->r, c->r, c->S[c->ring[i]], rho[i], sa, sb, 0.0));
    }
    DEV(lbk_update(c->dev, LBK_U_NEG, c->d, c->r, NULL, 0.0, -1, -1, 0.0));
    DEV(lbk_dot(c->dev, c->g, c->d, SLOT_LAST(m)));
    c->dmode = LBK_D_BUF;
    c->d_ready = 1;
    return 0;
}

static int commit(lbfgs_ctx* c, int dmode, double alpha, int cslot, double* tot, double cand) {
    if (c->unfused) return commit_unfused(c, alpha, tot);
    const int pair = c->free_pair;
    const double* dsrc = dmode == LBK_D_BUF ? c->d : c->rc;
    const double* s_last = dmode == LBK_D_TWOLOOP ? c->S[c->s_last_pair] : NULL;
    int obj = c->obj;
    if (ext_obj(c)) {
        /* f(x_new) (lbfgs.cpp:160), then - unless the step failed (:164-168) - grad(x_new)
         * (:171) onto the device for the commit kernel; both from the line search's cache
         * unless the reference call order asks for the reference's fresh calls */
        double f;
        int rc = host_f_at(c, alpha, c->refcalls, &f);
        if (rc) return rc;
        if (alpha < 1e-10) { /* the caller stops here; nothing else of tot is read */
            tot[LBK_C_F] = f;
            return 0;
        }
        rc = host_g_at(c, alpha, c->refcalls, c->gn);
        if (rc) return rc;
        obj = LBK_OBJ_NONE;
        DEV(lbk_commit(c->dev, obj, dmode, c->x, dsrc, s_last, c->g, c->rho_last, c->ref_b_last,
                       c->ref_a_last, alpha, c->xn, c->gn, c->S[pair], c->Y[pair], cslot, 0.0));
        DEVNC(lbk_fetch(c->dev, cslot, 7, tot));
        tot[LBK_C_F] = f;
    } else {
        const int with_cand = cand > 0.0 && dmode != LBK_D_BUF;
        DEV(lbk_commit(c->dev, obj, dmode, c->x, dsrc, s_last, c->g, c->rho_last, c->ref_b_last,
                       c->ref_a_last, alpha, c->xn, c->gn, c->S[pair], c->Y[pair], cslot, with_cand ? cand : 0.0));
        DEVNC(lbk_fetch(c->dev, cslot, with_cand ? 8 : 7, tot));
        if (with_cand) {
            c->cand_valid = 1;
            c->cand_alpha = cand;
            c->cand_f = tot[LBK_C_FC];
        }
    }
    c->commits++;
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * One iteration of lbfgs.cpp:72-199. Returns 0 to continue, 1 when finished, < 0 on error.
 * ---------------------------------------------------------------------------------------- */
static void note_h(lbfgs_ctx* c) {
    if (c->h_min < 0 || c->h < c->h_min) c->h_min = c->h;
    if (c->h > c->h_max) c->h_max = c->h;
}

/* the backtracking search's second step, f reduced by the commit pass (line_search.cpp:26) */
static double first_cand(const lbfgs_ctx* c) {
    return (c->batch && c->ls == LBFGS_LS_BACKTRACKING) ? c->K.initial_step * c->K.backtracking_alpha : 0.0;
}

/* a queued speculative launch the host does not take: wait for its record. It either did not go
 * (nothing written, reservations released) or ran on buffers the host no longer reads - which
 * holds only if the host also took the first trial and stored the pair in the iteration before
 * (the kernel's other tests - convergence, rho, gamma - can only differ by a rounding the
 * host then handles itself). */
static int spec_drop(lbfgs_ctx* c) {
    if (!c->sp_pend) return 0;
    c->sp_pend = 0;
    c->sp_dropped++;
    double t[1];
    int went = 0;
    DEVNC(lbk_small_fetch(c->dev, c->sp_epoch, c->sp_cslot, 1, t, &went, NULL, NULL));
    if (!went) c->passes--; /* a launch that did nothing is no pass */
    if (went && !c->sp_hostgo) {
        snprintf(c->err, sizeof c->err, "speculative iteration %d ran where the host stopped", c->sp_k);
        return LBFGS_ERR_STATE;
    }
    return 0;
}

/* queue iteration k + 1 behind iteration k's latest commit, assuming the pair is stored: the ring
 * then drops its oldest pair (h = m) or grows, the new pair is the current free one, x/xn and g/gn
 * swap, and alpha_{h-1} of the first loop is the commit's s.g (component SG). decided = 0: behind
 * the cooperative launch, whose commit at a0 the line search has yet to judge (the kernel
 * re-checks its first-trial test); decided > 0: behind a recommit at that step */
static int spec_next(lbfgs_ctx* c, double decided) {
    const int m = c->m, h = c->h, k = c->k;
    if (!c->spec_on || c->steps_left <= 0 || c->cur_epoch == 0 || c->K.initial_step < 1e-10) return 0;
    const int h1 = h < m ? h + 1 : m;
    if (!lbk_small_spec_ok(c->dev, h1)) return 0;
    int ring1[MMAX + 1], free1;
    if (h >= m) {
        for (int i = 0; i + 1 < m; ++i) ring1[i] = c->ring[i + 1];
        ring1[m - 1] = c->free_pair;
        free1 = c->ring[0];
    } else {
        for (int i = 0; i < h; ++i) ring1[i] = c->ring[i];
        ring1[h] = c->free_pair;
        free1 = h + 1;
    }
    const double* Sr[MMAX];
    const double* Yr[MMAX];
    double rho1[MMAX];
    for (int i = 0; i < h1; ++i) {
        Sr[i] = c->S[ring1[i]];
        Yr[i] = c->Y[ring1[i]];
        rho1[i] = i + 1 < h1 ? 1.0 / c->sy[ring1[i]] : 0.0; /* the new pair's: the kernel's */
    }
    const int cslot = SLOT_COMMIT0 + (k & 1), cslot1 = SLOT_COMMIT0 + ((k + 1) & 1);
    const int p01 = REF(cslot, LBK_C_SG);
    lbk_spec sp;
    sp.prev_slot = cslot;
    sp.ls = decided > 0.0 ? -1 : c->ls; /* a recommit's step is the host's already */
    sp.fx = c->f_cur;
    sp.c1 = c->K.c1;
    sp.c2 = c->K.c2;
    sp.tol = c->tol;
    sp.chain_epoch = c->cur_spec && decided <= 0.0 ? c->cur_epoch : 0;
    DEV(lbk_small_iter(c->dev, c->obj, h1, c->gn, c->q, c->r, Sr, Yr, rho1, 0.0, p01, c->K.initial_step, c->xn,
                       c->x, c->g, c->S[free1], c->Y[free1], SLOT_P0, SLOT_A0, SLOT_B0(m), cslot1, first_cand(c),
                       &sp, &c->sp_epoch));
    c->sp_alpha = decided > 0.0 ? decided : c->K.initial_step;
    c->sp_pend = 1;
    c->sp_k = k + 1;
    c->sp_h = h1;
    memcpy(c->sp_ring, ring1, sizeof(int) * (size_t)h1);
    c->sp_free = free1;
    c->sp_p0 = p01;
    c->sp_cslot = cslot1;
    c->sp_x = c->xn;
    c->sp_xn = c->x;
    c->sp_g = c->gn;
    c->sp_gn = c->g;
    memcpy(c->sp_rho, rho1, sizeof(double) * (size_t)h1);
    c->sp_hostgo = 0;
    return 0;
}

/* this iteration's cooperative (or single-workgroup) launch: the two-loop passes and the commit at a0 */
static int small_launch(lbfgs_ctx* c, const double* rho, const double* const* Sr, const double* const* Yr,
                        double gamma, int p0_ref) {
    DEV(lbk_small_iter(c->dev, c->obj, c->h, c->g, c->q, c->r, Sr, Yr, rho, gamma, p0_ref, c->K.initial_step,
                       c->x, c->xn, c->gn, c->S[c->free_pair], c->Y[c->free_pair], SLOT_P0, SLOT_A0,
                       SLOT_B0(c->m), SLOT_COMMIT0 + (c->k & 1), first_cand(c), NULL, &c->cur_epoch));
    c->cur_spec = 0;
    return 0;
}

/* the commit totals of this iteration's small launch. An adopted speculative launch that did not
 * go (its tests disagreed with the host's, possible only through a rounding difference: never
 * seen) is replaced by an ordinary launch; the one queued behind it was chained to it and did not
 * go either. One that went with another rho or gamma than the host's cannot be replaced (the
 * launch behind it has overwritten this iteration's x) and fails the solve. */
static int small_fetch(lbfgs_ctx* c, int cslot, double* tot) {
    int went = 1;
    double vr = 0.0, vg = 0.0;
    DEVNC(lbk_small_fetch(c->dev, c->cur_epoch, cslot, 8, tot, &went, &vr, &vg));
    if (!c->cur_spec) return 0;
    if (!went) {
        c->passes -= c->sp_pend ? 2 : 1; /* this launch and the one chained behind it did nothing */
        c->sp_pend = 0;
        c->sp_dropped++;
        double rho[MMAX];
        const double* Sr[MMAX];
        const double* Yr[MMAX];
        for (int i = 0; i < c->h; ++i) {
            rho[i] = 1.0 / c->sy[c->ring[i]];
            Sr[i] = c->S[c->ring[i]];
            Yr[i] = c->Y[c->ring[i]];
        }
        int rc = small_launch(c, rho, Sr, Yr, c->cur_gamma, c->cur_p0);
        if (rc) return rc;
        DEVNC(lbk_small_fetch(c->dev, c->cur_epoch, cslot, 8, tot, NULL, NULL, NULL));
        return 0;
    }
    if (memcmp(&vr, &c->cur_rho, sizeof vr) != 0 || memcmp(&vg, &c->cur_gamma, sizeof vg) != 0) {
        snprintf(c->err, sizeof c->err, "speculative iteration %d: device rho/gamma %.17g/%.17g, host %.17g/%.17g",
                 c->k, vr, vg, c->cur_rho, c->cur_gamma);
        return LBFGS_ERR_STATE;
    }
    c->sp_adopted++;
    return 0;
}

/* small n, the line search took another step than a0: the recommit, then iteration k + 1 queued
 * behind it (no line-search test: the step is decided), then the commit's totals once the stream
 * has passed the recommit */
static int commit_queued(lbfgs_ctx* c, int dmode, double alpha, int cslot, double* tot) {
    const int pair = c->free_pair;
    const double* dsrc = dmode == LBK_D_BUF ? c->d : c->rc;
    const double* s_last = dmode == LBK_D_TWOLOOP ? c->S[c->s_last_pair] : NULL;
    DEV(lbk_commit(c->dev, c->obj, dmode, c->x, dsrc, s_last, c->g, c->rho_last, c->ref_b_last, c->ref_a_last, alpha,
                   c->xn, c->gn, c->S[pair], c->Y[pair], cslot, 0.0));
    DEVNC(lbk_mark(c->dev)); /* an event, not a pass */
    int rc = alpha >= 1e-10 ? spec_next(c, alpha) : 0;
    if (rc) return rc;
    DEVNC(lbk_fetch_marked(c->dev, cslot, 7, tot));
    c->commits++;
    return 0;
}

/* the queued launch is this iteration's exactly (same history, buffers, slots and the host's
 * rho of the older pairs; rho and gamma of the newest pair are compared when its record is read) */
static int spec_matches(const lbfgs_ctx* c, int h, const double* rho, int p0_ref) {
    if (!c->sp_pend || c->sp_k != c->k || c->sp_h != h || c->sp_free != c->free_pair || c->sp_p0 != p0_ref ||
        c->sp_cslot != SLOT_COMMIT0 + (c->k & 1) || c->sp_x != c->x || c->sp_xn != c->xn || c->sp_g != c->g ||
        c->sp_gn != c->gn)
        return 0;
    for (int i = 0; i < h; ++i)
        if (c->sp_ring[i] != c->ring[i]) return 0;
    for (int i = 0; i + 1 < h; ++i)
        if (memcmp(&c->sp_rho[i], &rho[i], sizeof(double)) != 0) return 0;
    return 1;
}

static int iterate(lbfgs_ctx* c) {
    const int k = c->k, m = c->m, h = c->h;
    const double gnorm = sqrt(c->gg);
    int rc = trace_push(c, c->f_cur, gnorm, 1);
    if (rc) return rc;
    if (c->flags & LBFGS_FLAG_VERBOSE) { /* :76-78 */
        printf("Iteration %d, f = %g, |grad| = %g\n", k, c->f_cur, gnorm);
        fflush(stdout);
    }
    if (gnorm < c->tol) { /* :80-84 */
        say(c, "Converged!\n");
        c->status = LBFGS_STATUS_CONVERGED;
        rc = spec_drop(c);
        return rc ? rc : 1;
    }
    note_h(c);

    /* ---- search direction (:87-143) ---- */
    int dmode = LBK_D_NEG_G;
    int small_done = 0;
    const int small = !ext_obj(c) && !c->unfused && c->geo->world == 1 && lbk_small_ok(c->dev, h);
    c->cur_epoch = 0;
    c->cur_spec = 0;
    c->d_ready = 0;
    c->spec_valid = 0;
    c->cand_valid = 0;
    c->tc_n = 0;
    c->trial_passes = 0;
    host_invalidate(c);
    c->hxx_valid = 0;
    if (!(k == 0 || h == 0)) {
        int bad_rho = 0;
        for (int i = h - 1; i >= 0; --i)
            if (!isfinite(1.0 / c->sy[c->ring[i]])) bad_rho = 1; /* :102-108 */
        double gamma = 0.0;
        if (bad_rho) {
            say(c, "Warning: Invalid rho at iteration %d\n", k);
        } else {
            const int top = c->ring[h - 1];
            gamma = c->sy[top] / c->yy[top]; /* :117-118 */
            if (gamma <= 0 || !isfinite(gamma)) {
                say(c, "Warning: Invalid gamma at iteration %d\n", k);
            } else {
                dmode = LBK_D_TWOLOOP;
            }
        }
        if (dmode == LBK_D_TWOLOOP && c->unfused) {
            double rho[MMAX];
            for (int i = 0; i < h; ++i) rho[i] = 1.0 / c->sy[c->ring[i]];
            rc = twoloop_unfused(c, rho, gamma);
            if (rc) return rc;
            dmode = LBK_D_BUF;
        } else if (dmode == LBK_D_TWOLOOP && small) {
            /* one single-workgroup launch: the passes below and the commit at a0 */
            double rho[MMAX];
            const double* Sr[MMAX];
            const double* Yr[MMAX];
            for (int i = 0; i < h; ++i) {
                rho[i] = 1.0 / c->sy[c->ring[i]];
                Sr[i] = c->S[c->ring[i]];
                Yr[i] = c->Y[c->ring[i]];
            }
            const int top = c->ring[h - 1];
            const int p0_ref = c->sg_valid ? c->sg_ref : -1;
            c->cur_rho = rho[h - 1];
            c->cur_gamma = gamma;
            c->cur_p0 = p0_ref;
            if (spec_matches(c, h, rho, p0_ref)) { /* already queued behind the last iteration */
                c->sp_pend = 0;
                c->cur_epoch = c->sp_epoch;
                c->cur_spec = 1;
            } else {
                rc = spec_drop(c);
                if (rc) return rc;
                rc = small_launch(c, rho, Sr, Yr, gamma, p0_ref);
                if (rc) return rc;
            }
            /* the next iteration, queued before this one's results are read */
            rc = spec_next(c, 0.0);
            if (rc) return rc;
            c->rho_last = rho[h - 1];
            c->ref_b_last = REF(SLOT_B0(m) + h - 1, 0);
            c->ref_a_last = p0_ref >= 0 ? p0_ref : REF(SLOT_P0, 0); /* alpha_{h-1}: s_{h-1} . g */
            c->s_last_pair = top;
            c->rc = c->r;
            small_done = 1;
        } else if (dmode == LBK_D_TWOLOOP) {
            int refA[MMAX], refB[MMAX];
            double rho[MMAX];
            for (int i = 0; i < h; ++i) rho[i] = 1.0 / c->sy[c->ring[i]];
            const int top = c->ring[h - 1];
            if (!ext_obj(c) && c->geo->world == 1 && lbk_twoloop_ok(c->dev, h)) {
                /* LBFGS_PERSIST=2: the passes below in one persistent launch, same slots */
                const double* Sr[MMAX];
                const double* Yr[MMAX];
                for (int i = 0; i < h; ++i) {
                    Sr[i] = c->S[c->ring[i]];
                    Yr[i] = c->Y[c->ring[i]];
                }
                DEV(lbk_twoloop_persist(c->dev, h, c->g, c->q, c->r, Sr, Yr, rho, gamma, c->sg_valid ? c->sg_ref : -1,
                                        SLOT_P0, SLOT_A0, SLOT_B0(m)));
                refA[h - 1] = c->sg_valid ? c->sg_ref : REF(SLOT_P0, 0);
                for (int i = h - 2; i >= 0; --i) refA[i] = REF(SLOT_A0 + i, 0);
                for (int i = 0; i < h; ++i) refB[i] = REF(SLOT_B0(m) + i, 0);
                c->rc = c->r;
                c->rho_last = rho[h - 1];
                c->ref_b_last = refB[h - 1];
                c->ref_a_last = refA[h - 1];
                c->s_last_pair = top;
            } else {
                if (c->sg_valid) {
                    refA[h - 1] = c->sg_ref; /* s_{h-1}.g from the previous commit */
                } else {
                    DEV(lbk_dot(c->dev, c->S[top], c->g, SLOT_P0));
                    refA[h - 1] = REF(SLOT_P0, 0);
                }
                /* q and r are updated in place (the passes' q/r stay in the Infinity Cache; a
                 * ping-pong between two buffers measured neutral at 1e8 and -8 % at 1e7) */
                const double* qsrc = c->g;
                for (int i = h - 2; i >= 0; --i) {
                    DEV(lbk_axpy_dot(c->dev, c->q, qsrc, c->Y[c->ring[i + 1]], c->S[c->ring[i]], rho[i + 1],
                                     refA[i + 1], SLOT_A0 + i));
                    refA[i] = REF(SLOT_A0 + i, 0);
                    qsrc = c->q;
                }
                DEV(lbk_mid(c->dev, c->r, qsrc, c->Y[c->ring[0]], rho[0], gamma, refA[0], SLOT_B0(m)));
                refB[0] = REF(SLOT_B0(m), 0);
                for (int i = 0; i + 1 < h; ++i) {
                    DEV(lbk_axpy2_dot(c->dev, c->r, c->r, c->S[c->ring[i]], c->Y[c->ring[i + 1]], rho[i], refB[i],
                                      refA[i], SLOT_B0(m) + i + 1));
                    refB[i + 1] = REF(SLOT_B0(m) + i + 1, 0);
                }
                c->rc = c->r;
                c->rho_last = rho[h - 1];
                c->ref_b_last = refB[h - 1];
                c->ref_a_last = refA[h - 1];
                c->s_last_pair = top;
            }
        }
    }
    if (c->sp_pend && c->sp_k == k) { /* queued for this iteration, which took another path */
        rc = spec_drop(c);
        if (rc) return rc;
    }
    c->dmode = dmode;
    if (c->unfused && dmode == LBK_D_BUF) c->d_ready = 1;

    /* ---- descent check (:146-153) and the line search (:156) ---- */
    const int cslot = SLOT_COMMIT0 + (k & 1);
    double tot[LBK_KMAX];
    double gd;
    c->a0 = c->K.initial_step;
    const int sharded = c->geo->world > 1;
    if (!ext_obj(c) && !c->unfused) {
        /* last two-loop pass + first trial at a0 + commit fused in one pass. Sharded, the
         * stencil's halo of d at the rank edges comes from the neighbours' edge r (published
         * with the last second-loop pass's reduction) and s_{h-1}'s ghost cells; d = -g is
         * materialised first so that its edge values reach the neighbours through its slot. */
        if (sharded && c->dmode == LBK_D_TWOLOOP) {
            lbk_set_ghost_slot(c->dev, SLOT_B0(m) + h - 1);
        } else if (sharded) {
            rc = materialize_d(c);
            if (rc) return rc;
        }
        /* the backtracking search's second step, f reduced by the same pass (line_search.cpp:26) */
        const double cand = (c->batch && c->ls == LBFGS_LS_BACKTRACKING) ? c->a0 * c->K.backtracking_alpha : 0.0;
        if (small_done) { /* the commit at a0 ran inside lbk_small_iter */
            rc = small_fetch(c, cslot, tot);
            if (rc) return rc;
            c->commits++;
            if (cand > 0.0) {
                c->cand_valid = 1;
                c->cand_alpha = cand;
                c->cand_f = tot[LBK_C_FC];
            }
        } else {
            rc = commit(c, c->dmode, c->a0, cslot, tot, cand);
            if (rc) return rc;
        }
        gd = tot[LBK_C_GD];
        if (gd >= 0) {
            say(c, "Warning: Not a descent direction, using gradient\n");
            c->dmode = dmode = LBK_D_NEG_G;
            c->d_ready = 0;
            if (sharded) {
                rc = materialize_d(c);
                if (rc) return rc;
            }
            rc = commit(c, c->dmode, c->a0, cslot, tot, cand);
            if (rc) return rc;
            gd = tot[LBK_C_GD];
        }
        c->spec_valid = 1;
        c->spec_f = tot[LBK_C_F];
        c->spec_dphi = tot[LBK_C_DPHI];
        memcpy(c->spec_tot, tot, sizeof tot);
    } else {
        rc = materialize_d(c);
        if (rc) return rc;
        DEVNC(lbk_fetch(c->dev, SLOT_LAST(m), 1, &gd));
        if (gd >= 0) {
            say(c, "Warning: Not a descent direction, using gradient\n");
            c->dmode = LBK_D_NEG_G;
            c->d_ready = 0;
            host_invalidate(c);
            rc = materialize_d(c);
            if (rc) return rc;
            DEVNC(lbk_fetch(c->dev, SLOT_LAST(m), 1, &gd));
        }
    }

    double alpha = 0.0;
    c->search_cslot = (!ext_obj(c) && !c->unfused) ? cslot : -1; /* a device search may commit */
    c->search_committed = 0;
    c->recommit_a0 = 0;
    rc = run_line_search(c, gd, &alpha);
    c->search_cslot = -1;
    if (rc) return rc;
    if (c->flags & LBFGS_FLAG_TRACE) c->tr_a[c->tr_len - 1] = alpha;

    /* ---- commit (:159-198) ---- */
    if (c->search_committed) {
        /* the device search's launch committed at its step already (the commit below, D_BUF):
         * its totals, then iteration k + 1 queued behind it as commit_queued would */
        if (small_done && c->spec_on) {
            rc = spec_drop(c);
            if (rc) return rc;
        }
        DEVNC(lbk_fetch(c->dev, cslot, 7, tot));
        c->commits++;
        if (small_done && c->spec_on && alpha >= 1e-10) {
            rc = spec_next(c, alpha);
            if (rc) return rc;
        }
    } else if (!(c->spec_valid && alpha == c->a0) || c->recommit_a0) {
        /* batched: d may still be unmaterialised (formed on the fly again, same bits) */
        if (!(c->batch && !c->unfused && !ext_obj(c) && !c->d_ready &&
              (c->dmode == LBK_D_TWOLOOP || (c->dmode == LBK_D_NEG_G && c->geo->world == 1)))) {
            rc = materialize_d(c);
            if (rc) return rc;
        }
        if (small_done && c->spec_on) { /* the next iteration queued behind the recommit */
            rc = spec_drop(c);
            if (!rc) rc = commit_queued(c, c->d_ready ? LBK_D_BUF : c->dmode, alpha, cslot, tot);
        } else {
            rc = commit(c, c->d_ready ? LBK_D_BUF : c->dmode, alpha, cslot, tot, 0.0);
        }
        if (rc) return rc;
    }
    c->f_cur = tot[LBK_C_F];
    c->sp_hostgo = alpha == c->sp_alpha && tot[LBK_C_SY] > 0; /* what a queued launch of k + 1 assumed */
    if (alpha < 1e-10) { /* :164-168 */
        say(c, "Warning: Line search failed at iteration %d\n", k);
        c->status = LBFGS_STATUS_LS_FAILED;
        return 1;
    }
    const double sy = tot[LBK_C_SY];
    if (sy > 0) { /* :182-191 */
        const int pair = c->free_pair;
        if (c->h >= m) {
            const int oldest = c->ring[0];
            for (int i = 0; i + 1 < m; ++i) c->ring[i] = c->ring[i + 1];
            c->ring[m - 1] = pair;
            c->free_pair = oldest;
        } else {
            c->ring[c->h++] = pair;
            c->free_pair = c->h; /* pool slots 0..h-1 used, h is free */
        }
        c->sy[pair] = sy;
        c->yy[pair] = tot[LBK_C_YY];
        c->sg_valid = !c->unfused;
        c->sg_ref = REF(cslot, LBK_C_SG);
    } else {
        say(c, "Warning: Skipping update, sy = %g\n", sy); /* :192-195 */
        c->sg_valid = 0;
    }
    /* x = x_new, g = g_new (:197-198) */
    double* t = c->x;
    c->x = c->xn;
    c->xn = t;
    t = c->g;
    c->g = c->gn;
    c->gn = t;
    c->gg = tot[LBK_C_GG];
    c->k++;
    return 0;
}


/* ------------------------------------------------------------------------------------------
 * Vector-free mode (LBFGS_FLAG_VECTOR_FREE; outside the bit-parity contract with the
 * reference's operation order). lbfgs.cpp:87-143's two-loop recursion runs
 * on the host over the Gram matrix of the basis [s_0..s_{h-1}, y_0..y_{h-1}, g] (q and r are
 * coefficient vectors); one device pass forms d from the basis, takes the first trial and the
 * commit, and reduces g_new and y_new against the basis. The s_new row is derived,
 * s_new . v = alpha (d . v). Every sum below runs over s terms (ring order), then y terms, then
 * the g term, starting from 0.0 (oracle/lbfgs_oracle.c restates it in the same order).
 * ---------------------------------------------------------------------------------------- */
#define GI(c, p, q) ((p) * ((c)->m + 1) + (q))

/* coefficient vector (ds, dy, dg) dotted with basis vector s_{ring i} or y_{ring i} */
static double vf_dot_s(const lbfgs_ctx* c, int i, const double* ds, const double* dy, double dg) {
    const int ri = c->ring[i];
    double a = 0.0;
    for (int j = 0; j < c->h; ++j) a = a + ds[j] * c->Gss[GI(c, ri, c->ring[j])];
    for (int j = 0; j < c->h; ++j) a = a + dy[j] * c->Gsy[GI(c, ri, c->ring[j])];
    return a + dg * c->Gsg[ri];
}
static double vf_dot_y(const lbfgs_ctx* c, int i, const double* ds, const double* dy, double dg) {
    const int ri = c->ring[i];
    double a = 0.0;
    for (int j = 0; j < c->h; ++j) a = a + ds[j] * c->Gsy[GI(c, c->ring[j], ri)];
    for (int j = 0; j < c->h; ++j) a = a + dy[j] * c->Gyy[GI(c, ri, c->ring[j])];
    return a + dg * c->Gyg[ri];
}

static int vf_commit(lbfgs_ctx* c, double alpha, double* tot) {
    int hb = 0;
    DEV(lbk_vf_commit(c->dev, c->obj, c->vf_h, c->x, c->g, c->vf_S, c->vf_Y, c->vf_cs, c->vf_cy, c->vf_cg, alpha,
                      c->vf_cand, c->xn, c->gn, c->S[c->free_pair], c->Y[c->free_pair], LBK_WSLOT0, &hb));
    DEVNC(lbk_fetch(c->dev, LBK_WSLOT0, LBK_VF_YB + 4 * hb + LBK_VF_NA, tot));
    c->vf_hb = hb;
    c->commits++;
    return 0;
}

static int iterate_vf(lbfgs_ctx* c) {
    const int k = c->k, m = c->m, h = c->h;
    const double gnorm = sqrt(c->gg);
    int rc = trace_push(c, c->f_cur, gnorm, 1);
    if (rc) return rc;
    if (c->flags & LBFGS_FLAG_VERBOSE) {
        printf("Iteration %d, f = %g, |grad| = %g\n", k, c->f_cur, gnorm);
        fflush(stdout);
    }
    if (gnorm < c->tol) {
        say(c, "Converged!\n");
        c->status = LBFGS_STATUS_CONVERGED;
        return 1;
    }
    note_h(c);

    /* ---- direction in coefficient space (:87-143): d = -(r) with r over the basis ---- */
    c->vf_h = h;
    for (int j = 0; j < h; ++j) {
        c->vf_S[j] = c->S[c->ring[j]];
        c->vf_Y[j] = c->Y[c->ring[j]];
        c->vf_cs[j] = c->vf_cy[j] = 0.0;
    }
    c->vf_cg = -1.0;
    if (!(k == 0 || h == 0)) {
        int bad_rho = 0;
        for (int i = h - 1; i >= 0; --i)
            if (!isfinite(1.0 / c->Gsy[GI(c, c->ring[i], c->ring[i])])) bad_rho = 1;
        const int top = c->ring[h - 1];
        if (bad_rho) {
            say(c, "Warning: Invalid rho at iteration %d\n", k);
        } else {
            const double gamma = c->Gsy[GI(c, top, top)] / c->Gyy[GI(c, top, top)];
            if (gamma <= 0 || !isfinite(gamma)) {
                say(c, "Warning: Invalid gamma at iteration %d\n", k);
            } else {
                double ds[MMAX], dy[MMAX], a[MMAX], dg = 1.0;
                for (int j = 0; j < h; ++j) ds[j] = dy[j] = 0.0;
                for (int i = h - 1; i >= 0; --i) {
                    const double rho = 1.0 / c->Gsy[GI(c, c->ring[i], c->ring[i])];
                    a[i] = rho * vf_dot_s(c, i, ds, dy, dg);
                    dy[i] = dy[i] - a[i];
                }
                for (int j = 0; j < h; ++j) {
                    ds[j] = ds[j] * gamma;
                    dy[j] = dy[j] * gamma;
                }
                dg = dg * gamma;
                for (int i = 0; i < h; ++i) {
                    const double rho = 1.0 / c->Gsy[GI(c, c->ring[i], c->ring[i])];
                    const double beta = rho * vf_dot_y(c, i, ds, dy, dg);
                    ds[i] = ds[i] + (a[i] - beta);
                }
                for (int j = 0; j < h; ++j) {
                    c->vf_cs[j] = -ds[j];
                    c->vf_cy[j] = -dy[j];
                }
                c->vf_cg = -dg;
            }
        }
    }
    /* g . d from the Gram row of g */
    double gd = 0.0;
    for (int j = 0; j < h; ++j) gd = gd + c->vf_cs[j] * c->Gsg[c->ring[j]];
    for (int j = 0; j < h; ++j) gd = gd + c->vf_cy[j] * c->Gyg[c->ring[j]];
    gd = gd + c->vf_cg * c->gg;
    if (gd >= 0) { /* :146-153 */
        say(c, "Warning: Not a descent direction, using gradient\n");
        for (int j = 0; j < h; ++j) c->vf_cs[j] = c->vf_cy[j] = 0.0;
        c->vf_cg = -1.0;
        gd = 0.0;
        for (int j = 0; j < h; ++j) gd = gd + c->vf_cs[j] * c->Gsg[c->ring[j]];
        for (int j = 0; j < h; ++j) gd = gd + c->vf_cy[j] * c->Gyg[c->ring[j]];
        gd = gd + c->vf_cg * c->gg;
    }
    c->dmode = D_VF;
    c->d_ready = 0;
    c->cand_valid = 0;
    c->tc_n = 0;
    c->trial_passes = 0;
    c->gt_valid = 0;

    /* ---- fused first trial + commit at a0, then the line search (:156) ---- */
    c->a0 = c->K.initial_step;
    c->vf_cand[0] = c->a0 * c->K.backtracking_alpha; /* the steps line_search.cpp:27 would try next */
    for (int j = 1; j < LBK_VF_NA; ++j) c->vf_cand[j] = c->vf_cand[j - 1] * c->K.backtracking_alpha;
    c->vf_cand_valid = 0;
    rc = vf_commit(c, c->a0, c->vf_spec);
    if (rc) return rc;
    const double* T = c->vf_spec;
    const int gb = LBK_VF_YB + 2 * c->vf_hb; /* g_new . b_l components */
    for (int j = 0; j < LBK_VF_NA; ++j) c->vf_cand_f[j] = T[LBK_VF_YB + 4 * c->vf_hb + j];
    c->vf_cand_valid = 1;
    double dgn = 0.0;                        /* g_new . d */
    for (int j = 0; j < h; ++j) dgn = dgn + c->vf_cs[j] * T[gb + j];
    for (int j = 0; j < h; ++j) dgn = dgn + c->vf_cy[j] * T[gb + h + j];
    dgn = dgn + c->vf_cg * T[LBK_VF_GGO];
    c->spec_valid = 1;
    c->spec_f = T[LBK_VF_F];
    c->spec_dphi = dgn;

    double alpha = 0.0;
    rc = run_line_search(c, gd, &alpha);
    if (rc) return rc;
    if (c->flags & LBFGS_FLAG_TRACE) c->tr_a[c->tr_len - 1] = alpha;

    /* ---- commit (:159-198) ---- */
    if (alpha == c->a0) {
        memcpy(c->vf_tot, c->vf_spec, sizeof c->vf_tot);
    } else {
        rc = vf_commit(c, alpha, c->vf_tot);
        if (rc) return rc;
        T = c->vf_tot;
        dgn = 0.0;
        for (int j = 0; j < h; ++j) dgn = dgn + c->vf_cs[j] * T[gb + j];
        for (int j = 0; j < h; ++j) dgn = dgn + c->vf_cy[j] * T[gb + h + j];
        dgn = dgn + c->vf_cg * T[LBK_VF_GGO];
    }
    T = c->vf_tot;
    c->f_cur = T[LBK_VF_F];
    if (alpha < 1e-10) { /* :164-168 */
        say(c, "Warning: Line search failed at iteration %d\n", k);
        c->status = LBFGS_STATUS_LS_FAILED;
        return 1;
    }
    const double sy = T[LBK_VF_SY];
    const int yb = LBK_VF_YB;
    if (sy > 0) { /* :182-191 */
        const int p = c->free_pair;
        /* derived row of s_new = alpha d against the old basis (old g row) */
        double dS[MMAX], dY[MMAX];
        for (int q = 0; q < h; ++q) {
            const int rq = c->ring[q];
            double a = 0.0, b = 0.0;
            for (int j = 0; j < h; ++j) a = a + c->vf_cs[j] * c->Gss[GI(c, c->ring[j], rq)];
            for (int j = 0; j < h; ++j) a = a + c->vf_cy[j] * c->Gsy[GI(c, rq, c->ring[j])];
            dS[q] = a + c->vf_cg * c->Gsg[rq];
            for (int j = 0; j < h; ++j) b = b + c->vf_cs[j] * c->Gsy[GI(c, c->ring[j], rq)];
            for (int j = 0; j < h; ++j) b = b + c->vf_cy[j] * c->Gyy[GI(c, c->ring[j], rq)];
            dY[q] = b + c->vf_cg * c->Gyg[rq];
        }
        double dd = 0.0;
        for (int j = 0; j < h; ++j) dd = dd + c->vf_cs[j] * dS[j];
        for (int j = 0; j < h; ++j) dd = dd + c->vf_cy[j] * dY[j];
        dd = dd + c->vf_cg * gd;
        for (int q = 0; q < h; ++q) {
            const int rq = c->ring[q];
            c->Gss[GI(c, p, rq)] = c->Gss[GI(c, rq, p)] = alpha * dS[q];
            c->Gsy[GI(c, p, rq)] = alpha * dY[q];
            c->Gsy[GI(c, rq, p)] = T[yb + q];
            c->Gyy[GI(c, p, rq)] = c->Gyy[GI(c, rq, p)] = T[yb + h + q];
            c->Gsg[rq] = T[gb + q];
            c->Gyg[rq] = T[gb + h + q];
        }
        c->Gss[GI(c, p, p)] = (alpha * alpha) * dd;
        c->Gsy[GI(c, p, p)] = sy;
        c->Gyy[GI(c, p, p)] = T[LBK_VF_YY];
        c->Gsg[p] = alpha * dgn;
        c->Gyg[p] = T[LBK_VF_YG];
        if (c->h >= m) {
            const int oldest = c->ring[0];
            for (int i = 0; i + 1 < m; ++i) c->ring[i] = c->ring[i + 1];
            c->ring[m - 1] = p;
            c->free_pair = oldest;
        } else {
            c->ring[c->h++] = p;
            c->free_pair = c->h;
        }
    } else {
        say(c, "Warning: Skipping update, sy = %g\n", sy); /* :192-195 */
        for (int q = 0; q < h; ++q) {
            c->Gsg[c->ring[q]] = T[gb + q];
            c->Gyg[c->ring[q]] = T[gb + h + q];
        }
    }
    double* t = c->x;
    c->x = c->xn;
    c->xn = t;
    t = c->g;
    c->g = c->gn;
    c->gn = t;
    c->gg = T[LBK_VF_GG];
    c->k++;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* ------------------------------------------------------------------------------------------
 * LBFGS_FLAG_CUDA_COMPAT: LBFGS_CUDA of parallel-implementation/L-BFGS.cu:195-358 with the
 * line searches of parallel-implementation/line_search.cpp, on device vectors. The reference
 * reads every cuBLAS dot back to the host (host-pointer mode); so does this path (one fetch per
 * dot), and its line searches run on the host over device evaluations: f(x + a d) and
 * g(x + a d) . d by the trial kernel, f(x) by the objective kernel, g0 . d as a canonical dot.
 * ---------------------------------------------------------------------------------------- */
static int cu_dot(lbfgs_ctx* c, const double* a, const double* b, double* out) {
    DEV(lbk_dot(c->dev, a, b, SLOT_MISC(c->m)));
    DEVNC(lbk_fetch(c->dev, SLOT_MISC(c->m), 1, out));
    return 0;
}

static int cu_fx(lbfgs_ctx* c, double* f) { /* f(x): the objective kernel, its gradient into scratch */
    double t[2];
    DEV(lbk_eval(c->dev, c->obj, c->x, c->gt, SLOT_TRIAL(c->m)));
    DEVNC(lbk_fetch(c->dev, SLOT_TRIAL(c->m), 2, t));
    *f = t[0];
    c->trials_f++;
    return 0;
}

static int cu_ft(lbfgs_ctx* c, double a, double* f, double* gnd) { /* f(x + a d) [, g(x + a d) . d] */
    double t[2];
    DEV(lbk_trial(c->dev, c->obj, c->x, c->d, a, gnd ? c->gt : NULL, SLOT_TRIAL(c->m)));
    DEVNC(lbk_fetch(c->dev, SLOT_TRIAL(c->m), gnd ? 2 : 1, t));
    *f = t[0];
    if (gnd) {
        *gnd = t[1];
        c->trials_fg++;
    } else {
        c->trials_f++;
    }
    return 0;
}

#define CU(call)                    \
    do {                            \
        const int rc_ = (call);     \
        if (rc_) return rc_;        \
    } while (0)

static int cu_backtracking(lbfgs_ctx* c, double gd, double* out) { /* line_search.cpp:21-40 */
    const lbfgs_constants* K = &c->K;
    double fx, ft, alpha = K->initial_step;
    CU(cu_fx(c, &fx)); /* the reference re-evaluates f(x) per trial: the same value */
    for (;;) {
        CU(cu_ft(c, alpha, &ft, NULL));
        if (!(fx - ft < K->c1 * alpha * gd)) break;
        alpha *= K->backtracking_alpha;
        if (alpha < K->backtracking_tol) break;
    }
    *out = alpha < 1e-4 ? 0.5 : alpha;
    return 0;
}

static int cu_backtracking_wolfe(lbfgs_ctx* c, double gd, double* out) { /* :42-147, its own constants */
    const double C1 = 1e-4, C2 = 0.9, TOL = 1e-10;
    double alpha = 1.0, f_current, alpha_lo = 0.0, alpha_hi = DBL_MAX;
    double ca[24], cf[24]; /* the search's cache of f by alpha */
    int nc = 0, iter = 0;
    CU(cu_fx(c, &f_current));
    while (iter++ < 20) {
        int hit = -1;
        for (int j = 0; j < nc; ++j)
            if (ca[j] == alpha) hit = j;
        double f_new;
        if (hit >= 0) {
            f_new = cf[hit];
        } else {
            CU(cu_ft(c, alpha, &f_new, NULL));
            if (nc < 24) {
                ca[nc] = alpha;
                cf[nc++] = f_new;
            }
        }
        if (f_new <= f_current + C1 * alpha * gd) {
            double fg, gnd;
            CU(cu_ft(c, alpha, &fg, &gnd)); /* grad(x_new) . d */
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
    *out = alpha;
    return 0;
}

static double cu_cubic(double a0, double a1, double p0, double dp0, double p1, double dp1) { /* :10-15 */
    const double d1 = dp0 + dp1 - 3 * (p1 - p0) / (a1 - a0);
    const double d2 = copysign(sqrt(d1 * d1 - dp0 * dp1), a1 - a0);
    return a0 + (a1 - a0) * (dp0 + d2 - d1) / (dp0 - dp1 + 2 * d2);
}

static double cu_quad(double a0, double p0, double dp0, double p1) { /* :17-20 */
    return a0 - 0.5 * dp0 * a0 * a0 / (p1 - p0 - dp0 * a0);
}

static int cu_interpolation(lbfgs_ctx* c, double gd, double* out) { /* :149-213 */
    const lbfgs_constants* K = &c->K;
    double f_x, alpha = K->initial_step, alpha_prev = 0.0, f_prev;
    CU(cu_fx(c, &f_x));
    f_prev = f_x;
    int it = 0;
    while (it++ < 20) {
        double f_new;
        CU(cu_ft(c, alpha, &f_new, NULL));
        if (f_new <= f_x + K->c1 * alpha * gd) {
            *out = alpha;
            return 0;
        }
        if (alpha < K->wolfe_interp_min) {
            *out = K->wolfe_interp_min;
            return 0;
        }
        if (alpha_prev > 0) {
            const double delta = alpha - alpha_prev;
            if (fabs(delta) < 1e-10) {
                alpha *= 0.5;
            } else {
                const double ga = (f_new - f_x - gd * alpha) / (alpha * alpha);
                alpha = cu_cubic(alpha_prev, alpha, f_prev, gd, f_new, ga);
                if (alpha < 0.1 * alpha_prev || alpha > 0.9 * alpha_prev) alpha = alpha_prev * 0.5;
            }
        } else {
            alpha = cu_quad(alpha, f_new, gd, f_x);
            if (alpha < 0.1 * K->initial_step || alpha > 0.9 * K->initial_step) alpha = K->initial_step * 0.5;
        }
        alpha_prev = alpha;
        f_prev = f_new;
    }
    *out = alpha < 1e-4 ? 0.5 : alpha;
    return 0;
}

/* :216-275: endpoints sorted, the midpoint whenever a step is not finite or the cubic has no
 * real minimiser, the result kept 10 % inside the bracket */
static double cu_safe_cubic(double a0, double a1, double p0, double dp0, double p1, double dp1) {
    if (a0 > a1) {
        double t = a0;
        a0 = a1;
        a1 = t;
        t = p0;
        p0 = p1;
        p1 = t;
        t = dp0;
        dp0 = dp1;
        dp1 = t;
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
    const double mn = (r < hi) ? r : hi; /* std::min(hi, r) */
    return (lo < mn) ? mn : lo;          /* std::max(lo, .) */
}

static int cu_wolfe(lbfgs_ctx* c, double gd, double* out) { /* :277-368 */
    const lbfgs_constants* K = &c->K;
    double f_x, alpha = K->initial_step;
    CU(cu_fx(c, &f_x));
    double alpha_lo = 0.0, alpha_hi = INFINITY, f_lo = f_x, dphi_lo = gd;
    for (int iter = 0; iter < 20; ++iter) {
        double f_new;
        CU(cu_ft(c, alpha, &f_new, NULL));
        if (f_new > f_x + K->c1 * alpha * gd || (f_new >= f_lo && iter > 0)) {
            alpha_hi = alpha;
            alpha = cu_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, (f_new - f_x - gd * alpha) / (alpha * alpha));
            continue;
        }
        double fg, dphi_new;
        CU(cu_ft(c, alpha, &fg, &dphi_new)); /* grad(x_new) . d */
        if (fabs(dphi_new) <= -K->c2 * gd) {
            *out = alpha;
            return 0;
        }
        if (dphi_new >= 0) {
            alpha_hi = alpha;
            alpha = cu_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        } else {
            alpha_lo = alpha;
            f_lo = f_new;
            dphi_lo = dphi_new;
            if (alpha_hi == INFINITY)
                alpha *= 2;
            else
                alpha = cu_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        }
        if (alpha < K->wolfe_interp_min) {
            *out = K->wolfe_interp_min;
            return 0;
        }
    }
    *out = alpha;
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * LBFGS_FLAG_CUDA_VARIANT: the inline searches of the four variant files. Each trial transfers
 * x + a d to the host copy x_host, so f(x_host) at the next iteration is the f of the last trial
 * point transferred (cv_fhost), not f(x). ok = the search's line_search_success.
 * ---------------------------------------------------------------------------------------- */
static int cv_backtracking(lbfgs_ctx* c, double gd, double* out) { /* L-BFGS-Backtracking.cu:293-341 */
    const double C1 = 1e-4, TOL = 1e-10; /* :153-156, the file's own constants */
    double fx, ft, step = 1.0;
    CU(cu_fx(c, &fx)); /* f(x_host), x_host freshly copied from d_x */
    for (;;) {
        CU(cu_ft(c, step, &ft, NULL));
        if (ft <= fx + C1 * step * gd) break;
        step *= 0.5;
        if (step < TOL) {
            step = 0.5;
            break;
        }
    }
    *out = step;
    return 0;
}

static int cv_interpolation(lbfgs_ctx* c, double gd, double* out, int* ok) { /* L-BFGS-Interpolation.cu:259-342 */
    const lbfgs_constants* K = &c->K;
    const double f_x = c->cv_fhost;
    double alpha = K->initial_step, alpha_prev = 0.0, f_prev = c->cv_f0;
    *ok = 0;
    for (int iter = 0; iter < 20; ++iter) {
        double f_new;
        CU(cu_ft(c, alpha, &f_new, NULL));
        c->cv_fhost = f_new;
        if (f_new <= f_x + K->c1 * alpha * gd) {
            *ok = 1;
            break;
        }
        if (alpha < K->wolfe_interp_min) {
            alpha = K->wolfe_interp_min;
            break;
        }
        if (alpha_prev > 0) {
            const double delta = alpha - alpha_prev;
            if (fabs(delta) < 1e-10) {
                alpha *= 0.5;
            } else {
                const double ga = (f_new - f_x - gd * alpha) / (alpha * alpha);
                double next = cu_cubic(alpha_prev, alpha, f_prev, gd, f_new, ga);
                if (next < 0.1 * alpha_prev || next > 0.9 * alpha_prev) next = alpha_prev * 0.5;
                alpha = next;
            }
        } else {
            double next = cu_quad(alpha, f_new, gd, f_x);
            if (next < 0.1 * K->initial_step || next > 0.9 * K->initial_step) next = K->initial_step * 0.5;
            alpha = next;
        }
        alpha_prev = alpha; /* after the update (:335) */
        f_prev = f_new;
    }
    if (alpha < 1e-4) alpha = 0.5; /* :339-342 */
    *out = alpha;
    return 0;
}

static int cv_wolfe(lbfgs_ctx* c, double gd, double* out, int* ok) { /* L-BFGS-Wolfe.cu:259-349 */
    const lbfgs_constants* K = &c->K;
    const double f_x = c->cv_fhost;
    double alpha = K->initial_step, alpha_lo = 0.0, alpha_hi = INFINITY, f_lo = c->cv_f0, dphi_lo = gd;
    *ok = 0;
    for (int iter = 0; iter < 20; ++iter) {
        double f_new;
        CU(cu_ft(c, alpha, &f_new, NULL));
        c->cv_fhost = f_new;
        if (f_new > f_x + K->c1 * alpha * gd || (f_new >= f_lo && iter > 0)) {
            alpha_hi = alpha;
            alpha = cu_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, (f_new - f_x - gd * alpha) / (alpha * alpha));
            continue; /* past the WOLFE_INTERP_MIN floor */
        }
        double fg, dphi_new;
        CU(cu_ft(c, alpha, &fg, &dphi_new)); /* grad(x_host) . d */
        if (fabs(dphi_new) <= -K->c2 * gd) {
            *ok = 1;
            break;
        }
        if (dphi_new >= 0) {
            alpha_hi = alpha;
            alpha = cu_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        } else {
            alpha_lo = alpha;
            f_lo = f_new;
            dphi_lo = dphi_new;
            if (alpha_hi == INFINITY)
                alpha *= 2;
            else
                alpha = cu_safe_cubic(alpha_lo, alpha_hi, f_lo, dphi_lo, f_new, dphi_new);
        }
        if (alpha < K->wolfe_interp_min) {
            alpha = K->wolfe_interp_min;
            break;
        }
    }
    *out = alpha;
    return 0;
}

static int cv_backtracking_wolfe(lbfgs_ctx* c, double gd, double* out, int* ok) { /* L-BFGS-Backtracking_Wolfe.cu:256-397 */
    const double C1 = 1e-4, C2 = 0.9, TOL = 1e-10; /* :261-264, the file's own constants */
    const double f_x = c->cv_fhost;
    double alpha = 1.0, alpha_lo = 0.0, alpha_hi = DBL_MAX;
    double ca[24], cf[24], cgd[24]; /* cache: f by alpha, and g(x + alpha d) . d once evaluated */
    int cg[24], nc = 0;
    *ok = 0;
    for (int iter = 0; iter < 20; ++iter) {
        int hit = -1;
        for (int j = 0; j < nc; ++j)
            if (ca[j] == alpha) hit = j;
        if (hit < 0) {
            double f_new;
            CU(cu_ft(c, alpha, &f_new, NULL));
            c->cv_fhost = f_new;
            hit = nc++;
            ca[hit] = alpha;
            cf[hit] = f_new;
            cg[hit] = 0;
        }
        if (cf[hit] <= f_x + C1 * alpha * gd) {
            if (!cg[hit]) { /* x + alpha d transferred again, its gradient evaluated */
                double fg;
                c->cv_fhost = cf[hit];
                CU(cu_ft(c, alpha, &fg, &cgd[hit]));
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
            double f_t;
            alpha = TOL;
            CU(cu_ft(c, alpha, &f_t, NULL));
            c->cv_fhost = f_t;
            break;
        }
    }
    *out = alpha;
    return 0;
}

/* one iteration k of L-BFGS.cu:195-358; returns 1 when the solve ended */
static int iterate_cuda(lbfgs_ctx* c) {
    const int k = c->k, m = c->m;
    if (k == 0) {
        DEV(lbk_elementwise(c->dev, 2, c->d, c->g, NULL, 0.0)); /* negateVector :208 */
    } else {
        DEVNC(lbk_copy(c->dev, c->q, c->g)); /* :212 */
        const int lo = k - m > 0 ? k - m : 0;
        for (int i = k - 1; i >= lo; --i) { /* :216-235 */
            const int sl = i % m;
            if (c->sy[sl] <= 1e-10) continue; /* alpha[sl], rho[sl] keep their last values */
            c->cu_rho[sl] = 1.0 / c->sy[sl];
            double sq;
            CU(cu_dot(c, c->S[sl], c->q, &sq));
            c->cu_alpha[sl] = c->cu_rho[sl] * sq;
            DEV(lbk_elementwise(c->dev, 3, c->q, c->q, c->Y[sl], -c->cu_alpha[sl])); /* daxpy */
        }
        const int last = (k - 1) % m; /* :237-262 */
        const double ys = c->sy[last], yy = c->yy[last];
        const double gamma = (yy > 0 && ys > 1e-10) ? ys / yy : 1.0;
        DEV(lbk_elementwise(c->dev, 0, c->r, c->q, NULL, gamma)); /* scaleByRho */
        for (int i = lo; i < k; ++i) { /* :264-274 */
            const int sl = i % m;
            double yr;
            CU(cu_dot(c, c->Y[sl], c->r, &yr));
            const double beta = c->cu_rho[sl] * yr;
            const double diff = c->cu_alpha[sl] - beta;
            DEV(lbk_elementwise(c->dev, 3, c->r, c->r, c->S[sl], diff));
        }
        DEV(lbk_elementwise(c->dev, 2, c->d, c->r, NULL, 0.0)); /* :276 */
    }
    double gd, step;
    if (c->cuda == 2) { /* the variants: the current gradient (d_g), their own searches */
        int ok = 1;
        CU(cu_dot(c, c->g, c->d, &gd));
        switch (c->ls) {
            case LBFGS_LS_BACKTRACKING: CU(cv_backtracking(c, gd, &step)); break;
            case LBFGS_LS_INTERPOLATION: CU(cv_interpolation(c, gd, &step, &ok)); break;
            case LBFGS_LS_WOLFE: CU(cv_wolfe(c, gd, &step, &ok)); break;
            default: CU(cv_backtracking_wolfe(c, gd, &step, &ok)); break;
        }
        say(c, "alpha: %g\n", step);
        if (c->ls == LBFGS_LS_BACKTRACKING) {
            if (step < 1e-4) /* L-BFGS-Backtracking.cu:345-348 */
                say(c, "Warning: Line search resulted in very small step size at iteration %d\n", k);
        } else if (!ok && step < 1e-10) { /* e.g. L-BFGS-Wolfe.cu:353-366 */
            say(c, "Warning: Line search failed at iteration %d\n", k);
            c->status = LBFGS_STATUS_LS_FAILED;
            return 1;
        }
    } else { /* the line search with the iteration-0 gradient (:199, :293) */
        CU(cu_dot(c, c->g0c, c->d, &gd));
        switch (c->ls) {
            case LBFGS_LS_BACKTRACKING: CU(cu_backtracking(c, gd, &step)); break;
            case LBFGS_LS_INTERPOLATION: CU(cu_interpolation(c, gd, &step)); break;
            case LBFGS_LS_WOLFE: CU(cu_wolfe(c, gd, &step)); break;
            default: CU(cu_backtracking_wolfe(c, gd, &step)); break;
        }
        if (step < 1e-10) { /* :295-306 */
            say(c, "Warning: Line search failed at iteration %d\n", k);
            c->status = LBFGS_STATUS_LS_FAILED;
            return 1;
        }
        say(c, "alpha: %g\n", step); /* :308 */
    }
    DEV(lbk_point(c->dev, c->xn, c->x, c->d, step)); /* updateSolution :310 */
    double t[2];
    DEV(lbk_eval(c->dev, c->obj, c->xn, c->gn, SLOT_COMMIT0)); /* grad(x_new) :323, f(x_new) :348 */
    DEVNC(lbk_fetch(c->dev, SLOT_COMMIT0, 2, t));
    const int sl = k % m; /* updateVectors :332, whatever s.y */
    DEV(lbk_elementwise(c->dev, 3, c->S[sl], c->xn, c->x, -1.0));
    DEV(lbk_elementwise(c->dev, 3, c->Y[sl], c->gn, c->g, -1.0));
    CU(cu_dot(c, c->S[sl], c->Y[sl], &c->sy[sl])); /* the next iteration's ddot(s, y) and ddot(y, y) */
    CU(cu_dot(c, c->Y[sl], c->Y[sl], &c->yy[sl]));
    {
        double* tp = c->x; /* :335-340 */
        c->x = c->xn;
        c->xn = tp;
        tp = c->g;
        c->g = c->gn;
        c->gn = tp;
    }
    c->commits++;
    c->f_cur = t[0];
    c->gg = t[1];
    const double norm_g = sqrt(t[1]); /* :342-345 */
    say(c, "Iteration %d: norm_g = %g\n", k, norm_g);
    say(c, "Optimum value: %g\n", t[0]);
    if (c->flags & LBFGS_FLAG_TRACE) {
        CU(trace_push(c, t[0], norm_g, 1));
        c->tr_a[c->tr_len - 1] = step;
    }
    const int h = k + 1 < m ? k + 1 : m; /* ring slots written */
    if (c->h_min < 0 || h < c->h_min) c->h_min = h;
    if (h > c->h_max) c->h_max = h;
    c->k++;
    if (norm_g <= c->tol) { /* :353-357 */
        say(c, "Convergence achieved at iteration %d\n", k);
        c->status = LBFGS_STATUS_CONVERGED;
        return 1;
    }
    return 0;
}
#undef CU

int lbfgs_solver_init(lbfgs_ctx* c, int objective, const lbfgs_host_fn* cb, int line_search,
                      const lbfgs_constants* k, const double* x0_host, double tolerance,
                      unsigned flags) {
    if (!c || !x0_host) return LBFGS_ERR_BAD_ARG;
    if (objective < 0 || objective > LBFGS_OBJ_DENSE_QUAD) return LBFGS_ERR_BAD_ARG;
    if (line_search < 0 || line_search > LBFGS_LS_BACKTRACKING_WOLFE) return LBFGS_ERR_BAD_ARG;
    if (objective == LBFGS_OBJ_DENSE_QUAD && !c->dense_set) return LBFGS_ERR_STATE;
    c->refcalls = (flags & LBFGS_FLAG_REFERENCE_CALLS) != 0;
    if (objective == LBFGS_OBJ_HOST) {
        if (!cb || !cb->f || !cb->grad || c->geo->world != 1) return LBFGS_ERR_BAD_ARG;
        c->cb = *cb;
        if (host_bufs(c)) return LBFGS_ERR_NOMEM;
    }
    host_invalidate(c);
    c->hxx_valid = 0;
    c->cb_f = c->cb_g = 0;
    {
        const int rc = spec_drop(c);
        if (rc) return rc;
    }
    /* speculative next iteration at small n (LBFGS_SPEC=0: off; the same iterates either way) */
    c->spec_on = 1;
    {
        const char* e = getenv("LBFGS_SPEC");
        if (e) c->spec_on = atoi(e) != 0;
    }
    c->cur_epoch = 0;
    c->cur_spec = 0;
    c->sp_adopted = c->sp_dropped = 0;
    c->search_launches = c->search_commits = 0;
    c->unfused = (flags & LBFGS_FLAG_UNFUSED) != 0;
    c->batch = 1;
    {
        const char* e = getenv("LBFGS_BATCH");
        if (e) c->batch = atoi(e) != 0;
    }
    if (c->unfused && (objective >= LBFGS_OBJ_HOST || c->geo->world != 1)) return LBFGS_ERR_BAD_ARG;
    c->vf = (flags & LBFGS_FLAG_VECTOR_FREE) != 0;
    if (c->vf) {
        if (c->unfused || objective >= LBFGS_OBJ_HOST || c->m > LBK_VF_HMAX) return LBFGS_ERR_BAD_ARG;
        const size_t P = (size_t)c->m + 1;
        if (!c->Gss) {
            c->Gss = (double*)calloc(P * P, sizeof(double));
            c->Gsy = (double*)calloc(P * P, sizeof(double));
            c->Gyy = (double*)calloc(P * P, sizeof(double));
            c->Gsg = (double*)calloc(P, sizeof(double));
            c->Gyg = (double*)calloc(P, sizeof(double));
            if (!c->Gss || !c->Gsy || !c->Gyy || !c->Gsg || !c->Gyg) return LBFGS_ERR_NOMEM;
        }
    }
    c->cuda = (flags & LBFGS_FLAG_CUDA_COMPAT) != 0;
    if ((flags & LBFGS_FLAG_CUDA_VARIANT) && !c->cuda) return LBFGS_ERR_BAD_ARG;
    if (c->cuda && (flags & LBFGS_FLAG_CUDA_VARIANT)) c->cuda = 2;
    if (c->cuda) {
        if (c->unfused || c->vf || objective >= LBFGS_OBJ_HOST || c->geo->world != 1) return LBFGS_ERR_BAD_ARG;
        if (!c->g0c && !(c->g0c = lbk_vec_alloc(c->dev))) return LBFGS_ERR_NOMEM;
        memset(c->cu_alpha, 0, sizeof c->cu_alpha); /* L-BFGS.cu:191-192: vector<double> alpha(m), rho(m) */
        memset(c->cu_rho, 0, sizeof c->cu_rho);
    }
    c->obj = objective;
    c->ls = line_search;
    if (k)
        c->K = *k;
    else
        lbfgs_constants_default(&c->K);
    c->tol = tolerance;
    c->flags = flags;
    c->k = 0;
    c->h = 0;
    c->free_pair = 0;
    c->sg_valid = 0;
    c->status = LBFGS_STATUS_RUNNING;
    c->finished = 0;
    c->msg_len = 0;
    if (c->msg) c->msg[0] = 0;
    c->tr_len = 0;
    c->trials_f = c->trials_fg = c->commits = c->passes = 0;

    DEVNC(lbk_upload(c->dev, c->x, x0_host)); /* x = x0 */
    if (objective == LBFGS_OBJ_HOST) {         /* :29-30 */
        c->f_cur = c->cb.f(x0_host, c->n, c->cb.user);
        const int b = c->hg_cur;
        c->hg_cur ^= 1;
        DEVNC(lbk_xfer_wait(c->dev, XF_G0 + b));
        c->cb.grad(x0_host, c->n, c->hg[b], c->cb.user);
        c->cb_f++;
        c->cb_g++;
        DEVNC(lbk_upload_local(c->dev, c->g, c->hg[b]));
        DEV(lbk_dot(c->dev, c->g, c->g, SLOT_INIT));
        DEVNC(lbk_fetch(c->dev, SLOT_INIT, 1, &c->gg));
    } else {
        double t[2];
        if (objective == LBFGS_OBJ_DENSE_QUAD)
            DEV(lbk_dense_eval(c->dev, c->x, c->g, SLOT_INIT));
        else
            DEV(lbk_eval(c->dev, objective, c->x, c->g, SLOT_INIT));
        DEVNC(lbk_fetch(c->dev, SLOT_INIT, 2, t));
        c->f_cur = t[0];
        c->gg = t[1];
        if (c->vf) DEVNC(lbk_vf_ghost_init(c->dev, c->x, c->g, LBK_WSLOT0));
    }
    if (c->cuda) { /* L-BFGS.cu:115, :199 - the host gradient every line search will be given */
        DEVNC(lbk_copy(c->dev, c->g0c, c->g));
        c->cv_f0 = c->cv_fhost = c->f_cur; /* the variants' initial_f = f(x_host), x_host = x0 */
        say(c, "Starting\n");
    }
    c->inited = 1;
    return 0;
}

static void fill_result(lbfgs_ctx* c, lbfgs_result* out, double t0, double b0) {
    if (!out) return;
    out->iterations = c->k;
    out->status = c->status;
    out->f = c->f_cur;
    out->gnorm = sqrt(c->gg);
    out->trials_f = c->trials_f;
    out->trials_fg = c->trials_fg;
    out->commits = c->commits;
    out->passes = c->passes;
    out->bytes = lbk_bytes_moved(c->dev) - b0;
    out->seconds = now_s() - t0;
    out->h_min = c->h_min;
    out->h_max = c->h_min < 0 ? -1 : c->h_max;
    out->f_calls = c->cb_f;
    out->grad_calls = c->cb_g;
}

int lbfgs_solver_step(lbfgs_ctx* c, int max_steps, lbfgs_result* out) {
    if (!c || !c->inited) return LBFGS_ERR_STATE;
    const double t0 = now_s(), b0 = lbk_bytes_moved(c->dev);
    c->h_min = -1;
    c->h_max = -1;
    if (!c->finished) {
        for (int s = 0; s < max_steps; ++s) {
            c->steps_left = max_steps - s - 1;
            TRACE_PUSH("lbfgs iteration");
            int rc = c->cuda ? iterate_cuda(c) : c->vf ? iterate_vf(c) : iterate(c);
            TRACE_POP();
            if (rc < 0) {
                (void)spec_drop(c);
                return rc;
            }
            if (rc == 1) {
                c->finished = 1;
                break;
            }
        }
        int rc = spec_drop(c);
        if (rc) return rc;
    }
    fill_result(c, out, t0, b0);
    return c->finished ? c->status : LBFGS_STATUS_RUNNING;
}

int lbfgs_get_x(lbfgs_ctx* c, double* x_out_host) {
    if (!c || !x_out_host) return LBFGS_ERR_BAD_ARG;
    DEVNC(lbk_download(c->dev, x_out_host, c->x));
    return 0;
}

int lbfgs_minimize(lbfgs_ctx* c, int objective, const lbfgs_host_fn* cb, int line_search,
                   const lbfgs_constants* k, const double* x0_host, double* x_out_host,
                   int max_iterations, double tolerance, unsigned flags, lbfgs_result* out) {
    const double t0 = now_s();
    if (!c) return LBFGS_ERR_BAD_ARG;
    const double b0 = lbk_bytes_moved(c->dev);
    int rc = lbfgs_solver_init(c, objective, cb, line_search, k, x0_host, tolerance, flags);
    if (rc) return rc;
    rc = lbfgs_solver_step(c, max_iterations, NULL); /* sets h_min / h_max for the whole solve */
    if (rc < 0) return rc;
    if (!c->finished) { /* :201-202 (the CUDA path's loop just ends, L-BFGS.cu:358-365) */
        if (!c->cuda) {
            rc = trace_push(c, c->f_cur, sqrt(c->gg), 1);
            if (rc) return rc;
            say(c, "Maximum iterations reached\n");
        }
        c->status = LBFGS_STATUS_MAX_ITER;
        c->finished = 1;
    }
    if (x_out_host) {
        rc = lbfgs_get_x(c, x_out_host);
        if (rc) return rc;
    }
    fill_result(c, out, t0, b0);
    return c->status;
}

int lbfgs_messages(const lbfgs_ctx* c, char* buf, int cap) {
    if (!c || !buf || cap <= 0) return LBFGS_ERR_BAD_ARG;
    int k = c->msg_len < cap - 1 ? c->msg_len : cap - 1;
    if (k > 0) memcpy(buf, c->msg, (size_t)k);
    buf[k] = 0;
    return c->msg_len;
}

int lbfgs_trace_len(const lbfgs_ctx* c) { return c ? c->tr_len : 0; }

int lbfgs_trace_enable(lbfgs_ctx* c, int on) {
    if (!c || !c->inited) return LBFGS_ERR_STATE;
    if (on)
        c->flags |= LBFGS_FLAG_TRACE;
    else
        c->flags &= ~LBFGS_FLAG_TRACE;
    return 0;
}

int lbfgs_trace_get(const lbfgs_ctx* c, double* f, double* gnorm, double* alpha, uint64_t* c1,
                    uint64_t* c2, int cap) {
    if (!c) return LBFGS_ERR_BAD_ARG;
    int k = c->tr_len < cap ? c->tr_len : cap;
    for (int i = 0; i < k; ++i) {
        if (f) f[i] = c->tr_f[i];
        if (gnorm) gnorm[i] = c->tr_gn[i];
        if (alpha) alpha[i] = c->tr_a[i];
        if (c1) c1[i] = c->tr_c1[i];
        if (c2) c2[i] = c->tr_c2[i];
    }
    return k;
}

/* ------------------------------------------------------------------------------------------
 * Device primitives over host buffers (tests, drop-in vector_utils). They use the context's
 * work vectors and therefore end any solve in progress.
 * ---------------------------------------------------------------------------------------- */
int lbfgs_dev_dot(lbfgs_ctx* c, const double* a, const double* b, double* out) {
    if (!c || !a || !b || !out) return LBFGS_ERR_BAD_ARG;
    c->inited = 0;
    DEVNC(lbk_upload(c->dev, c->q, a));
    DEVNC(lbk_upload(c->dev, c->r, b));
    DEV(lbk_dot(c->dev, c->q, c->r, SLOT_MISC(c->m)));
    DEVNC(lbk_fetch(c->dev, SLOT_MISC(c->m), 1, out));
    return 0;
}

int lbfgs_dev_norm(lbfgs_ctx* c, const double* v, double* out) {
    if (!c || !v || !out) return LBFGS_ERR_BAD_ARG;
    double t;
    int rc = lbfgs_dev_dot(c, v, v, &t);
    if (rc) return rc;
    *out = sqrt(t);
    return 0;
}

int lbfgs_dev_objective(lbfgs_ctx* c, int obj, const double* x, double* f_out, double* g_out) {
    if (!c || !x || obj < 0 || obj == LBFGS_OBJ_HOST || obj > LBFGS_OBJ_DENSE_QUAD) return LBFGS_ERR_BAD_ARG;
    if (obj == LBFGS_OBJ_DENSE_QUAD && !c->dense_set) return LBFGS_ERR_STATE;
    c->inited = 0;
    double t[2];
    DEVNC(lbk_upload(c->dev, c->q, x));
    if (obj == LBFGS_OBJ_DENSE_QUAD)
        DEV(lbk_dense_eval(c->dev, c->q, c->gt, SLOT_MISC(c->m)));
    else
        DEV(lbk_eval(c->dev, obj, c->q, c->gt, SLOT_MISC(c->m)));
    DEVNC(lbk_fetch(c->dev, SLOT_MISC(c->m), 2, t));
    if (f_out) *f_out = t[0];
    if (g_out) DEVNC(lbk_download(c->dev, g_out, c->gt));
    return 0;
}

int lbfgs_dev_trial(lbfgs_ctx* c, int obj, const double* x, const double* d, double alpha,
                    double* f_out, double* g_out, double* dphi_out) {
    if (!c || !x || !d || obj < 0 || obj >= LBFGS_OBJ_HOST) return LBFGS_ERR_BAD_ARG;
    c->inited = 0;
    double t[2];
    DEVNC(lbk_upload(c->dev, c->q, x));
    DEVNC(lbk_upload(c->dev, c->d, d));
    DEV(lbk_trial(c->dev, obj, c->q, c->d, alpha, g_out ? c->gt : NULL, SLOT_MISC(c->m)));
    DEVNC(lbk_fetch(c->dev, SLOT_MISC(c->m), 2, t));
    if (f_out) *f_out = t[0];
    if (dphi_out) *dphi_out = t[1];
    if (g_out) DEVNC(lbk_download(c->dev, g_out, c->gt));
    return 0;
}

int lbfgs_dev_twoloop(lbfgs_ctx* c, const double* g, const double* const* S, const double* const* Y,
                      int h, double* d_out, double* gd_out) {
    if (!c || !g || h < 1 || h > c->m || !S || !Y) return LBFGS_ERR_BAD_ARG;
    c->inited = 0;
    const int m = c->m;
    DEVNC(lbk_upload(c->dev, c->g, g));
    for (int i = 0; i < h; ++i) {
        DEVNC(lbk_upload(c->dev, c->S[i], S[i]));
        DEVNC(lbk_upload(c->dev, c->Y[i], Y[i]));
        c->ring[i] = i;
        DEV(lbk_dot(c->dev, c->S[i], c->Y[i], SLOT_MISC(m)));
        DEVNC(lbk_fetch(c->dev, SLOT_MISC(m), 1, &c->sy[i]));
        DEV(lbk_dot(c->dev, c->Y[i], c->Y[i], SLOT_MISC(m)));
        DEVNC(lbk_fetch(c->dev, SLOT_MISC(m), 1, &c->yy[i]));
    }
    int refA[MMAX], refB[MMAX];
    double rho[MMAX];
    for (int i = 0; i < h; ++i) rho[i] = 1.0 / c->sy[i];
    const double gamma = c->sy[h - 1] / c->yy[h - 1];
    DEV(lbk_dot(c->dev, c->S[h - 1], c->g, SLOT_P0));
    refA[h - 1] = REF(SLOT_P0, 0);
    const double* qsrc = c->g;
    for (int i = h - 2; i >= 0; --i) {
        DEV(lbk_axpy_dot(c->dev, c->q, qsrc, c->Y[i + 1], c->S[i], rho[i + 1], refA[i + 1], SLOT_A0 + i));
        refA[i] = REF(SLOT_A0 + i, 0);
        qsrc = c->q;
    }
    DEV(lbk_mid(c->dev, c->r, qsrc, c->Y[0], rho[0], gamma, refA[0], SLOT_B0(m)));
    refB[0] = REF(SLOT_B0(m), 0);
    for (int i = 0; i + 1 < h; ++i) {
        DEV(lbk_axpy2_dot(c->dev, c->r, c->r, c->S[i], c->Y[i + 1], rho[i], refB[i], refA[i], SLOT_B0(m) + i + 1));
        refB[i + 1] = REF(SLOT_B0(m) + i + 1, 0);
    }
    DEV(lbk_last(c->dev, c->d, c->r, c->S[h - 1], c->g, rho[h - 1], refB[h - 1], refA[h - 1], SLOT_LAST(m)));
    double gd;
    DEVNC(lbk_fetch(c->dev, SLOT_LAST(m), 1, &gd));
    if (gd_out) *gd_out = gd;
    if (d_out) DEVNC(lbk_download(c->dev, d_out, c->d));
    return 0;
}

/* Line search alone (line_search.cpp:19-189) at x along d with gradient g: the same driver code
 * as inside lbfgs_minimize, with every trial evaluated on the device (or through the host
 * callbacks for LBFGS_OBJ_HOST). f(x) and g.d are evaluated once (the reference re-evaluates
 * them with identical values). Single rank. */
int lbfgs_line_search(lbfgs_ctx* c, int objective, const lbfgs_host_fn* cb, int line_search,
                      const lbfgs_constants* k, const double* x, const double* d, const double* g,
                      double* alpha_out) {
    if (!c || !x || !d || !g || !alpha_out || c->geo->world != 1) return LBFGS_ERR_BAD_ARG;
    if (objective < 0 || objective > LBFGS_OBJ_DENSE_QUAD) return LBFGS_ERR_BAD_ARG;
    if (line_search < 0 || line_search > LBFGS_LS_BACKTRACKING_WOLFE) return LBFGS_ERR_BAD_ARG;
    if (objective == LBFGS_OBJ_DENSE_QUAD && !c->dense_set) return LBFGS_ERR_STATE;
    c->refcalls = 0; /* the standalone search evaluates f(x) once (see above) */
    if (objective == LBFGS_OBJ_HOST) {
        if (!cb || !cb->f || (!cb->grad && (line_search == LBFGS_LS_WOLFE || line_search == LBFGS_LS_BACKTRACKING_WOLFE)))
            return LBFGS_ERR_BAD_ARG;
        c->cb = *cb;
        if (host_bufs(c)) return LBFGS_ERR_NOMEM;
    }
    c->cb_f = c->cb_g = 0;
    c->inited = 0;
    c->unfused = 0;
    c->batch = 1;
    {
        const char* e = getenv("LBFGS_BATCH");
        if (e) c->batch = atoi(e) != 0;
    }
    c->cand_valid = 0;
    c->tc_n = 0;
    c->trial_passes = 0;
    c->cuda = 0;
    c->obj = objective;
    c->ls = line_search;
    if (k)
        c->K = *k;
    else
        lbfgs_constants_default(&c->K);
    const int m = c->m;
    DEVNC(lbk_upload(c->dev, c->x, x));
    DEVNC(lbk_upload(c->dev, c->d, d));
    DEVNC(lbk_upload(c->dev, c->g, g));
    if (objective == LBFGS_OBJ_HOST) {
        c->f_cur = c->cb.f(x, c->n, c->cb.user);
        c->cb_f++;
    } else if (objective == LBFGS_OBJ_DENSE_QUAD) {
        DEV(lbk_dense_eval(c->dev, c->x, c->gt, SLOT_MISC(m)));
        DEVNC(lbk_fetch(c->dev, SLOT_MISC(m), 1, &c->f_cur));
    } else {
        double t[2];
        DEV(lbk_eval(c->dev, objective, c->x, NULL, SLOT_MISC(m)));
        DEVNC(lbk_fetch(c->dev, SLOT_MISC(m), 1, t));
        c->f_cur = t[0];
    }
    double gd;
    DEV(lbk_dot(c->dev, c->g, c->d, SLOT_LAST(m)));
    DEVNC(lbk_fetch(c->dev, SLOT_LAST(m), 1, &gd));
    c->dmode = LBK_D_BUF;
    c->d_ready = 1;
    c->spec_valid = 0;
    c->search_cslot = -1;
    host_invalidate(c);
    c->hxx_valid = 0;
    double alpha = 0.0;
    int rc;
    switch (line_search) {
        case LBFGS_LS_BACKTRACKING: rc = ls_backtracking(c, gd, &alpha); break;
        case LBFGS_LS_INTERPOLATION: rc = ls_interpolation(c, gd, &alpha); break;
        case LBFGS_LS_WOLFE: rc = ls_wolfe(c, gd, &alpha); break;
        default: rc = ls_backtracking_wolfe(c, gd, &alpha); break;
    }
    if (rc) return rc;
    *alpha_out = alpha;
    return 0;
}

/* vector_utils.cpp:43-73 on the device: op 0 out = alpha*a, 1 out = a+b, 2 out = -a */
int lbfgs_dev_elementwise(lbfgs_ctx* c, int op, const double* a, const double* b, double alpha,
                          double* out) {
    if (!c || !a || !out || op < 0 || op > 2 || (op == 1 && !b)) return LBFGS_ERR_BAD_ARG;
    c->inited = 0;
    DEVNC(lbk_upload(c->dev, c->q, a));
    if (op == 1) DEVNC(lbk_upload(c->dev, c->r, b));
    DEV(lbk_elementwise(c->dev, op, c->d, c->q, c->r, alpha));
    DEVNC(lbk_download(c->dev, out, c->d));
    return 0;
}

/* ---- profiling ---- */
void lbfgs_prof_enable(lbfgs_ctx* c, int on) { lbk_prof_enable(c->dev, on); }
void lbfgs_prof_reset(lbfgs_ctx* c) { lbk_prof_reset(c->dev); }
int lbfgs_prof_get(lbfgs_ctx* c, int kind, double* ms, int64_t* launches, double* bytes) {
    return lbk_prof_get(c->dev, kind, ms, launches, bytes) == 0 ? 0 : LBFGS_ERR_BAD_ARG;
}
