/* host_device_double.c — TEST DOUBLE, sanitizer job only (tests/sanitize/Makefile).
 *
 * A host-memory implementation of the device-layer interface the C driver programs against
 * (cuda-lbfgs_amd/csrc/lbfgs_device.h), so that the driver's host logic - the line searches,
 * the history ring, the slot references, the batched-trial caches, the host-callback call
 * sequencing and the C++ drop-in shim - can run under AddressSanitizer / UBSan on the CPU
 * (GPU sanitizers are not available on the MI355X pool). Every reduction is formed with the
 * oracle's canonical-order routines (oracle/lbfgs_oracle.c, compiled into this file), so a solve
 * through this double must reproduce the oracle's ORC_CANON trajectory bit for bit, which
 * tests/sanitize/san_main.c checks.
 *
 * It is never linked into liblbfgs_hip.so, never loaded by the product, bench.py or smoke();
 * the product path has no CPU fallback. One rank only; vector-free mode, sharding, the peer
 * exchange and RCCL report "unsupported".
 */
#include "../../oracle/lbfgs_oracle.c"

#include "lbfgs_device.h"

#define DBL_FRONT 8

struct lbk_ctx {
    lbk_geo geo;
    double slots[LBK_NSLOTS][LBK_GROUPS][LBK_KMAX];
    double bytes;
    char err[256];
    double* scratch[6];
    double *dA, *db; /* dense quadratic data */
    /* the small-n single-launch iteration and its speculative form (LBFGS_DOUBLE_SMALL=1; the
     * product uses it for nseg <= its cooperative limit): launches run at once, in stream order */
    int small_on;
    int twoloop_on;
    int wolfe_on; /* the device-resident line searches (LBFGS_DEV_SEARCH, with the small-n form) */
    unsigned long long epoch, vd[4];
    int rec_went[4];
    double rec_rho[4], rec_gamma[4];
};

struct lbk_group {
    int world;
};

/* ---- geometry ---- */
int lbk_geometry_plan(int64_t n, int rank, int world, lbk_geo* out) {
    if (n < 1 || world != 1 || rank != 0) return -1;
    memset(out, 0, sizeof *out);
    int64_t L, nseg;
    orc_canon_geometry(n, &L, &nseg);
    out->n = n;
    out->L = L;
    out->nseg = nseg;
    out->seg_lo = 0;
    out->seg_hi = nseg;
    out->elem_lo = 0;
    out->n_loc = n;
    out->g_lo = 0;
    out->g_hi = LBK_GROUPS;
    out->rank = 0;
    out->world = 1;
    out->vf_f = orc_vf_factor(n);
    return 0;
}
int lbk_vf_factor(int64_t n) { return orc_vf_factor(n); }

int lbk_create(lbk_ctx** out, int device, int64_t n, int rank, int world, const void* nccl_id, lbk_group* grp) {
    (void)device;
    *out = NULL;
    if (world != 1 || grp || nccl_id) return -1;
    lbk_ctx* c = (lbk_ctx*)calloc(1, sizeof *c);
    if (!c) return -4;
    if (lbk_geometry_plan(n, rank, world, &c->geo) != 0) {
        free(c);
        return -1;
    }
    for (int i = 0; i < 6; ++i) {
        c->scratch[i] = (double*)calloc((size_t)n + 2, sizeof(double));
        if (!c->scratch[i]) return -4;
    }
    const char* e = getenv("LBFGS_DOUBLE_SMALL");
    c->small_on = e && atoi(e) != 0;
    e = getenv("LBFGS_DOUBLE_TWOLOOP");  /* the driver's persistent two-loop branch (LBFGS_PERSIST=2) */
    c->twoloop_on = e && atoi(e) != 0;
    e = getenv("LBFGS_DEV_WOLFE");
    c->wolfe_on = !e || atoi(e) != 0;
    e = getenv("LBFGS_DEV_SEARCH");
    if (e) c->wolfe_on = atoi(e) != 0;
    *out = c;
    return 0;
}
void lbk_destroy(lbk_ctx* c) {
    if (!c) return;
    free(c->dA);
    free(c->db);
    for (int i = 0; i < 6; ++i) free(c->scratch[i]);
    free(c);
}
const lbk_geo* lbk_geometry(const lbk_ctx* c) { return &c->geo; }
const char* lbk_last_error(const lbk_ctx* c) { return c ? c->err : "no context"; }
int lbk_unique_id(void* out128) {
    (void)out128;
    return -3;
}
int lbk_device_count(void) { return 0; }
lbk_group* lbk_group_create(int world) {
    (void)world;
    return NULL;
}
void lbk_group_destroy(lbk_group* g) { free(g); }
void lbk_set_ghost_slot(lbk_ctx* c, int slot) {
    (void)c;
    (void)slot;
}
int lbk_peer_handle(lbk_ctx* c, void* out) {
    (void)c;
    (void)out;
    return -1;
}
int lbk_peer_connect(lbk_ctx* c, const void* h) {
    (void)c;
    (void)h;
    return -1;
}
int lbk_peer_enable(lbk_ctx* c, int on) {
    (void)c;
    (void)on;
    return -5;
}
int lbk_rccl_attach(lbk_ctx* c, const void* id) {
    (void)c;
    (void)id;
    return -1;
}
int lbk_exchange_backend(const lbk_ctx* c) {
    (void)c;
    return 0;
}

int lbk_exchange_fold(const lbk_ctx* c) {
    (void)c;
    return 0;
}
int lbk_exchange_bench(lbk_ctx* c, int b, int ks, int it, double* us) {
    (void)c, (void)b, (void)ks, (void)it, (void)us;
    return -1;
}
int lbk_cu_partition(const lbk_ctx* c) {
    (void)c;
    return 0;
}
int lbk_coop_info(const lbk_ctx* c, int* a, int* b, int* f) {
    (void)c;
    if (a) *a = 0;
    if (b) *b = 0;
    if (f) *f = 0;
    return 0;
}
int lbk_vec_fallbacks(const lbk_ctx* c) {
    (void)c;
    return 0;
}
int lbk_vec_pool_stats(const lbk_ctx* c, int* pooled, double* held_gb) {
    (void)c;
    if (pooled) *pooled = 0;
    if (held_gb) *held_gb = 0.0;
    return 1; /* host memory: plain */
}
int lbk_wait_stats(const lbk_ctx* c, double* s, unsigned long long* w, int* a) {
    (void)c;
    if (s) *s = 0.0;
    if (w) *w = 0;
    if (a) *a = 0;
    return 0;
}
int lbk_stream_probe(lbk_ctx* c, double* q, const double* const* ys, const double* const* ss, int npairs,
                     int launches, double* us, int variant, double* const* outs) {
    (void)c, (void)q, (void)ys, (void)ss, (void)npairs, (void)launches, (void)variant, (void)outs;
    *us = 0.0;  /* no device: nothing to time */
    return 0;
}

/* ---- memory: ghost cells at [-1] and [n] (zero), as lbk_vec_alloc's layout ---- */
double* lbk_vec_alloc(lbk_ctx* c) {
    double* p = (double*)calloc((size_t)c->geo.n_loc + DBL_FRONT + 8, sizeof(double));
    return p ? p + DBL_FRONT : NULL;
}
void lbk_vec_free(lbk_ctx* c, double* v) {
    (void)c;
    if (v) free(v - DBL_FRONT);
}
void* lbk_host_alloc(size_t bytes) { return malloc(bytes); }
void lbk_host_free(void* p) { free(p); }
int lbk_upload(lbk_ctx* c, double* dst, const double* h) {
    memcpy(dst, h, sizeof(double) * (size_t)c->geo.n_loc);
    return 0;
}
int lbk_download(lbk_ctx* c, double* h, const double* src) {
    memcpy(h, src, sizeof(double) * (size_t)c->geo.n_loc);
    return 0;
}
int lbk_copy(lbk_ctx* c, double* dst, const double* src) {
    memcpy(dst - 1, src - 1, sizeof(double) * (size_t)(c->geo.n_loc + 2));
    return 0;
}
int lbk_download_local(lbk_ctx* c, double* h, const double* src) { return lbk_download(c, h, src); }
int lbk_upload_local(lbk_ctx* c, double* dst, const double* h) { return lbk_upload(c, dst, h); }
int lbk_download_local_async(lbk_ctx* c, double* h, const double* src, int tag) {
    if (tag < 0 || tag >= 4) return -1;
    return lbk_download(c, h, src);
}
int lbk_upload_local_async(lbk_ctx* c, double* dst, const double* h, int tag) {
    if (tag < 0 || tag >= 4) return -1;
    return lbk_upload(c, dst, h);
}
int lbk_xfer_wait(lbk_ctx* c, int tag) {
    (void)c;
    return (tag < 0 || tag >= 4) ? -1 : 0;
}
int lbk_sync(lbk_ctx* c) {
    (void)c;
    return 0;
}

/* ---- slots ---- */
static int slot_ok(lbk_ctx* c, int slot) {
    if (slot < 0 || slot >= LBK_NSLOTS) {
        snprintf(c->err, sizeof c->err, "double: slot %d unsupported", slot);
        return 0;
    }
    return 1;
}
static double ref_total(lbk_ctx* c, int ref) {
    const int s = ref / LBK_KMAX, k = ref % LBK_KMAX;
    double t = c->slots[s][0][k];
    for (int g = 1; g < LBK_GROUPS; ++g) t = t + c->slots[s][g][k];
    return t;
}
/* component k of `slot` := canonical groups of a.b (kind 0) or of sum a[0..limit) (kind 1) */
static void put(lbk_ctx* c, int slot, int k, const double* a, const double* b, int64_t limit, int kind) {
    double q8[LBK_GROUPS];
    canon_groups(a, b, c->geo.n, limit, kind, q8);
    for (int g = 0; g < LBK_GROUPS; ++g) c->slots[slot][g][k] = q8[g];
}
int lbk_fetch_groups(lbk_ctx* c, int slot, double* g64) {
    if (!slot_ok(c, slot)) return -1;
    memcpy(g64, c->slots[slot], sizeof c->slots[slot]);
    return 0;
}
int lbk_fetch(lbk_ctx* c, int slot, int ncomp, double* totals) {
    if (!slot_ok(c, slot) || ncomp > LBK_KMAX) return -1;
    for (int k = 0; k < ncomp; ++k) totals[k] = ref_total(c, slot * LBK_KMAX + k);
    return 0;
}
double lbk_total(const double* g64, int comp) {
    double t = g64[comp];
    for (int g = 1; g < LBK_GROUPS; ++g) t = t + g64[g * LBK_KMAX + comp];
    return t;
}

/* f terms of z (per element, the canonical restatement of orc_f) into t; returns the sum limit */
static int64_t f_terms(int obj, const double* z, int64_t n, double* t) {
    if (obj == LBK_OBJ_ROSENBROCK) {
        for (int64_t i = 0; i + 1 < n; i++) {
            const double term1 = z[i + 1] - z[i] * z[i];
            const double term2 = 1 - z[i];
            t[i] = 100.0 * term1 * term1 + term2 * term2;
        }
        return n - 1;
    }
    if (obj == LBK_OBJ_QUAD_TRIDIAG) {
        for (int64_t i = 0; i < n; i++) {
            const double dterm = 1000.0 * z[i] * z[i];
            t[i] = (i + 1 < n) ? dterm + 100.0 * z[i] * z[i + 1] : dterm;
        }
        return n;
    }
    for (int64_t i = 0; i < n; i++) t[i] = (z[i] - 1) * (z[i] - 1);
    return n;
}

#define CHECK_SLOT(slot) \
    if (!slot_ok(c, slot)) return -1
#define ACCOUNT(vecs) c->bytes += (vecs) * 8.0 * (double)c->geo.n_loc

/* ---- the passes ---- */
int lbk_dot(lbk_ctx* c, const double* a, const double* b, int slot) {
    CHECK_SLOT(slot);
    put(c, slot, 0, a, b, c->geo.n, 0);
    ACCOUNT(2);
    return 0;
}
int lbk_axpy_dot(lbk_ctx* c, double* qout, const double* qin, const double* y, const double* s, double rho,
                 int ref_alpha, int slot) {
    CHECK_SLOT(slot);
    const double alpha = rho * ref_total(c, ref_alpha);
    for (int64_t i = 0; i < c->geo.n; ++i) qout[i] = qin[i] - alpha * y[i];
    put(c, slot, 0, s, qout, c->geo.n, 0);
    ACCOUNT(4);
    return 0;
}
int lbk_mid(lbk_ctx* c, double* rout, const double* qin, const double* y0, double rho0, double gamma,
            int ref_alpha, int slot) {
    CHECK_SLOT(slot);
    const double alpha = rho0 * ref_total(c, ref_alpha);
    for (int64_t i = 0; i < c->geo.n; ++i) rout[i] = (qin[i] - alpha * y0[i]) * gamma;
    put(c, slot, 0, y0, rout, c->geo.n, 0);
    ACCOUNT(3);
    return 0;
}
static double coef_ab(lbk_ctx* c, double rho, int ref_beta, int ref_alpha) {
    const double beta = rho * ref_total(c, ref_beta);
    const double alpha = rho * ref_total(c, ref_alpha);
    return alpha - beta;
}
int lbk_axpy2_dot(lbk_ctx* c, double* r, const double* rin, const double* s, const double* ynext, double rho,
                  int ref_beta, int ref_alpha, int slot) {
    CHECK_SLOT(slot);
    const double coef = coef_ab(c, rho, ref_beta, ref_alpha);
    for (int64_t i = 0; i < c->geo.n; ++i) r[i] = rin[i] + s[i] * coef;
    put(c, slot, 0, ynext, r, c->geo.n, 0);
    ACCOUNT(4);
    return 0;
}
int lbk_last(lbk_ctx* c, double* dout, const double* r, const double* s, const double* g, double rho, int ref_beta,
             int ref_alpha, int slot) {
    CHECK_SLOT(slot);
    const double coef = coef_ab(c, rho, ref_beta, ref_alpha);
    for (int64_t i = 0; i < c->geo.n; ++i) dout[i] = -(r[i] + s[i] * coef);
    put(c, slot, 0, g, dout, c->geo.n, 0);
    ACCOUNT(4);
    return 0;
}
int lbk_negdot(lbk_ctx* c, double* dout, const double* g, int slot) {
    CHECK_SLOT(slot);
    for (int64_t i = 0; i < c->geo.n; ++i) dout[i] = -g[i];
    put(c, slot, 0, g, dout, c->geo.n, 0);
    ACCOUNT(2);
    return 0;
}
int lbk_eval(lbk_ctx* c, int obj, const double* x, double* gout, int slot) {
    CHECK_SLOT(slot);
    if (obj < 0 || obj > LBK_OBJ_QUAD_SEPARABLE) return -1;
    const int64_t n = c->geo.n;
    double* t = c->scratch[0];
    double* g = gout ? gout : c->scratch[1];
    put(c, slot, 0, t, NULL, f_terms(obj, x, n, t), 1);
    orc_grad(obj, x, n, g);
    put(c, slot, 1, g, g, n, 0);
    ACCOUNT(gout ? 2 : 1);
    return 0;
}
/* d per dmode into dd */
static void form_dir(lbk_ctx* c, int dmode, const double* dsrc, const double* s_last, const double* g, double rho,
                     int ref_beta, int ref_alpha, double* dd) {
    const int64_t n = c->geo.n;
    if (dmode == LBK_D_BUF) {
        memcpy(dd, dsrc, sizeof(double) * (size_t)n);
    } else if (dmode == LBK_D_NEG_G) {
        for (int64_t i = 0; i < n; ++i) dd[i] = -g[i];
    } else {
        const double coef = coef_ab(c, rho, ref_beta, ref_alpha);
        for (int64_t i = 0; i < n; ++i) dd[i] = -(dsrc[i] + s_last[i] * coef);
    }
}
int lbk_trial(lbk_ctx* c, int obj, const double* x, const double* d, double alpha, double* gout, int slot) {
    CHECK_SLOT(slot);
    if (obj < 0 || obj > LBK_OBJ_QUAD_SEPARABLE) return -1;
    const int64_t n = c->geo.n;
    double *z = c->scratch[0], *t = c->scratch[1], *g = gout ? gout : c->scratch[2];
    for (int64_t i = 0; i < n; ++i) z[i] = x[i] + alpha * d[i];
    put(c, slot, 0, t, NULL, f_terms(obj, z, n, t), 1);
    orc_grad(obj, z, n, g);
    put(c, slot, 1, g, d, n, 0);
    ACCOUNT(gout ? 3 : 2);
    return 0;
}
int lbk_trials(lbk_ctx* c, int obj, int dmode, const double* x, const double* dsrc, const double* s_last,
               const double* gg, double rho, int ref_beta, int ref_alpha, const double* alphas, int nc, int dphi,
               int slot) {
    CHECK_SLOT(slot);
    if (obj < 0 || obj > LBK_OBJ_QUAD_SEPARABLE || nc < 1 || nc > LBK_TRIALS_NC || (dphi && nc != 1)) return -1;
    const int64_t n = c->geo.n;
    double *dd = c->scratch[3], *z = c->scratch[0], *t = c->scratch[1], *g = c->scratch[2];
    form_dir(c, dmode, dsrc, s_last, gg, rho, ref_beta, ref_alpha, dd);
    for (int j = 0; j < nc; ++j) {
        for (int64_t i = 0; i < n; ++i) z[i] = x[i] + alphas[j] * dd[i];
        put(c, slot, j, t, NULL, f_terms(obj, z, n, t), 1);
        if (dphi && j == 0) {
            orc_grad(obj, z, n, g);
            put(c, slot, nc, g, dd, n, 0);
        }
    }
    ACCOUNT(dmode == LBK_D_TWOLOOP ? 3 : 2);
    return 0;
}
int lbk_commit(lbk_ctx* c, int obj, int dmode, const double* x, const double* dsrc, const double* s_last,
               const double* g, double rho, int ref_beta, int ref_alpha, double alpha, double* xn, double* gn,
               double* s_out, double* y_out, int slot, double cand) {
    CHECK_SLOT(slot);
    const int64_t n = c->geo.n;
    double *dd = c->scratch[3], *t = c->scratch[1], *z = c->scratch[0];
    form_dir(c, dmode, dsrc, s_last, g, rho, ref_beta, ref_alpha, dd);
    for (int64_t i = 0; i < n; ++i) xn[i] = x[i] + alpha * dd[i];
    if (obj != LBK_OBJ_NONE) {
        put(c, slot, LBK_C_F, t, NULL, f_terms(obj, xn, n, t), 1);
        orc_grad(obj, xn, n, gn);
    }
    for (int64_t i = 0; i < n; ++i) {
        s_out[i] = xn[i] - x[i];
        y_out[i] = gn[i] - g[i];
    }
    put(c, slot, LBK_C_GD, g, dd, n, 0);
    put(c, slot, LBK_C_SY, s_out, y_out, n, 0);
    put(c, slot, LBK_C_YY, y_out, y_out, n, 0);
    put(c, slot, LBK_C_GG, gn, gn, n, 0);
    put(c, slot, LBK_C_SG, s_out, gn, n, 0);
    put(c, slot, LBK_C_DPHI, gn, dd, n, 0);
    if (cand > 0.0 && obj != LBK_OBJ_NONE && dmode != LBK_D_BUF) {
        for (int64_t i = 0; i < n; ++i) z[i] = x[i] + cand * dd[i];
        put(c, slot, LBK_C_FC, t, NULL, f_terms(obj, z, n, t), 1);
    }
    ACCOUNT(4.0 + (dmode == LBK_D_BUF ? 3.0 : dmode == LBK_D_NEG_G ? 2.0 : 4.0));
    return 0;
}
int lbk_point(lbk_ctx* c, double* z, const double* x, const double* d, double alpha) {
    for (int64_t i = -1; i <= c->geo.n; ++i) z[i] = x[i] + alpha * d[i];
    ACCOUNT(3);
    return 0;
}
int lbk_elementwise(lbk_ctx* c, int op, double* out, const double* a, const double* b, double alpha) {
    for (int64_t i = 0; i < c->geo.n; ++i) {
        switch (op) {
            case 0: out[i] = alpha * a[i]; break;
            case 1: out[i] = a[i] + b[i]; break;
            case 2: out[i] = -a[i]; break;
            default: out[i] = a[i] + alpha * b[i]; break;
        }
    }
    ACCOUNT(op == 1 || op == 3 ? 3 : 2);
    return 0;
}
int lbk_update(lbk_ctx* c, int op, double* out, const double* a, const double* b, double rho, int slot_a, int slot_b,
               double scal) {
    double coef = 0.0;
    if (op == LBK_U_AXPY_Q) coef = rho * ref_total(c, slot_a * LBK_KMAX);
    if (op == LBK_U_AXPY_R) coef = (rho * ref_total(c, slot_a * LBK_KMAX)) - (rho * ref_total(c, slot_b * LBK_KMAX));
    for (int64_t i = 0; i < c->geo.n; ++i) {
        switch (op) {
            case LBK_U_AXPY_Q: out[i] = a[i] - coef * b[i]; break;
            case LBK_U_AXPY_R: out[i] = a[i] + b[i] * coef; break;
            case LBK_U_SCALE: out[i] = a[i] * scal; break;
            case LBK_U_NEG: out[i] = -a[i]; break;
            case LBK_U_SUB: out[i] = a[i] - b[i]; break;
            default: out[i] = a[i] + scal * b[i]; break;
        }
    }
    ACCOUNT(3);
    return 0;
}
int lbk_checksum(lbk_ctx* c, const double* x, uint64_t* c1, uint64_t* c2) {
    orc_checksum(x, c->geo.n, c1, c2);
    return 0;
}

/* ---- dense quadratic objective (the oracle's dense_row order) ---- */
int lbk_dense_set(lbk_ctx* c, const double* A, const double* b) {
    const int64_t n = c->geo.n;
    free(c->dA);
    free(c->db);
    c->dA = (double*)malloc(sizeof(double) * (size_t)(n * n));
    c->db = (double*)malloc(sizeof(double) * (size_t)n);
    if (!c->dA || !c->db) return -4;
    memcpy(c->dA, A, sizeof(double) * (size_t)(n * n));
    memcpy(c->db, b, sizeof(double) * (size_t)n);
    return 0;
}
int lbk_dense_eval(lbk_ctx* c, const double* x, double* gout, int slot) {
    CHECK_SLOT(slot);
    if (!c->dA) return -1;
    const int64_t n = c->geo.n;
    double* t = c->scratch[4];
    for (int64_t i = 0; i < n; ++i) {
        const double r = dense_row(c->dA + i * n, x, n);
        t[i] = x[i] * r + c->db[i] * x[i];
        if (gout) gout[i] = 2.0 * r + c->db[i];
    }
    put(c, slot, 0, t, NULL, n, 1);
    if (gout) put(c, slot, 1, gout, gout, n, 0);
    ACCOUNT((double)n + 3.0);
    return 0;
}

/* ---- not modelled: vector-free mode, the small-n single-launch forms ---- */
int lbk_vf_commit(lbk_ctx* c, int obj, int h, const double* x, const double* g, const double* const* S,
                  const double* const* Y, const double* cs, const double* cy, double cg, double alpha,
                  const double* cand, double* xn, double* gn, double* so, double* yo, int wslot, int* hb_out) {
    (void)obj, (void)h, (void)x, (void)g, (void)S, (void)Y, (void)cs, (void)cy, (void)cg, (void)alpha, (void)cand;
    (void)xn, (void)gn, (void)so, (void)yo, (void)wslot, (void)hb_out;
    snprintf(c->err, sizeof c->err, "double: vector-free mode unsupported");
    return -1;
}
int lbk_vf_dir(lbk_ctx* c, int h, double* d, const double* g, const double* const* S, const double* const* Y,
               const double* cs, const double* cy, double cg) {
    (void)c, (void)h, (void)d, (void)g, (void)S, (void)Y, (void)cs, (void)cy, (void)cg;
    return -1;
}
int lbk_vf_bucket(int h) { return h <= LBK_VF_HMAX ? h : -1; }
int lbk_vf_ghost_init(lbk_ctx* c, double* x, double* g, int wslot) {
    (void)c, (void)x, (void)g, (void)wslot;
    return 0;
}
int lbk_small_ok(const lbk_ctx* c, int h) { return c->small_on && h >= 1 && h <= 16; }

/* k_coop_search's loops on this double's trial evaluation (lbk_trials, D_BUF: f at the halving
 * chain, or f and g.d) and its commit (lbk_commit, D_BUF) */
int lbk_search_dev_ok(const lbk_ctx* c, int obj) {
    return c->small_on && c->wolfe_on && obj >= 0 && obj <= LBK_OBJ_QUAD_SEPARABLE;
}
static double wolfe_cubic(double a0, double a1, double p0, double dp0, double p1, double dp1) {
    const double d1 = dp0 + dp1 - 3 * (p1 - p0) / (a1 - a0);
    const double d2 = copysign(sqrt(d1 * d1 - dp0 * dp1), a1 - a0);
    return a0 + (a1 - a0) * (dp0 + d2 - d1) / (dp0 - dp1 + 2 * d2);
}
/* 1: a value, 0: the pass budget is spent, -1: error */
static int dbl_trial(lbk_ctx* c, int obj, int ls, const double* x, const double* d, lbk_search* s, int* pass,
                     double alpha, int need_g, double* f, double* dphi) {
    const int slot = LBK_NSLOTS - 1; /* a slot the driver never names */
    if (s->have_spec && alpha == s->spec_a) {
        *f = s->spec_f;
        *dphi = s->spec_dphi;
        return 1;
    }
    if (!need_g && s->have_cand && alpha == s->cand_a) {
        *f = s->cand_f;
        return 1;
    }
    for (int j = 0; j < s->tc_n; ++j)
        if (alpha == s->tc_a[j] && (!need_g || (j == 0 && s->tc_dphi_ok))) {
            *f = s->tc_f[j];
            *dphi = s->tc_dphi;
            return 1;
        }
    if (*pass >= LBK_SEARCH_PASSES) return 0;
    (*pass)++;
    if (ls == 2 || ls == 3) {
        double t[2];
        if (lbk_trials(c, obj, LBK_D_BUF, x, d, NULL, NULL, 0.0, -1, -1, &alpha, 1, 1, slot) != 0) return -1;
        if (lbk_fetch(c, slot, 2, t) != 0) return -1;
        s->tc_n = 1;
        s->tc_a[0] = alpha;
        s->tc_f[0] = t[0];
        s->tc_dphi = t[1];
        s->tc_dphi_ok = 1;
        s->passes_fg++;
        *f = t[0];
        *dphi = t[1];
    } else {
        double a[LBK_TRIALS_NC], t[LBK_TRIALS_NC];
        a[0] = alpha;
        for (int j = 1; j < LBK_TRIALS_NC; ++j) a[j] = a[j - 1] * (ls == 0 ? s->beta : 0.5);
        if (lbk_trials(c, obj, LBK_D_BUF, x, d, NULL, NULL, 0.0, -1, -1, a, LBK_TRIALS_NC, 0, slot) != 0) return -1;
        if (lbk_fetch(c, slot, LBK_TRIALS_NC, t) != 0) return -1;
        s->tc_n = LBK_TRIALS_NC;
        for (int j = 0; j < LBK_TRIALS_NC; ++j) {
            s->tc_a[j] = a[j];
            s->tc_f[j] = t[j];
        }
        s->tc_dphi = 0.0;
        s->tc_dphi_ok = 0;
        s->passes_f++;
        *f = t[0];
    }
    return 1;
}
#define TRIAL(al, ng, f, dp)                                                          \
    do {                                                                              \
        const int r_ = dbl_trial(c, obj, ls, x, d, &s, &pass, (al), (ng), (f), (dp)); \
        if (r_ < 0) return -1;                                                        \
        if (r_ == 0) goto out;                                                        \
    } while (0)
int lbk_search_dev(lbk_ctx* c, int obj, int ls, const double* x, const double* d, lbk_search* st,
                   const lbk_search_commit* cm) {
    if (!lbk_search_dev_ok(c, obj)) return -1;
    lbk_search s = *st;
    s.done = s.committed = s.passes_f = s.passes_fg = 0;
    int pass = 0;
    double alpha = s.alpha, dd = 0.0;
    if (ls == 0) {
        for (;;) {
            double ft;
            TRIAL(alpha, 0, &ft, &dd);
            if (!(s.f_x - ft < s.c1 * alpha * s.gd)) break;
            alpha *= s.beta;
            if (alpha < s.tol) break;
        }
        s.done = 1;
        s.step = alpha;
    } else if (ls == 1) {
        for (;;) {
            if (!(s.iter++ < 20)) {
                s.done = 1;
                s.step = alpha;
                break;
            }
            double f_new;
            const int r = dbl_trial(c, obj, ls, x, d, &s, &pass, alpha, 0, &f_new, &dd);
            if (r < 0) return -1;
            if (r == 0) {
                s.iter--;
                break;
            }
            if (f_new <= s.f_x + s.c1 * alpha * s.gd) {
                s.done = 1;
                s.step = alpha;
                break;
            }
            if (alpha < s.amin) {
                s.done = 1;
                s.step = s.amin;
                break;
            }
            if (s.alpha_prev > 0) {
                if (fabs(alpha - s.alpha_prev) < 1e-10) {
                    alpha *= 0.5;
                } else {
                    const double ga = (f_new - s.f_x - s.gd * alpha) / (alpha * alpha);
                    alpha = wolfe_cubic(s.alpha_prev, alpha, s.f_prev, s.gd, f_new, ga);
                    if (alpha < 0.1 * s.alpha_prev || alpha > 0.9 * s.alpha_prev) alpha = s.alpha_prev * 0.5;
                }
            } else {
                alpha = alpha - 0.5 * s.gd * alpha * alpha / (s.f_x - f_new - s.gd * alpha);
                if (alpha < 0.1 * s.init || alpha > 0.9 * s.init) alpha = s.init * 0.5;
            }
            s.alpha_prev = alpha;
            s.f_prev = f_new;
        }
    } else if (ls == 2) {
        for (;;) {
            if (s.iter >= 20) {
                s.done = 1;
                s.step = alpha;
                break;
            }
            double f_new, dphi_new;
            TRIAL(alpha, 0, &f_new, &dphi_new);
            if (f_new > s.f_x + s.c1 * alpha * s.gd || (f_new >= s.f_lo && s.iter > 0)) {
                s.alpha_hi = alpha;
                alpha = wolfe_cubic(s.alpha_lo, s.alpha_hi, s.f_lo, s.dphi_lo, f_new,
                                    (f_new - s.f_x - s.gd * alpha) / (alpha * alpha));
                ++s.iter;
                continue;
            }
            TRIAL(alpha, 1, &f_new, &dphi_new);
            if (fabs(dphi_new) <= -s.c2 * s.gd) {
                s.done = 1;
                s.step = alpha;
                break;
            }
            if (dphi_new >= 0) {
                s.alpha_hi = alpha;
                alpha = wolfe_cubic(s.alpha_lo, s.alpha_hi, s.f_lo, s.dphi_lo, f_new, dphi_new);
            } else {
                s.alpha_lo = alpha;
                s.f_lo = f_new;
                s.dphi_lo = dphi_new;
                alpha = s.alpha_hi == INFINITY ? alpha * 2
                                               : wolfe_cubic(s.alpha_lo, s.alpha_hi, s.f_lo, s.dphi_lo, f_new, dphi_new);
            }
            if (alpha < s.amin) {
                s.done = 1;
                s.step = s.amin;
                break;
            }
            ++s.iter;
        }
    } else {
        for (;;) {
            double fn, dphi;
            TRIAL(alpha, 1, &fn, &dphi);
            if (fn > s.f_x + s.c1 * alpha * s.gd) {
                alpha *= s.beta;
            } else if (dphi < s.c2 * s.gd) {
                alpha *= 1.1;
            } else {
                break;
            }
            if (alpha < s.tol) break;
        }
        s.done = 1;
        s.step = alpha;
    }
out:
    s.alpha = alpha;
    if (s.done && cm && cm->slot >= 0 && !(s.have_spec && s.step == s.spec_a)) {
        if (lbk_commit(c, obj, LBK_D_BUF, x, d, NULL, cm->g, 0.0, -1, -1, s.step, cm->xn, cm->gn, cm->so, cm->yo,
                       cm->slot, 0.0) != 0)
            return -1;
        s.committed = 1;
    }
    *st = s;
    return 0;
}
#undef TRIAL
int lbk_small_spec_ok(const lbk_ctx* c, int h) { return lbk_small_ok(c, h); }

/* the prologue of a speculative launch (k_coop_iter's spec_ok), on this double's slots */
static int spec_tests(lbk_ctx* c, const lbk_spec* sp, double a0, double* rg) {
    if (sp->chain_epoch && c->vd[sp->chain_epoch & 3] != ((sp->chain_epoch << 1) | 1ull)) return 0;
    const int p = sp->prev_slot * LBK_KMAX;
    const double gd = ref_total(c, p + LBK_C_GD), ft = ref_total(c, p + LBK_C_F), dphi = ref_total(c, p + LBK_C_DPHI);
    const double sy = ref_total(c, p + LBK_C_SY), yy = ref_total(c, p + LBK_C_YY), gg = ref_total(c, p + LBK_C_GG);
    const double fx = sp->fx, al = a0, c1 = sp->c1, c2 = sp->c2;
    rg[0] = 1.0 / sy;
    rg[1] = sy / yy;
    int take = 1;
    if (sp->ls < 0) {
    } else if (gd >= 0) {
        return 0;
    } else switch (sp->ls) {
        case 0: take = !(fx - ft < c1 * al * gd); break;
        case 1: take = ft <= fx + c1 * al * gd; break;
        case 2: take = !(ft > fx + c1 * al * gd) && fabs(dphi) <= -c2 * gd; break;
        default: take = !(ft > fx + c1 * al * gd) && !(dphi < c2 * gd); break;
    }
    if (!take || (sp->ls >= 0 && al < 1e-10) || !(sy > 0)) return 0;
    if (sqrt(gg) < sp->tol) return 0;
    if (!isfinite(rg[0]) || rg[1] <= 0 || !isfinite(rg[1])) return 0;
    return 1;
}

/* the launch sequence the cooperative kernel fuses: P0 dot unless p0_ref >= 0, the first loop,
 * mid, the second loop, the TWOLOOP commit at a0 */
int lbk_small_iter(lbk_ctx* c, int obj, int h, const double* g, double* q, double* r, const double* const* S,
                   const double* const* Y, const double* rho, double gamma, int p0_ref, double a0, const double* x,
                   double* xn, double* gn, double* so, double* yo, int slot_p0, int slot_a0, int slot_b0, int slot_c,
                   double cand, const lbk_spec* spec, unsigned long long* epoch) {
    if (epoch) *epoch = 0;
    if (!lbk_small_ok(c, h) || h > 16) return -1;
    const unsigned long long e = ++c->epoch;
    const int i4 = (int)(e & 3);
    if (epoch) *epoch = e;
    double rho_top = rho[h - 1];
    if (spec) {
        double rg[2];
        const int went = spec_tests(c, spec, a0, rg);
        c->vd[i4] = (e << 1) | (unsigned long long)went;
        c->rec_went[i4] = went;
        c->rec_rho[i4] = rg[0];
        c->rec_gamma[i4] = rg[1];
        if (!went) return 0;
        rho_top = rg[0];
        gamma = rg[1];
    } else {
        c->rec_went[i4] = 1;
        c->rec_rho[i4] = rho_top;
        c->rec_gamma[i4] = gamma;
    }
    int refA[16], refB[16];
    if (p0_ref >= 0) {
        refA[h - 1] = p0_ref;
    } else {
        if (lbk_dot(c, S[h - 1], g, slot_p0)) return -1;
        refA[h - 1] = slot_p0 * LBK_KMAX;
    }
    const double* qsrc = g;
    for (int i = h - 2; i >= 0; --i) {
        if (lbk_axpy_dot(c, q, qsrc, Y[i + 1], S[i], i + 1 == h - 1 ? rho_top : rho[i + 1], refA[i + 1], slot_a0 + i))
            return -1;
        refA[i] = (slot_a0 + i) * LBK_KMAX;
        qsrc = q;
    }
    if (lbk_mid(c, r, qsrc, Y[0], h == 1 ? rho_top : rho[0], gamma, refA[0], slot_b0)) return -1;
    refB[0] = slot_b0 * LBK_KMAX;
    for (int i = 0; i + 1 < h; ++i) {
        if (lbk_axpy2_dot(c, r, r, S[i], Y[i + 1], rho[i], refB[i], refA[i], slot_b0 + i + 1)) return -1;
        refB[i + 1] = (slot_b0 + i + 1) * LBK_KMAX;
    }
    return lbk_commit(c, obj, LBK_D_TWOLOOP, x, r, S[h - 1], g, rho_top, refB[h - 1], refA[h - 1], a0, xn, gn, so, yo,
                      slot_c, cand);
}
/* the persistent two-loop: the same passes into the same slots, no commit */
int lbk_twoloop_ok(const lbk_ctx* c, int h) { return c->twoloop_on && h >= 1 && h <= 16; }
int lbk_twoloop_persist(lbk_ctx* c, int h, const double* g, double* q, double* r, const double* const* S,
                        const double* const* Y, const double* rho, double gamma, int p0_ref, int slot_p0,
                        int slot_a0, int slot_b0) {
    if (!lbk_twoloop_ok(c, h)) return -1;
    int refA[16], refB[16];
    if (p0_ref >= 0) {
        refA[h - 1] = p0_ref;
    } else {
        if (lbk_dot(c, S[h - 1], g, slot_p0)) return -1;
        refA[h - 1] = slot_p0 * LBK_KMAX;
    }
    const double* qsrc = g;
    for (int i = h - 2; i >= 0; --i) {
        if (lbk_axpy_dot(c, q, qsrc, Y[i + 1], S[i], rho[i + 1], refA[i + 1], slot_a0 + i)) return -1;
        refA[i] = (slot_a0 + i) * LBK_KMAX;
        qsrc = q;
    }
    if (lbk_mid(c, r, qsrc, Y[0], rho[0], gamma, refA[0], slot_b0)) return -1;
    refB[0] = slot_b0 * LBK_KMAX;
    for (int i = 0; i + 1 < h; ++i) {
        if (lbk_axpy2_dot(c, r, r, S[i], Y[i + 1], rho[i], refB[i], refA[i], slot_b0 + i + 1)) return -1;
        refB[i + 1] = (slot_b0 + i + 1) * LBK_KMAX;
    }
    return 0;
}

int lbk_mark(lbk_ctx* c) {
    (void)c;
    return 0;
}
int lbk_fetch_marked(lbk_ctx* c, int slot, int ncomp, double* totals) { return lbk_fetch(c, slot, ncomp, totals); }

int lbk_small_fetch(lbk_ctx* c, unsigned long long epoch, int slot, int ncomp, double* totals, int* went,
                    double* rho, double* gamma) {
    if (went) *went = 1;
    if (epoch == 0) return lbk_fetch(c, slot, ncomp, totals);
    if (epoch > c->epoch || epoch + 4 <= c->epoch) return -1;
    const int i4 = (int)(epoch & 3);
    if (rho) *rho = c->rec_rho[i4];
    if (gamma) *gamma = c->rec_gamma[i4];
    if (!c->rec_went[i4]) {
        if (went) *went = 0;
        return 0;
    }
    return lbk_fetch(c, slot, ncomp, totals);
}

/* ---- profiling ---- */
void lbk_prof_enable(lbk_ctx* c, int on) {
    (void)c;
    (void)on;
}
int lbk_prof_get(lbk_ctx* c, int kind, double* ms, int64_t* launches, double* bytes) {
    (void)c;
    if (kind < 0 || kind >= LBK_K_COUNT) return -1;
    *ms = 0.0;
    *launches = 0;
    *bytes = 0.0;
    return 0;
}
void lbk_prof_reset(lbk_ctx* c) { (void)c; }
double lbk_bytes_moved(const lbk_ctx* c) { return c->bytes; }
