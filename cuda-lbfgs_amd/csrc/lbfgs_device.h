/* lbfgs_device.h — internal C interface between the C host driver (lbfgs_driver.c) and the
 * HIP device layer (lbfgs_kernels.hip). Not installed; the public ABI is include/lbfgs_hip.h.
 *
 * Every vector is an fp64 array of the rank's n_loc elements, addressed from its element 0,
 * with ghost cells at [-1] and [n_loc] and zeroed padding behind it (see lbk_vec_alloc).
 * Every reduction is written as 8 group partials into a result slot:
 *   slot s, component k  ->  slots[s*LBK_SLOT + g*LBK_KMAX + k], g = 0..7
 * and its value is the fixed-order sum Q0+Q1+...+Q7 (lbk_total).
 */
#ifndef LBFGS_DEVICE_H
#define LBFGS_DEVICE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LBK_KMAX 8
#define LBK_GROUPS 8
#define LBK_SLOT (LBK_GROUPS * LBK_KMAX) /* doubles per slot */
#define LBK_NSLOTS 256
#define LBK_SEGS 8192
#define LBK_SEG_PER_GROUP 1024
/* canonical minimum segment length LBK_MIDL for LBK_MIDL_LO <= n <= LBK_MIDL_HI, else 512; the
 * vector-free commit's base length is LBK_MIDL only from LBK_VFL_LO (shorter segments below) */
#define LBK_MIDL 2048
#define LBK_MIDL_LO 65536
#define LBK_VFL_LO 262144
#define LBK_MIDL_HI 2097152 /* 4 * 1024 * 512: sharding needs more elements at L = 512 */

/* wide result slots (vector-free mode: 4h + 6 components): ids LBK_WSLOT0 + w */
#define LBK_VF_HMAX 20
#define LBK_KW (4 * LBK_VF_HMAX + 16)
/* sharded vector-free: the rank's first / last element of x, g, s, y ride the wide slot's
 * spare components (group g_lo / g_hi - 1) into the neighbours' ghost cells */
#define LBK_VF_EDGE0 (LBK_KW - 8)
#define LBK_VF_EDGE1 (LBK_KW - 4)
#define LBK_WSLOT (LBK_GROUPS * LBK_KW)
#define LBK_NWSLOTS 4
#define LBK_WSLOT0 LBK_NSLOTS

/* vector-free commit components (basis b_l = s_0..s_{h-1}, y_0..y_{h-1}; HB = bucket of h) */
#define LBK_VF_F 0   /* f(x_new)             */
#define LBK_VF_SY 1  /* s_new . y_new        */
#define LBK_VF_YY 2  /* y_new . y_new        */
#define LBK_VF_GG 3  /* g_new . g_new        */
#define LBK_VF_YG 4  /* y_new . g_new        */
#define LBK_VF_GGO 5 /* g_new . g_old        */
#define LBK_VF_YB 6  /* + l: y_new . b_l (l < 2h); g_new . b_l at LBK_VF_YB + 2 HB + l */
/* + j at LBK_VF_YB + 4 HB: f(x + cand_j d) at the line search's next candidate steps */
#define LBK_VF_NA 1

/* objective ids (match include/lbfgs_hip.h) */
#define LBK_OBJ_ROSENBROCK 0
#define LBK_OBJ_QUAD_TRIDIAG 1
#define LBK_OBJ_QUAD_SEPARABLE 2
#define LBK_OBJ_NONE 3 /* gradient supplied in a buffer, f computed elsewhere (host callback) */
#define LBK_OBJ_DENSE 4 /* f = x'Ax + b'x (lbk_dense_set / lbk_dense_eval; not a stencil pass) */
#define LBK_DENSE_NMAX 65536

/* direction modes of the commit kernel */
#define LBK_D_BUF 0     /* d read from a buffer */
#define LBK_D_NEG_G 1   /* d = -g                           (lbfgs.cpp:90, :151) */
#define LBK_D_TWOLOOP 2 /* d = -(r + s (alpha_i - beta_i)) (last second-loop pass, :137-143) */

/* commit reduction components */
#define LBK_C_GD 0   /* g . d            */
#define LBK_C_F 1    /* f(x + a d)       */
#define LBK_C_SY 2   /* s . y            */
#define LBK_C_YY 3   /* y . y            */
#define LBK_C_GG 4   /* g_new . g_new    */
#define LBK_C_SG 5   /* s . g_new  (alpha of the next first pass) */
#define LBK_C_DPHI 6 /* g_new . d        */
#define LBK_C_FC 7   /* f(x + cand d): the line search's next step, computed alongside */

/* batched trials: steps per f-only pass (backtracking / interpolation halving chains) */
#define LBK_TRIALS_NC 4

/* kernel kinds, for profiling / byte accounting */
enum {
    LBK_K_DOT = 0, LBK_K_AXPY_DOT, LBK_K_MID, LBK_K_AXPY2_DOT, LBK_K_LAST, LBK_K_NEGDOT,
    LBK_K_EVAL, LBK_K_TRIAL_F, LBK_K_TRIAL_FG, LBK_K_COMMIT, LBK_K_POINT, LBK_K_CHECKSUM,
    LBK_K_UPDATE, LBK_K_VF_COMMIT, LBK_K_VF_DIR, LBK_K_SMALL_ITER, LBK_K_GROUP_REDUCE,
    LBK_K_EXCHANGE /* sharded: a reduction exchange (mailbox kernel or RCCL all-gather) */, LBK_K_COUNT
};

typedef struct {
    int64_t n;       /* global length */
    int64_t L;       /* canonical segment length */
    int64_t nseg;    /* global number of non-empty segments */
    int64_t seg_lo;  /* first global segment of this rank */
    int64_t seg_hi;  /* one past the last */
    int64_t elem_lo; /* global index of local element 0 */
    int64_t n_loc;   /* local elements */
    int g_lo, g_hi;  /* groups owned by this rank */
    int rank, world;
    int vf_f;        /* vector-free commit segment = vf_f canonical segments (lbk_vf_factor) */
} lbk_geo;

typedef struct lbk_ctx lbk_ctx;
typedef struct lbk_group lbk_group; /* host exchange group for emulated ranks (tests) */

/* lifecycle. world > 1: RCCL communicator from nccl_id (may be NULL: peer exchange only), or
 * the host group grp */
int lbk_create(lbk_ctx** out, int device, int64_t n, int rank, int world, const void* nccl_id,
               lbk_group* grp);
/* canonical geometry and this rank's shard, no device needed (0, or < 0 if not shardable) */
int lbk_geometry_plan(int64_t n, int rank, int world, lbk_geo* out);
/* segments of the vector-free commit, in canonical segments: the largest F in {1, 2, 4, 8}
 * with F L <= 8192 and ceil(n / (F L)) >= 1024 (restated as orc_vf_factor) */
int lbk_vf_factor(int64_t n);
lbk_group* lbk_group_create(int world);
void lbk_group_destroy(lbk_group* g);
/* sharded: the slot whose all-gather carries the neighbours' edge d (after lbk_last/negdot) */
void lbk_set_ghost_slot(lbk_ctx* c, int slot);
void lbk_destroy(lbk_ctx* c);
const lbk_geo* lbk_geometry(const lbk_ctx* c);
const char* lbk_last_error(const lbk_ctx* c);
int lbk_unique_id(void* out128);
int lbk_device_count(void);
/* sharded contexts (world > 1, one process per GPU): peer mailboxes over xGMI (lbfgs_xgmi.h).
 * handle: LBK_PEER_HANDLE_BYTES = 64; connect maps all peers' mailboxes (world handles in rank
 * order) and self-tests the exchange; enable switches every later exchange to it. */
int lbk_peer_handle(lbk_ctx* c, void* out);
int lbk_peer_connect(lbk_ctx* c, const void* handles);
int lbk_peer_enable(lbk_ctx* c, int on);
/* a sharded context created without an RCCL id takes a communicator (bounded init + self-test) */
int lbk_rccl_attach(lbk_ctx* c, const void* nccl_id);
/* 0 none (one rank), 1 RCCL, 2 xGMI peer mailboxes, 3 host group (emulated ranks) */
int lbk_exchange_backend(const lbk_ctx* c);
int lbk_exchange_fold(const lbk_ctx* c);
/* collective: iters back-to-back exchanges of a ks-component slot through backend 1 or 2;
 * host wall time per exchange in microseconds */
int lbk_exchange_bench(lbk_ctx* c, int backend, int ks, int iters, double* us);
/* LBFGS_CU_PARTITION: CUs of this rank's solver stream (0: not partitioned) */
int lbk_cu_partition(const lbk_ctx* c);
/* the cooperative forms' grid caps (segments) and the device searches redone on the host loop */
int lbk_coop_info(const lbk_ctx* c, int* coop_max, int* search_max, int* fallbacks);
/* host waits on completion words: seconds slept in the spin-then-sleep phase, waits completed,
 * whether the wait is adaptive (LBFGS_WAIT) */
int lbk_wait_stats(const lbk_ctx* c, double* slept_s, unsigned long long* waits, int* adaptive);
/* vectors allocated with a plain hipMalloc because a physically contiguous one was refused */
int lbk_vec_fallbacks(const lbk_ctx* c);
/* the context's allocation mode (0 pool, 1 plain, 2 contiguous), its vectors taken from or added
 * to the process-wide contiguous pool, and the GiB the pool owns */
int lbk_vec_pool_stats(const lbk_ctx* c, int* pooled, double* held_gb);
/* box probe: `launches` back-to-back 3 R + 1 W streams over (q, y, s) in the two-loop passes'
 * geometry and cache policy, q written back unchanged; launch i reads the pair pool's
 * y[(i + 1) % npairs] and s[i % npairs] (another pair every launch, as the passes: only q's tail
 * is left in the Infinity Cache by the launch before); mean microseconds per launch */
int lbk_stream_probe(lbk_ctx* c, double* q, const double* const* ys, const double* const* ss, int npairs,
                     int launches, double* us, int variant, double* const* outs);

/* memory */
double* lbk_vec_alloc(lbk_ctx* c);
void lbk_vec_free(lbk_ctx* c, double* v);
void* lbk_host_alloc(size_t bytes); /* pinned host memory (NULL on failure) */
void lbk_host_free(void* p);
int lbk_upload(lbk_ctx* c, double* dst, const double* host_global);     /* incl. ghosts */
int lbk_download(lbk_ctx* c, double* host_global, const double* src);   /* local part */
int lbk_copy(lbk_ctx* c, double* dst, const double* src);               /* incl. ghosts */
int lbk_download_local(lbk_ctx* c, double* host_local, const double* src);
int lbk_upload_local(lbk_ctx* c, double* dst, const double* host_local);
/* asynchronous local-range transfers on the solver stream; lbk_xfer_wait(tag) blocks until the
 * last transfer issued with that tag (0..3) has completed (host buffers must be pinned) */
int lbk_download_local_async(lbk_ctx* c, double* host_local, const double* src, int tag);
int lbk_upload_local_async(lbk_ctx* c, double* dst, const double* host_local, int tag);
int lbk_xfer_wait(lbk_ctx* c, int tag);

/* kernels (async on the context stream). 'slot' = result slot index; slot references
 * (prev, beta, alpha) are (slot index, component) pairs packed as slot*LBK_KMAX + comp. */
int lbk_dot(lbk_ctx* c, const double* a, const double* b, int slot);
int lbk_axpy_dot(lbk_ctx* c, double* qout, const double* qin, const double* y, const double* s,
                 double rho, int ref_alpha, int slot);
int lbk_mid(lbk_ctx* c, double* rout, const double* qin, const double* y0, double rho0,
            double gamma, int ref_alpha, int slot);
int lbk_axpy2_dot(lbk_ctx* c, double* r, const double* rin, const double* s, const double* ynext, double rho,
                  int ref_beta, int ref_alpha, int slot);
int lbk_last(lbk_ctx* c, double* dout, const double* r, const double* s, const double* g,
             double rho, int ref_beta, int ref_alpha, int slot);
int lbk_negdot(lbk_ctx* c, double* dout, const double* g, int slot);
int lbk_eval(lbk_ctx* c, int obj, const double* x, double* gout, int slot);  /* f, g.g */
int lbk_trial(lbk_ctx* c, int obj, const double* x, const double* d, double alpha,
              double* gout, int slot);                                           /* f, gt.d */
/* commit at x + alpha*d (d per dmode); writes xn, s_out, y_out and (obj != NONE) gn.
 * For obj == NONE the new gradient is read from gn (host-supplied). */
int lbk_commit(lbk_ctx* c, int obj, int dmode, const double* x, const double* dsrc,
               const double* s_last, const double* g, double rho, int ref_beta, int ref_alpha,
               double alpha, double* xn, double* gn, double* s_out, double* y_out, int slot, double cand);
/* batched line-search trials along d (dmode as the commit's: a buffer, -g, or the last two-loop
 * update formed on the fly): f at alphas[0..nc-1] (components 0..nc-1) and, with dphi,
 * g(x + alphas[0] d) . d (component nc; nc = 1 only). nc is 1 or LBK_TRIALS_NC. Device
 * objectives only. */
int lbk_trials(lbk_ctx* c, int obj, int dmode, const double* x, const double* dsrc, const double* s_last,
               const double* g, double rho, int ref_beta, int ref_alpha, const double* alphas, int nc, int dphi,
               int slot);
/* dense quadratic objective: A (n x n, row-major, symmetric) and b uploaded once; eval at x writes
 * slot components f and (with gout) gout . gout, and grad = 2 A x + b into gout */
int lbk_dense_set(lbk_ctx* c, const double* A, const double* b);
int lbk_dense_eval(lbk_ctx* c, const double* x, double* gout, int slot);
/* z = x + alpha * d (host-callback objectives) */
int lbk_point(lbk_ctx* c, double* z, const double* x, const double* d, double alpha);
/* elementwise primitives (op: 0 alpha*a, 1 a+b, 2 -a, 3 a+alpha*b) over the local range */
/* vector-free mode: d = sum_l c_l b_l + cg g (l ascending, then g) formed on the fly; commit at
 * x + alpha d with the wide reductions above into wide slot `wslot`. *hb_out = the bucket HB
 * that fixes the component layout. lbk_vf_dir materialises d. */
int lbk_vf_commit(lbk_ctx* c, int obj, int h, const double* x, const double* g, const double* const* S,
                  const double* const* Y, const double* cs, const double* cy, double cg, double alpha,
                  const double* cand /* LBK_VF_NA */, double* xn, double* gn, double* so, double* yo, int wslot,
                  int* hb_out);
int lbk_vf_dir(lbk_ctx* c, int h, double* d, const double* g, const double* const* S, const double* const* Y,
               const double* cs, const double* cy, double cg);
int lbk_vf_bucket(int h);
/* sharded vector-free: fill the ghost cells of x and g from the neighbours (solver start) */
int lbk_vf_ghost_init(lbk_ctx* c, double* x, double* g, int wslot);

/* small n (nseg within the context's limit, one rank, 1 <= h <= 16): the two-loop passes
 * (P0 dot unless p0_ref >= 0, axpy_dot, mid, axpy2_dot into the given slots) and the TWOLOOP
 * commit at a0 into slot_c, in one single-workgroup launch; the same slot contents and vectors as
 * the multi-launch sequence. S/Y in ring order (oldest first). */
int lbk_small_ok(const lbk_ctx* c, int h);
/* Speculative launch of the NEXT iteration (cooperative form, one rank, host-mirrored slots):
 * enqueued behind the current iteration's launch before the host has read its results. The
 * kernel's prologue restates, from the current iteration's commit slot `prev_slot`, every host
 * decision between the two iterations - the line search `ls` (LBFGS_LS_* numbering) takes the
 * first trial a0 (f at x is `fx`), the pair is stored (s.y > 0), the next iteration has not
 * converged (|g| >= tol), its rho and gamma are valid - and computes the newest pair's rho and
 * gamma itself (rho[h-1] and gamma are ignored). If any test fails no workgroup writes anything.
 * ls = -1: the current iteration's step is already decided (a recommit at the line search's
 * step): no line-search test. cand > 0: the commit also reduces f at x + cand d (LBK_C_FC).
 * `chain_epoch` (0: none) is the launch this one follows when that was speculative as well: its
 * device verdict must be "went". */
typedef struct {
    int prev_slot, ls;
    double fx, c1, c2, tol;
    unsigned long long chain_epoch;
} lbk_spec;
int lbk_small_spec_ok(const lbk_ctx* c, int h);
/* small n, single rank: a line search (lbfgs_driver.c ls_*, LBFGS_LS_* numbering) continued on
 * the device from the top of one of its iterations, in one cooperative launch (k_coop_search),
 * d materialised. The state is the host loop's: its constants, the values the host already holds
 * (the commit's first trial, the backtracking commit's f at its next step, the last trial pass),
 * and the loop variables; the launch evaluates at most LBK_SEARCH_PASSES trial passes and returns
 * the state as the host loop would have left it - done with the step, or (pass budget spent) at
 * the top of an iteration, for the host to continue. With a commit request and the search done at
 * another step than the commit's first trial, the launch also commits at that step (the D_BUF
 * commit of lbk_commit, cand 0, into cm->slot) and sets `committed`. */
#define LBK_SEARCH_PASSES 20
typedef struct {
    double f_x, gd, c1, c2, amin, init, beta, tol; /* constants */
    double spec_a, spec_f, spec_dphi;               /* the commit's first trial (have_spec) */
    double cand_a, cand_f;                          /* backtracking: f at the next step (have_cand) */
    double tc_a[LBK_TRIALS_NC], tc_f[LBK_TRIALS_NC], tc_dphi; /* the last trial pass: tc_n steps */
    int have_spec, have_cand, tc_n, tc_dphi_ok;
    double alpha, alpha_lo, alpha_hi, f_lo, dphi_lo, alpha_prev, f_prev; /* loop variables */
    int iter;
    int done, committed, passes_f, passes_fg; /* results */
    double step;
} lbk_search;
typedef struct {
    const double* g;
    double *xn, *gn, *so, *yo;
    int slot; /* < 0: no commit */
} lbk_search_commit;
int lbk_search_dev_ok(const lbk_ctx* c, int obj);
/* -6: the launch's grid barrier timed out (nothing stored, st unchanged); the device search is then
 * off for the context and the caller goes on with the host loop */
int lbk_search_dev(lbk_ctx* c, int obj, int ls, const double* x, const double* d, lbk_search* st,
                   const lbk_search_commit* cm);
/* *epoch: the launch's id for lbk_small_fetch (0: not a cooperative host-mirrored launch) */
int lbk_small_iter(lbk_ctx* c, int obj, int h, const double* g, double* q, double* r, const double* const* S,
                   const double* const* Y, const double* rho, double gamma, int p0_ref, double a0, const double* x,
                   double* xn, double* gn, double* so, double* yo, int slot_p0, int slot_a0, int slot_b0,
                   int slot_c, double cand, const lbk_spec* spec, unsigned long long* epoch);
/* Persistent two-loop (LBFGS_PERSIST=2, large n, one rank): the two-loop passes of
 * lbk_small_iter (P0 dot unless p0_ref >= 0, axpy_dot into slot_a0 + i, mid into slot_b0,
 * axpy2_dot into slot_b0 + i) in one launch of resident workgroups, the same slot contents and
 * vectors as the launch sequence; the commit is the caller's next launch. lbk_twoloop_ok: the
 * mode is on and its grid fits this n. */
int lbk_twoloop_ok(const lbk_ctx* c, int h);
int lbk_twoloop_persist(lbk_ctx* c, int h, const double* g, double* q, double* r, const double* const* S,
                        const double* const* Y, const double* rho, double gamma, int p0_ref, int slot_p0,
                        int slot_a0, int slot_b0);
/* waits for launch `epoch` to finish its commit (spinning on a pinned word, no stream
 * synchronisation: a speculative launch queued behind it keeps running), then the fixed-order
 * totals of slot_c. *went (may be NULL): 0 if a speculative launch found a test failing (it wrote
 * nothing and its reservations are released; the slot is stale); *rho / *gamma: the values a
 * speculative launch computed. epoch 0: lbk_fetch. */
int lbk_small_fetch(lbk_ctx* c, unsigned long long epoch, int slot, int ncomp, double* totals, int* went,
                    double* rho, double* gamma);
/* a mark in the stream after the launches so far, and the fixed-order totals of a host-mirrored
 * slot once the stream has passed the mark (work queued after the mark keeps running) */
int lbk_mark(lbk_ctx* c);
int lbk_fetch_marked(lbk_ctx* c, int slot, int ncomp, double* totals);

/* unfused mode: out = op(a, b) with device-side coefficients (see k_update) */
enum { LBK_U_AXPY_Q = 0, LBK_U_AXPY_R, LBK_U_SCALE, LBK_U_NEG, LBK_U_SUB, LBK_U_POINT };
int lbk_update(lbk_ctx* c, int op, double* out, const double* a, const double* b, double rho, int slot_a,
               int slot_b, double scal);
int lbk_elementwise(lbk_ctx* c, int op, double* out, const double* a, const double* b, double alpha);
int lbk_checksum(lbk_ctx* c, const double* x, uint64_t* c1, uint64_t* c2); /* sync */

/* results */
int lbk_fetch(lbk_ctx* c, int slot, int ncomp, double* totals);   /* sync, fixed-order totals */
int lbk_fetch_groups(lbk_ctx* c, int slot, double* groups64);     /* sync, raw 8 x KMAX */
double lbk_total(const double* groups64, int comp);
int lbk_sync(lbk_ctx* c);

/* profiling: per-kind event timing (enable before the timed region) */
void lbk_prof_enable(lbk_ctx* c, int on);
int lbk_prof_get(lbk_ctx* c, int kind, double* ms, int64_t* launches, double* bytes);
void lbk_prof_reset(lbk_ctx* c);
double lbk_bytes_moved(const lbk_ctx* c); /* algorithmic bytes of all launches so far */

#ifdef __cplusplus
}
#endif
#endif
