/* lbfgs_hip.h — public C ABI of the MI355X-native L-BFGS solver (liblbfgs_hip.so).
 *
 * Drop-in boundary for the reference's L-BFGS path (ndzajic1/cuda-lbfgs @ 2025-03-02):
 *   - lbfgs_minimize()          replaces LBFGS(f, grad, x0, method, max_iterations, m, tol,
 *                               verbose)  sequential-implementation/lbfgs.h:17-25 (def.
 *                               lbfgs.cpp:17-203), and LBFGS_CUDA(...)
 *                               parallel-implementation/L-BFGS.cu:105-112 (and the 4 variants'
 *                               string-less form, e.g. L-BFGS-Backtracking.cu:139-145).
 *   - LBFGS_LS_*                the line-search names accepted at lbfgs.cpp:40-70 /
 *                               L-BFGS.cu:120-153 ("backtracking", "interpolation", "wolfe",
 *                               "backtracking_wolfe"); line_search.h:10-26.
 *   - lbfgs_constants           config.h:5-17 (lbfgs_constants_default) and the CUDA path's
 *                               constants.h:5-21 (lbfgs_constants_cuda, C2 = 0.7).
 *   - LBFGS_OBJ_*               the benchmark objectives rosenbrock/rosenbrock_grad
 *                               (benchmark.cpp:58-81 = functions.cpp:26-49),
 *                               generate_quadratic_function/_gradient (benchmark.cpp:16-56),
 *                               quadratic/quadratic_grad (main.cpp:7-21 = functions.cpp:6-24),
 *                               evaluated on the GPU; LBFGS_OBJ_HOST calls user callbacks.
 *   - lbfgs_dev_*               the BLAS-1 primitives of vector_utils.cpp:32-86 on the device.
 *
 * Differences in form, not in semantics: the reference takes std::vector / std::function by
 * value and allocates device memory per call; here a persistent context owns the device
 * memory (allocation amortised) and x0 / x are caller-owned host buffers. Errors are status
 * codes, never exit() (reference: checkCudaError -> exit, L-BFGS.cu:76-92) and never C++
 * exceptions across the ABI; the C++ header lbfgs.h restores the reference's exceptions.
 * Non-convergence and line-search failure are not errors, as in the reference: the status
 * says why, and the same messages as the reference are printed unless LBFGS_FLAG_QUIET.
 *
 * Threading: one host thread per context. All vectors are fp64.
 */
#ifndef LBFGS_HIP_H
#define LBFGS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LBFGS_HIP_ABI_VERSION 2

typedef struct lbfgs_ctx lbfgs_ctx;

/* objectives */
enum {
    LBFGS_OBJ_ROSENBROCK = 0,     /* benchmark.cpp:58-81 */
    LBFGS_OBJ_QUAD_TRIDIAG = 1,   /* generate_quadratic_function(n), benchmark.cpp:16-56 */
    LBFGS_OBJ_QUAD_SEPARABLE = 2, /* main.cpp:7-21 */
    LBFGS_OBJ_HOST = 3,           /* user callbacks (lbfgs_host_fn) */
    LBFGS_OBJ_DENSE_QUAD = 4      /* f = x'Ax + b'x on the device (lbfgs_set_dense_quadratic) */
};

/* line searches, lbfgs.cpp:40-70 */
enum {
    LBFGS_LS_BACKTRACKING = 0,      /* "backtracking"       line_search.cpp:19-30 */
    LBFGS_LS_INTERPOLATION = 1,     /* "interpolation"      line_search.cpp:57-121 */
    LBFGS_LS_WOLFE = 2,             /* "wolfe"              line_search.cpp:125-189 */
    LBFGS_LS_BACKTRACKING_WOLFE = 3 /* "backtracking_wolfe" line_search.cpp:33-55 */
};

/* status (>= 0) and errors (< 0) */
enum {
    LBFGS_STATUS_CONVERGED = 0, /* "Converged!"                          lbfgs.cpp:80-84 */
    LBFGS_STATUS_MAX_ITER = 1,  /* "Maximum iterations reached"          lbfgs.cpp:201-202 */
    LBFGS_STATUS_LS_FAILED = 2, /* "Warning: Line search failed ..."     lbfgs.cpp:164-168 */
    LBFGS_STATUS_RUNNING = 3,   /* lbfgs_solver_step budget used, not finished */
    LBFGS_ERR_BAD_ARG = -1,     /* incl. unknown line search (lbfgs.cpp:69 invalid_argument) */
    LBFGS_ERR_HIP = -2,
    LBFGS_ERR_RCCL = -3,
    LBFGS_ERR_NOMEM = -4,
    LBFGS_ERR_STATE = -5,
    LBFGS_ERR_CALLBACK = -6
};

/* flags */
#define LBFGS_FLAG_VERBOSE 1u /* print "Iteration k, f = .., |grad| = .." (lbfgs.cpp:76-78) */
#define LBFGS_FLAG_QUIET 2u   /* suppress the reference's stdout messages */
#define LBFGS_FLAG_TRACE 4u   /* record per-iteration f, |g|, alpha, x checksums (tests) */
/* one kernel per BLAS-1 operation, as parallel-implementation/L-BFGS.cu:208-280 composes
 * cuBLAS calls (separate dot and axpy passes, materialised trial points, f re-evaluated at
 * the commit). Same iterates, bit for bit, as the fused default; single rank, device
 * objectives only. BASELINE configs[1] ("unfused per-vector kernels"). */
#define LBFGS_FLAG_UNFUSED 8u
/* vector-free (Gram-matrix) L-BFGS: the two-loop recursion on the host over the Gram matrix of
 * the basis {s_i, y_i, g}; one fused device pass per iteration forms d, takes the first trial,
 * commits and reduces the new Gram rows (~2m+6 vector passes instead of 8m+3). The same
 * algorithm in exact arithmetic; rounding differs from the reference's operation order
 * (f within 1e-10 over horizons comparable to the canonical order's). Single rank,
 * device objectives, m <= 20. */
#define LBFGS_FLAG_VECTOR_FREE 16u
/* host-callback objectives: call f and grad exactly as the reference does, call for call
 * (its re-evaluations of f(x) in every line search, line_search.cpp:24,42,65,133, and of f and
 * grad at x_new after it, lbfgs.cpp:160,171), for callables with side effects or counters.
 * Default: one f and at most one grad call per distinct point (same iterates either way for a
 * deterministic objective). */
#define LBFGS_FLAG_REFERENCE_CALLS 32u
/* the CUDA path's semantics, LBFGS_CUDA of parallel-implementation/L-BFGS.cu:105-380, for callers
 * that want its iterates rather than the sequential LBFGS's: the first-loop pairs with s.y <= 1e-10
 * skipped (their alpha and rho kept from the last time the ring slot was used, :222-223), gamma = 1
 * when y.y or s.y fail (:237-262), the ring slot k % m written unconditionally (:332), every line
 * search given the iteration-0 gradient (:199,293), the line searches of
 * parallel-implementation/line_search.cpp (their 0.5 floors, the bisection Wolfe search, the
 * safeguarded cubic), convergence tested after the step with <= (:353), and its stdout lines
 * ("alpha: ..", "Iteration k: norm_g = ..", "Optimum value: .."). Single rank, device objectives;
 * every vector stays on the device, scalars round-trip per dot as the cuBLAS host-pointer calls do.
 * Bit-exact with the oracle's restatement of that path (ORC_CANON); parity with the CUDA program
 * itself is unpinned (no CUDA toolchain here), its line searches are pinned against
 * line_search.cpp compiled here. Trace entry k = the state iteration k prints after its step.
 * The caller passes the CUDA path's constants with it (lbfgs_constants_cuda: parallel-
 * implementation/constants.h, C2 = 0.7); the flag does not change the constants it is given. */
#define LBFGS_FLAG_CUDA_COMPAT 64u
/* with LBFGS_FLAG_CUDA_COMPAT: the string-less LBFGS_CUDA of the four variant files instead, each
 * with its own inline line search (the line_search argument names the file): backtracking =
 * L-BFGS-Backtracking.cu:293-348 (correct-sign Armijo, 0.5 when the step falls below 1e-10, the
 * "very small step size" warning below 1e-4), interpolation = L-BFGS-Interpolation.cu:259-358,
 * wolfe = L-BFGS-Wolfe.cu:259-366, backtracking_wolfe = L-BFGS-Backtracking_Wolfe.cu:256-415.
 * Their searches take the current gradient, f(x) from the host copy of the last trial point the
 * previous search transferred (x0 at k = 0), and the interpolation and Wolfe searches start
 * f_prev / f_lo from f(x0) every iteration. Parity unpinned (the searches are inline in .cu files). */
#define LBFGS_FLAG_CUDA_VARIANT 128u

typedef struct {
    double c1;                 /* C1 = 1e-4                  config.h:5 */
    double c2;                 /* C2 = 0.9 (constants.h: 0.7) config.h:6 */
    double initial_step;       /* INITIAL_STEP_SIZE = 1.0    config.h:9 */
    double backtracking_alpha; /* BACKTRACKING_ALPHA = 0.5   config.h:12 */
    double backtracking_tol;   /* BACKTRACKING_TOL = 1e-8    config.h:13 */
    double wolfe_interp_min;   /* WOLFE_INTERP_MIN = 1e-10   config.h:16 */
    double wolfe_interp_max;   /* WOLFE_INTERP_MAX = 10.0    config.h:17 (unused, as in ref) */
} lbfgs_constants;

void lbfgs_constants_default(lbfgs_constants* k); /* sequential-implementation/config.h */
void lbfgs_constants_cuda(lbfgs_constants* k);    /* parallel-implementation/constants.h */

/* Dense quadratic objective (LBFGS_OBJ_DENSE_QUAD): f(x) = x'Ax + b'x, grad = 2Ax + b, A symmetric
 * n x n row-major (n <= 65536), evaluated on the device - the known-answer problems of the
 * reference's sequential-implementation/matrices.h (mat<n>, linear<n>, minimum<n>). Row i of Ax is
 * one wavefront (lane l sums j = l, l+64, ... with fma, then a butterfly); f sums the terms
 * x_i (Ax)_i + b_i x_i in the canonical order (restated by the oracle). Uploads A and b into the
 * context; one rank. */
int lbfgs_set_dense_quadratic(lbfgs_ctx* ctx, const double* A, const double* b);

/* Host-callback objective (LBFGS_OBJ_HOST). x has n entries (global vector). */
typedef double (*lbfgs_host_f)(const double* x, int64_t n, void* user);
typedef void (*lbfgs_host_grad)(const double* x, int64_t n, double* g_out, void* user);
typedef struct {
    lbfgs_host_f f;
    lbfgs_host_grad grad;
    void* user;
} lbfgs_host_fn;

typedef struct {
    int iterations;      /* iterations performed (k at exit) */
    int status;          /* LBFGS_STATUS_* */
    double f;            /* f at the returned x's iterate (f_current) */
    double gnorm;        /* |g| at the last convergence test */
    int64_t trials_f;    /* extra f-only trial passes */
    int64_t trials_fg;   /* extra f+grad trial passes */
    int64_t commits;     /* commit passes (incl. the fused speculative ones) */
    int64_t passes;      /* device kernel launches */
    double bytes;        /* algorithmic HBM bytes moved by all launches (this rank) */
    double seconds;      /* wall time of the solve / step call */
    int h_min, h_max;    /* history pairs stored at the top of the iterations this call ran
                          * (h of SURVEY.md 8(d)'s B_iter; -1 when the call ran none) */
    int64_t f_calls;     /* host-callback objective: f / grad callbacks since solver init */
    int64_t grad_calls;
} lbfgs_result;

/* "src=<16 hex digits of sha256 over the library's sources> built=<date time> arch=gfx950":
 * identifies the sources a loaded library was built from (build provenance) */
const char* lbfgs_build_info(void);

/* Small n (cooperative iteration): iteration k + 1 is queued on the device behind iteration k
 * before the host has read k's results, and runs only if its prologue finds every host decision
 * in between as assumed (first trial taken, pair stored, no stop, valid rho and gamma); the host
 * then takes it instead of launching. Launches the host took / discarded since solver init.
 * LBFGS_SPEC=0 turns it off (bit-identical iterates either way). */
int lbfgs_spec_stats(const lbfgs_ctx* c, int64_t* adopted, int64_t* dropped);

/* Small n (one rank, a cooperative size, device objective): once a line search needs a trial pass
 * beyond the commit's first one, the rest of the search - and the commit at the step it finds -
 * runs in one cooperative launch instead of a launch and a host round trip per trial pass
 * (DESIGN.md §4.3). Launches and commits taken that way since solver init. LBFGS_DEV_SEARCH=0
 * turns it off (bit-identical iterates and counters either way). */
int lbfgs_search_stats(const lbfgs_ctx* c, int64_t* launches, int64_t* commits);

/* ---- context ---------------------------------------------------------------------------- */
/* n: global problem size; m: history length (1..64); device: HIP device ordinal. */
int lbfgs_ctx_create(lbfgs_ctx** out, int64_t n, int m, int device);
/* One process per GPU: shard the vectors across 'world' ranks (world | 8) with an RCCL
 * communicator created from 'unique_id' (128 bytes, from lbfgs_unique_id on rank 0), and/or
 * the xGMI peer exchange (lbfgs_peer_*). world = 1 with a unique_id builds a one-rank
 * communicator and routes every reduction through the sharded path's RCCL all-gather
 * (diagnostic: the RCCL leg on a one-GPU box, bit-identical to lbfgs_ctx_create). */
int lbfgs_ctx_create_sharded(lbfgs_ctx** out, int64_t n, int m, int device, int rank, int world,
                             const void* unique_id);
int lbfgs_unique_id(void* out128);
/* HIP devices visible to this process (0 when none) */
int lbfgs_device_count(void);
/* unique_id may be NULL: no RCCL communicator; the context then exchanges its reductions only
 * through the xGMI peer mailboxes below (lbfgs_peer_*), which must be connected and enabled
 * before the first solve.
 *
 * xGMI peer exchange. Every sharded context owns a small mailbox in uncached device memory;
 * a one-workgroup kernel stores the rank's group partials straight into every peer's mailbox
 * and polls its own (no collective library on the solver's critical path).
 * Bootstrap, on every rank: lbfgs_peer_handle -> all-gather the handles (any host channel,
 * e.g. torch.distributed gloo) -> lbfgs_peer_connect (maps the peers, self-tests the exchange,
 * up to ~30 s waiting for peers) -> agree on success across ranks -> lbfgs_peer_enable(1) on all
 * or none. A peer that stops answering mid-solve ends the wait after 60 s (LBFGS_XGMI_TIMEOUT)
 * with LBFGS_ERR_RCCL instead of a hang. */
#define LBFGS_PEER_HANDLE_BYTES 64
int lbfgs_peer_handle(lbfgs_ctx* ctx, void* out /* LBFGS_PEER_HANDLE_BYTES */);
int lbfgs_peer_connect(lbfgs_ctx* ctx, const void* handles /* world x LBFGS_PEER_HANDLE_BYTES */);
/* on = 1: exchanges through the mailboxes (after a successful connect on every rank); on = 0: back
 * to the RCCL communicator (LBFGS_ERR_STATE without one). Every rank must make the same choice. */
int lbfgs_peer_enable(lbfgs_ctx* ctx, int on);
/* A sharded context created without a unique_id takes an RCCL communicator afterwards (every rank
 * calls it with the same id). Every RCCL communicator of the library is created on a helper thread
 * and waited for with a bound (LBFGS_RCCL_TIMEOUT seconds, default 60), and so are the host's waits
 * on its collectives: a rank that never joins, a stalled bootstrap or a collective that does not
 * complete returns LBFGS_ERR_RCCL (the stalled init thread abandoned, a stalled collective's
 * communicator aborted), never a hang. This call also runs
 * one all-gather through the new communicator under the same bound. Exchanges stay on the
 * mailboxes until lbfgs_peer_enable(ctx, 0). */
int lbfgs_rccl_attach(lbfgs_ctx* ctx, const void* unique_id /* 128 bytes, lbfgs_unique_id */);
/* 0: one rank, 1: RCCL all-gathers, 2: xGMI peer mailboxes, 3: host group (emulated ranks) */
int lbfgs_exchange_backend(const lbfgs_ctx* ctx);
/* 1 when the mailbox exchanges of the two-loop are folded into the passes (the producing pass
 * pushes its reduction to the peers, the consuming pass polls it: no exchange launch between
 * them). On by default when every peer runs on a GPU of its own; LBFGS_XGMI_FOLD=2
 * forces it for ranks sharing a GPU, 0 turns it off. */
int lbfgs_exchange_fold(const lbfgs_ctx* ctx);
/* collective diagnostic (every rank calls it with the same arguments): `iters` back-to-back
 * exchanges of a `components`-wide result slot (8 = a two-loop reduction, up to 96) through
 * backend 1 (RCCL) or 2 (xGMI mailboxes); *us = host wall time per exchange */
int lbfgs_exchange_latency(lbfgs_ctx* ctx, int backend, int components, int iters, double* us);
/* LBFGS_CU_PARTITION=1 at context creation (sharded ranks sharing one GPU: tests and one-card
 * rehearsals of a multi-GPU run): the rank's solver stream is confined to its own cus / world
 * CUs, disjoint from every other rank's, so the ranks make progress as on distinct GPUs and the
 * folded exchanges run ungated, as across GPUs. Returns the rank's CU count, 0 when not
 * partitioned. */
int lbfgs_cu_partition(const lbfgs_ctx* ctx);
/* Diagnostic: the cooperative forms' grid caps in canonical segments, from each kernel's own
 * occupancy x the stream's CUs: *coop_max for the one-launch iteration (k_coop_iter), *search_max
 * for the device-resident line searches (k_coop_search; 0 when off); *fallbacks = device searches
 * whose grid barrier timed out (LBFGS_SEARCH_TIMEOUT, 2 s) and that the host loop redid. */
int lbfgs_coop_info(const lbfgs_ctx* ctx, int* coop_max, int* search_max, int* fallbacks);
/* The host's waits for device results poll a completion word in pinned memory. LBFGS_WAIT=adaptive
 * (default): a wait expected to last over 0.5 ms (its word's last four waits) sleeps through most of
 * it and spins for the rest; LBFGS_WAIT=spin: spin throughout. *slept_s = seconds slept so far,
 * *waits = waits completed, *adaptive = the mode. */
int lbfgs_wait_stats(const lbfgs_ctx* ctx, double* slept_s, uint64_t* waits, int* adaptive);
/* Vector allocation (LBFGS_VEC_ALLOC at context creation): by default ("pool") every
 * n-vector of 64 MiB .. 2 GiB is a physically contiguous device allocation (+3 % at n = 1e8) that is
 * never returned to the driver - a freed one waits in a process-wide pool (at most LBFGS_VEC_POOL_GB,
 * 32 GiB) for the next vector of its size - because freeing contiguous allocations corrupts later
 * ones on this ROCm stack; other sizes, "plain", and the pool's overflow are plain hipMalloc;
 * "contiguous" (A/B only) frees them. Returns how many of the context's vectors asked for a
 * contiguous allocation and got a plain one. */
int lbfgs_vector_fallbacks(const lbfgs_ctx* ctx);
/* The context's allocation mode (0 pool, 1 plain, 2 contiguous) or LBFGS_ERR_BAD_ARG; *pooled = its
 * vectors taken from or added to the pool, *held_gb = GiB the process's pool owns. */
int lbfgs_vector_pool(const lbfgs_ctx* ctx, int* pooled, double* held_gb);
/* Diagnostic (no reference counterpart): `launches` back-to-back streams of 3 reads + 1 write
 * over a scratch work vector and the context's history vectors (y, s of the pair pool, another
 * pair every launch as the two-loop passes read them) in the passes' geometry and cache policy;
 * the scratch vector starts as a copy of y_0 (random data: zeros stream ~3 % faster);
 * the solve's own vectors and state are untouched. *us = mean microseconds per
 * launch, *bytes = this rank's bytes per launch (32 n_loc). bench.py reports this box's rate for
 * the passes' access pattern beside the solver's. Call between lbfgs_solver_step calls of an
 * initialised solve. */
int lbfgs_stream_probe(lbfgs_ctx* ctx, int launches, double* us, double* bytes);
/* The same with the two-loop pass's machinery added piece by piece (the gap between
 * k_axpy_dot and the probe): variant 0 = lbfgs_stream_probe; 1 = alpha != 0 (the work vector
 * changes); 2 = + the pass's segment reduction, partials stored plainly (no stage 2); 3 = + the
 * collect stage 2 into a scratch result slot; 4 / 5 = the product's k_axpy_dot launch itself (source
 * slot read, collect stage 2) with alpha = 0 / != 0, chained through two scratch slots; 6 = the
 * commit's 4 reads + 4 writes (k_commit's loads, stores and cache policies, no stencil, f or
 * reductions) into scratch vectors: *bytes = 64 n_loc. Variants 8-13: 0-5 on the solver's own
 * work vector q instead of a scratch one (the next iteration rewrites q before reading it);
 * variants 16-22: 0-6 with the scratch vector filled with a copy of y_0 first (not zeros). */
int lbfgs_stream_probe_variant(lbfgs_ctx* ctx, int variant, int launches, double* us, double* bytes);
/* Diagnostic: the probe's stream (variant 0, alpha = 0) over three of the context's own vectors,
 * by index in allocation order: 0-7 x, g, xn, gn, d, q, r, gt; 8 + 2p S_p, 9 + 2p Y_p; 8 + 2(m + 1)
 * a scratch vector allocated for the call. The first is written back unchanged. */
int lbfgs_stream_probe_vectors(lbfgs_ctx* ctx, int q, int y, int s, int launches, double* us);
/* Diagnostic: the device address of vector k (the indexing above; not the scratch one) */
int lbfgs_vector_address(lbfgs_ctx* ctx, int k, uint64_t* addr);
/* Emulated ranks: 'world' contexts driven by threads of ONE process (e.g. on one GPU, one
 * stream each) exchange their reductions through host memory instead of RCCL. Same data path
 * and results as the RCCL shards; used to test sharding on a single GPU. */
typedef struct lbfgs_host_group lbfgs_host_group;
int lbfgs_host_group_create(lbfgs_host_group** out, int world);
void lbfgs_host_group_destroy(lbfgs_host_group* grp);
int lbfgs_ctx_create_emulated(lbfgs_ctx** out, int64_t n, int m, int device, int rank,
                              lbfgs_host_group* grp);
void lbfgs_ctx_destroy(lbfgs_ctx* ctx);
const char* lbfgs_last_error(const lbfgs_ctx* ctx);
/* this rank's slice [elem_lo, elem_lo + n_loc) of the global vector */
int lbfgs_local_range(const lbfgs_ctx* ctx, int64_t* elem_lo, int64_t* n_loc);
/* the shard plan without a device: rank's slice for (n, world); LBFGS_ERR_BAD_ARG when some
 * rank would own no segment (n <= (8 - 8/world) * 1024 * L) or world does not divide 8 */
int lbfgs_shard_range(int64_t n, int rank, int world, int64_t* elem_lo, int64_t* n_loc);

/* ---- solve (drop-in for LBFGS / LBFGS_CUDA) ------------------------------------------- */
/* x0_host / x_out_host: global vectors of n doubles (each rank passes the full vector; a
 * sharded rank writes only its slice of x_out_host). cb may be NULL unless objective is
 * LBFGS_OBJ_HOST; k may be NULL (config.h constants). */
int lbfgs_minimize(lbfgs_ctx* ctx, int objective, const lbfgs_host_fn* cb, int line_search,
                   const lbfgs_constants* k, const double* x0_host, double* x_out_host,
                   int max_iterations, double tolerance, unsigned flags, lbfgs_result* out);

/* stepping API: init once, then run iterations in chunks (benchmarks, checkpoints) */
int lbfgs_solver_init(lbfgs_ctx* ctx, int objective, const lbfgs_host_fn* cb, int line_search,
                      const lbfgs_constants* k, const double* x0_host, double tolerance,
                      unsigned flags);
int lbfgs_solver_step(lbfgs_ctx* ctx, int max_steps, lbfgs_result* out);
int lbfgs_get_x(lbfgs_ctx* ctx, double* x_out_host);
int lbfgs_sync(lbfgs_ctx* ctx);

/* messages printed by the last solve (the reference's stdout lines), NUL-terminated */
int lbfgs_messages(const lbfgs_ctx* ctx, char* buf, int cap);
/* per-iteration trace (LBFGS_FLAG_TRACE): entry k = state at the top of iteration k */
int lbfgs_trace_len(const lbfgs_ctx* ctx);
int lbfgs_trace_get(const lbfgs_ctx* ctx, double* f, double* gnorm, double* alpha,
                    uint64_t* c1, uint64_t* c2, int cap);
/* switch the trace on or off between lbfgs_solver_step calls of an initialised solve (entries
 * recorded so far are kept): bench.py traces the untimed history fill and warm-up, whose f / |g|
 * it checks against the reference, and times the steps after it untraced (the x checksums are
 * extra passes) */
int lbfgs_trace_enable(lbfgs_ctx* ctx, int on);

/* ---- line search alone (line_search.h:10-26 on the GPU) -------------------------------- */
/* Step size along d from x (gradient g at x) by one of the four line searches, every trial on
 * the device (or through cb for LBFGS_OBJ_HOST). Single rank; ends any solve in progress. */
int lbfgs_line_search(lbfgs_ctx* ctx, int objective, const lbfgs_host_fn* cb, int line_search,
                      const lbfgs_constants* k, const double* x_host, const double* d_host,
                      const double* g_host, double* alpha_out);

/* ---- device primitives (vector_utils.cpp:32-86 on the GPU) ----------------------------- */
/* op 0: out = alpha * a (scalarProduct), 1: out = a + b (add), 2: out = -a (negative) */
int lbfgs_dev_elementwise(lbfgs_ctx* ctx, int op, const double* a_host, const double* b_host,
                          double alpha, double* out_host);
/* Host-buffer convenience forms over the context's n (global vectors). Results are the
 * canonical fixed-order device reductions. */
int lbfgs_dev_dot(lbfgs_ctx* ctx, const double* a_host, const double* b_host, double* out);
int lbfgs_dev_norm(lbfgs_ctx* ctx, const double* v_host, double* out);
int lbfgs_dev_objective(lbfgs_ctx* ctx, int objective, const double* x_host, double* f_out,
                        double* g_out_host /* nullable */);
/* trial evaluation at x + alpha d: f, and (g_out_host != NULL) g_t and g_t . d */
int lbfgs_dev_trial(lbfgs_ctx* ctx, int objective, const double* x_host, const double* d_host,
                    double alpha, double* f_out, double* g_out_host, double* dphi_out);
/* one full device two-loop recursion (lbfgs.cpp:94-143) for a given history, oldest first.
 * S_host/Y_host: arrays of h pointers to n-vectors. Writes d and g.d. */
int lbfgs_dev_twoloop(lbfgs_ctx* ctx, const double* g_host, const double* const* S_host,
                      const double* const* Y_host, int h, double* d_out_host, double* gd_out);

/* ---- profiling (benchmarks) ------------------------------------------------------------ */
enum {
    LBFGS_KERNEL_DOT = 0, LBFGS_KERNEL_AXPY_DOT, LBFGS_KERNEL_MID, LBFGS_KERNEL_AXPY2_DOT,
    LBFGS_KERNEL_LAST, LBFGS_KERNEL_NEGDOT, LBFGS_KERNEL_EVAL, LBFGS_KERNEL_TRIAL_F,
    LBFGS_KERNEL_TRIAL_FG, LBFGS_KERNEL_COMMIT, LBFGS_KERNEL_POINT, LBFGS_KERNEL_CHECKSUM,
    LBFGS_KERNEL_UPDATE, LBFGS_KERNEL_VF_COMMIT, LBFGS_KERNEL_VF_DIR,
    LBFGS_KERNEL_SMALL_ITER, LBFGS_KERNEL_GROUP_REDUCE /* stage 2 of the reductions */,
    /* sharded runs: each reduction's exchange between ranks (the xGMI mailbox kernel, waiting
     * for the peers included, or the RCCL all-gather); bytes 0 */
    LBFGS_KERNEL_EXCHANGE,
    LBFGS_KERNEL_COUNT
};
void lbfgs_prof_enable(lbfgs_ctx* ctx, int on);
void lbfgs_prof_reset(lbfgs_ctx* ctx);
/* HIP-event time on the solver stream, launches and algorithmic bytes for a kernel kind */
int lbfgs_prof_get(lbfgs_ctx* ctx, int kind, double* ms, int64_t* launches, double* bytes);

#ifdef __cplusplus
}
#endif
#endif
