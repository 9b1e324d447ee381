// lbfgs_kernels.hip — lbk_* entry points: lifecycle, memory, the two-loop passes, objectives,
// results, exchange, profiling (kernels and helpers: lbfgs_kernels_impl.h).
#include "lbfgs_kernels_impl.h"

#include <atomic>
#include <mutex>
#include <unordered_set>
#include <thread>

// A slot the host reads whose launch leaves no completion word (stage 2 in several groups, the
// sharded exchange): this launch, queued behind everything issued so far, copies the slot from
// the device to its host mirror and then stores the epoch word the host polls (small_wait).
// Waiting on the stream instead (hipStreamSynchronize) registers an asynchronous handler with
// the runtime on every call, and the runtime thread serving them spins: ~1 core per process
// beside the waiting thread (tools/thread_probe.py, profiles/r05/config4_cpu/; eight such ranks
// exhausted a 16-CPU quota and configs[4] ran at half speed on one card).
__global__ __launch_bounds__(256) void k_slot_publish(const double* __restrict__ src, double* dst, int n,
                                                      unsigned long long* word, unsigned long long epoch) {
    for (int i = (int)threadIdx.x; i < n; i += 256) dst[i] = src[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(word, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" {

void xfer_pool_free(lbk_ctx* c);  // staged transfers' pinned pool (below)

int lbk_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int lbk_unique_id(void* out128) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return -3;
    memcpy(out128, &id, sizeof id);
    return 0;
}

// The factor is chosen from the 512-minimum segment length L0 (not the canonical L, which is
// longer for LBK_MIDL_LO <= n <= LBK_MIDL_HI); the vector-free segment length is F x canonical L.
int lbk_vf_factor(int64_t n) {
    const int64_t per = (n + LBK_SEGS - 1) / LBK_SEGS;
    int64_t L = ((per + 127) / 128) * 128;
    if (L < 512) L = 512;
    int F = 1;
#ifdef LBK_VF_FMAX  // experiments: cap the factor (1 = the original vector-free geometry)
    const int fmax = LBK_VF_FMAX;
#else
    const int fmax = 8;
#endif
    while (F < fmax && 2 * F * L <= 8192 && (n + 2 * F * L - 1) / (2 * F * L) >= 1024) F *= 2;
    return F;
}

int lbk_geometry_plan(int64_t n, int rank, int world, lbk_geo* out) {
    if (n < 1 || world < 1 || (LBK_GROUPS % world) != 0 || rank < 0 || rank >= world) return -1;
    lbk_geo& G = *out;
    G.n = n;
    // segment length: whole 128-element rows, at least 512 (one row per wave); rows rather
    // than 512-multiples keep all 8 groups populated for n >= 7.3e6 (sharding over 8 ranks)
    const int64_t per = (n + LBK_SEGS - 1) / LBK_SEGS;
    G.L = ((per + 127) / 128) * 128;
    // minimum segment length: 2048 elements where n cannot shard anyway (n <= 4 * 1024 * 512:
    // two ranks would need more than 4096 segments of 512), from 2^16 up; 512 elsewhere. Fewer,
    // longer segments bring mid n under the cooperative (<= 256 segments) and deferred
    // (<= 1024) stage-2 forms: measured +6..29 % at n = 1e5..2e6, vector-free +16..60 % from
    // 2^18 (profiles/r01/lmin_ab.txt; below 2^18 its commit keeps 512, see vf_base_len). The
    // oracle's orc_canon_geometry states the rule.
    const int64_t lmin = (n >= LBK_MIDL_LO && n <= LBK_MIDL_HI) ? LBK_MIDL : 512;
    if (G.L < lmin) G.L = lmin;
#ifdef LBK_DEBUG_SEGLEN  // timing experiments only (tools/gpu_ab_shardgeo.sh): breaks the canonical order
    G.L = LBK_DEBUG_SEGLEN;
#endif
    G.nseg = (n + G.L - 1) / G.L;
    G.rank = rank;
    G.world = world;
    G.g_lo = rank * (LBK_GROUPS / world);
    G.g_hi = (rank + 1) * (LBK_GROUPS / world);
    G.seg_lo = std::min<int64_t>((int64_t)G.g_lo * LBK_SEG_PER_GROUP, G.nseg);
    G.seg_hi = std::min<int64_t>((int64_t)G.g_hi * LBK_SEG_PER_GROUP, G.nseg);
    G.elem_lo = std::min<int64_t>(G.seg_lo * G.L, n);
    const int64_t elem_hi = std::min<int64_t>(G.seg_hi * G.L, n);
    G.n_loc = elem_hi - G.elem_lo;
    G.vf_f = lbk_vf_factor(n);
    // every rank must own at least one segment (n > (8 - 8/world) * 1024 * L)
    if (world > 1 && (G.nseg <= (int64_t)(LBK_GROUPS - LBK_GROUPS / world) * LBK_SEG_PER_GROUP)) return -7;
    return 0;
}

static int rccl_init(lbk_ctx* c, const void* nccl_id);

int lbk_create(lbk_ctx** out, int device, int64_t n, int rank, int world, const void* nccl_id, lbk_group* grp) {
    *out = nullptr;
    lbk_ctx* c = new (std::nothrow) lbk_ctx();
    if (!c) return -4;
    c->device = device;
    lbk_geo& G = c->geo;
    const int prc = lbk_geometry_plan(n, rank, world, &G);
    c->ghost_slot = -1;
    c->grp = grp;
    if (prc != 0) {
        snprintf(c->err, sizeof c->err, "cannot shard n=%lld over %d ranks (rank %d)", (long long)n, world, rank);
        *out = c;
        return -1;
    }
    if (world > 1 && vf_base_len(n, G.L) != G.L) {  // see vf_base_len: ranks must own whole vf segments
        snprintf(c->err, sizeof c->err, "n=%lld: vector-free base length differs from the canonical one under sharding",
                 (long long)n);
        *out = c;
        return -1;
    }
    // front pad 32 doubles: ghost at [-1] and element 0 on a 256-B boundary, so every 1-KiB
    // row load/store covers whole cache lines; back: whole rows + halo
    // non-temporal streaming of the history (the work vectors q/r/d keep the temporal policy,
    // LBK_WORK_TEMPORAL) once vectors no longer fit comfortably in the 256 MiB Infinity Cache.
    // Two-loop passes: -2 % at n_loc = 1e7, +1.3 % at 1.25e7, +4 % at 1e8; vector-free passes
    // (2m+6 vectors each): +1.5 % at 2e6, +5 % at 1e7 and above (profiles/r01/nt_threshold_ab.txt,
    // work_temporal_ab.txt). Override for both: LBFGS_NT=0/1
    c->nt = (G.n_loc * 8 > (88ll << 20)) ? 1 : 0;
    c->nt_vf = (G.n_loc * 8 > (12ll << 20)) ? 1 : 0;
    if (const char* e = getenv("LBFGS_NT")) c->nt = c->nt_vf = atoi(e) != 0;
    // stage-2 reduction: separate 8-workgroup kernel by default; in-launch tickets only for
    // tiny grids where the extra launch dominates (override: LBFGS_TICKET=0/1)
    // sharded runs with long segments too: one rank of an 8-GPU n = 1e8 run (1017 workgroups of
    // L = 12288 per pass) measured 1 % faster with tickets on one GPU (tools/gpu_ab_shardgeo.sh),
    // and the stage-2 launch before each all-gather disappears
    c->ticket = ((G.seg_hi - G.seg_lo) <= 64 || (world > 1 && G.L >= 8192)) ? 1 : 0;
    c->ticket_env = -1;
    if (const char* e = getenv("LBFGS_TICKET")) c->ticket = c->ticket_env = atoi(e) != 0;
    c->vec_doubles = LBK_FRONT + ((G.n_loc + 511) / 512) * 512 + 512;
    // measured (profiles/r01/coop_ab.txt): +48 % at n = 1e4 (14-15k -> 22k it/s), +41 % at 3e4,
    // +22 % at 1e5 (196 segments); -22 % at 391 segments and -38 % at 508, where the barrier's
    // fan-in and every workgroup's read of all partials outweigh the saved launches. Bit-identical
    // (tests/test_gpu_parity.py::test_cooperative_iteration_bit_exact). LBFGS_COOP=<segments>.
    // with the mid-n 2048-element segments (4x the work per workgroup) the crossover to the
    // deferred stage 2 comes earlier: at 245 segments (n = 5e5) deferred runs 6.8-7.0k it/s
    // against 5.4-5.6k cooperative, at 196 they tie, at 147 cooperative leads 7.9-8.1k to
    // 7.0-7.8k (profiles/r01/coop_long_ab.txt). Round 2's flagged partials and speculative
    // launches move it: at 245 segments (n = 5e5) cooperative 8.26k against deferred 6.61k, at
    // 342 (7e5) deferred leads 5.07k to 4.81k (profiles/r02/small_n/coop_limit_ab.txt)
    c->coop_max = 256;
    if (const char* e = getenv("LBFGS_COOP")) c->coop_max = std::min(atoi(e), LBK_COOP_SEGMAX);  // max segments
    // small n, every line search: the trials after the commit's first one, and the recommit at the
    // step found, in one cooperative launch (k_coop_search) instead of a launch and a host round
    // trip each; LBFGS_DEV_SEARCH=0: the host loop (LBFGS_DEV_WOLFE, its round-4 name, is read too)
    c->dev_wolfe = 1;
    if (const char* e = getenv("LBFGS_DEV_WOLFE")) c->dev_wolfe = atoi(e) != 0;
    if (const char* e = getenv("LBFGS_DEV_SEARCH")) c->dev_wolfe = atoi(e) != 0;
    // the device search's wait at each grid barrier (2 s; tests set 0 to force its time-out path,
    // after which the host loop redoes the search)
    c->search_timeout_s = 2.0;
    if (const char* e = getenv("LBFGS_SEARCH_TIMEOUT")) c->search_timeout_s = std::max(0.0, atof(e));
    c->wait_adaptive = 1;
    if (const char* e = getenv("LBFGS_WAIT")) c->wait_adaptive = strcmp(e, "spin") != 0;
    c->vec_mode = LBK_VEC_POOL;
    if (const char* e = getenv("LBFGS_VEC_ALLOC"))
        c->vec_mode = !strcmp(e, "plain") ? LBK_VEC_PLAIN : !strcmp(e, "contiguous") ? LBK_VEC_CONTIGUOUS : LBK_VEC_POOL;
    c->vec_pool_cap = size_t(32) << 30;
    if (const char* e = getenv("LBFGS_VEC_POOL_GB")) c->vec_pool_cap = (size_t)(std::max(0.0, atof(e)) * double(size_t(1) << 30));
    c->vec_pool_min = kPoolMinBytes;
    if (const char* e = getenv("LBFGS_VEC_POOL_MIN_MB")) c->vec_pool_min = (size_t)(std::max(0.0, atof(e)) * double(1 << 20));
    c->rccl_timeout_s = 60.0;
    if (const char* e = getenv("LBFGS_RCCL_TIMEOUT")) c->rccl_timeout_s = std::max(0.5, atof(e));
    // test hook "stall_ms,wait_s": a device-side stall ahead of every collective and the bound of the
    // host's waits on collectives (the communicator's init keeps LBFGS_RCCL_TIMEOUT)
    if (const char* e = getenv("LBFGS_DEBUG_RCCL_STALL")) {
        double st = 0.0, ws = 0.0;
        if (sscanf(e, "%lf,%lf", &st, &ws) == 2 && st > 0.0 && ws > 0.0 &&
            hipHostMalloc((void**)&c->stall_release_h, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent) ==
                hipSuccess &&
            hipHostGetDevicePointer((void**)&c->stall_release_d, c->stall_release_h, 0) == hipSuccess) {
            *c->stall_release_h = 0;
            c->rccl_stall_ms = st;
            c->rccl_wait_s = ws;
        }
    }
    c->pend_slot = -1;
    c->xf_slot = -1;
    // folded exchanges over the mailboxes: 1 (default) when every peer has a GPU of
    // its own; 2 also for ranks sharing a GPU (tests on grids that fit beside each other); 0 off
    c->fold_env = 1;
    if (const char* e = getenv("LBFGS_XGMI_FOLD")) c->fold_env = atoi(e);
    // measured (profiles/r01/defer_ab.txt): +21..32 % at n = 3e5 (586 segments); -14 % at 1954
    // segments and worse beyond, where every workgroup forms two or more group trees
    c->defer_max = LBK_SEG_PER_GROUP;
    if (const char* e = getenv("LBFGS_DEFER")) c->defer_max = atoi(e);  // max segments
    // measured +1 % at n = 1e7 (default and vector-free), +1 % vector-free and neutral default at
    // 1e8 (profiles/r01/rev_ab.txt); bit-identical either way (per-segment partials)
    c->rev_on = 1;
    if (const char* e = getenv("LBFGS_REV")) c->rev_on = atoi(e) != 0;
    // stage 2 inside the producing launch by each group's last-dispatched workgroup instead of a
    // reduce kernel after it: measured +0.2..0.9 % at n = 3e7..1e9 (segments of 3712..122112),
    // neutral at 1e7 and 1.5..3.5 % slower at 2.5e6..5e6, where short-lived workgroups leave the
    // collector waiting on stragglers (profiles/r03/collect_ab/). Default for segments of at least
    // 3072 elements; LBFGS_COLLECT=0/1 overrides
    c->collect_on = G.L >= 3072 ? 1 : 0;
    if (const char* e = getenv("LBFGS_COLLECT")) c->collect_on = atoi(e) != 0;
    // a collector waits for its group's other workgroups (at most 8 waiters per launch, all others
    // wait-free: the wait ends unless the GPU is time-shared with something that holds it)
    c->collect_timeout_s = 10.0;
    if (const char* e = getenv("LBFGS_COLLECT_TIMEOUT")) c->collect_timeout_s = std::max(0.1, atof(e));
    // sharded slots are completed by the exchange on the device: those fetch with a copy
    c->direct = world == 1 ? 1 : 0;
    if (const char* e = getenv("LBFGS_DIRECT")) c->direct = world == 1 && atoi(e) != 0;
    *out = c;
#define CK(expr)                                                                             \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) {                                                              \
            snprintf(c->err, sizeof c->err, "%s: %s", #expr, hipGetErrorString(e_));        \
            return -2;                                                                       \
        }                                                                                    \
    } while (0)
    CK(hipSetDevice(device));
    // LBFGS_CU_PARTITION=1 (sharded ranks sharing one GPU: tests and one-card rehearsals): rank r's
    // solver stream runs on CUs [r, r + 1) * cus / world only, so no rank's spinning workgroups can
    // occupy the CUs a peer's producing pass needs - the forward-progress situation of ranks on
    // distinct GPUs. The folded exchanges then run ungated (take_fold), exactly the code path they
    // take across GPUs.
    c->cu_part = 0;
    if (const char* e = getenv("LBFGS_CU_PARTITION")) c->cu_part = world > 1 && !grp && atoi(e) != 0;
    int pworld = world, prank = rank;
#ifdef LBK_DEBUG_CU_WORLD  // timing experiments only (variant builds): a one-rank context confined to
    // rank LBFGS_DEBUG_CU_RANK's (default 0) CU share of a LBK_DEBUG_CU_WORLD-rank partition
    if (world == 1 && !grp) {
        c->cu_part = 1;
        pworld = LBK_DEBUG_CU_WORLD;
        prank = 0;
        if (const char* e = getenv("LBFGS_DEBUG_CU_RANK")) prank = atoi(e) % LBK_DEBUG_CU_WORLD;
    }
#endif
    if (c->cu_part) {
        int cus = 0;
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        const int per = cus / pworld;
        if (per < 1) {
            snprintf(c->err, sizeof c->err, "LBFGS_CU_PARTITION: %d CUs cannot be split over %d ranks", cus, pworld);
            return -1;
        }
        std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
        for (int i = prank * per; i < (prank + 1) * per; ++i) mask[(size_t)i >> 5] |= 1u << (i & 31);
        CK(hipExtStreamCreateWithCUMask(&c->stream, (uint32_t)mask.size(), mask.data()));
        std::vector<uint32_t> got(mask.size(), 0u);
        CK(hipExtStreamGetCUMask(c->stream, (uint32_t)got.size(), got.data()));
        c->cu_count = 0;
        for (size_t i = 0; i < got.size(); ++i) c->cu_count += __builtin_popcount(got[i] & mask[i]);
        if (c->cu_count != per) {
            snprintf(c->err, sizeof c->err, "LBFGS_CU_PARTITION: stream CU mask holds %d of rank %d's %d CUs",
                     c->cu_count, rank, per);
            return -2;
        }
    } else {
        CK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    }
    CK(hipMalloc(&c->partials, sizeof(double) * LBK_KW * LBK_SEGS));
    CK(hipMalloc(&c->cnt, sizeof(unsigned) * 16));
    CK(hipMalloc(&c->slots, sizeof(double) * LBK_NSLOTS * LBK_SLOT));
    CK(hipHostMalloc(&c->h_slots, sizeof(double) * LBK_NSLOTS * LBK_SLOT, hipHostMallocMapped | hipHostMallocCoherent));
    memset(c->h_slots, 0, sizeof(double) * LBK_NSLOTS * LBK_SLOT);
    CK(hipHostGetDevicePointer((void**)&c->dh_slots, c->h_slots, 0));
    CK(hipMalloc(&c->d_ck, 2 * sizeof(unsigned long long)));
    CK(hipHostMalloc(&c->h_ck, 2 * sizeof(unsigned long long), hipHostMallocDefault));
    CK(hipMemset(c->partials, 0, sizeof(double) * LBK_KW * LBK_SEGS));
    CK(hipMalloc(&c->wslots, sizeof(double) * LBK_NWSLOTS * LBK_WSLOT));
    CK(hipHostMalloc(&c->h_wslots, sizeof(double) * LBK_NWSLOTS * LBK_WSLOT,
                     hipHostMallocMapped | hipHostMallocCoherent));
    memset(c->h_wslots, 0, sizeof(double) * LBK_NWSLOTS * LBK_WSLOT);
    CK(hipHostGetDevicePointer((void**)&c->dh_wslots, c->h_wslots, 0));
    CK(hipMemset(c->wslots, 0, sizeof(double) * LBK_NWSLOTS * LBK_WSLOT));
    CK(hipMemset(c->cnt, 0, sizeof(unsigned) * 16));
    CK(hipMemset(c->slots, 0, sizeof(double) * LBK_NSLOTS * LBK_SLOT));
    {
        const size_t llb = sizeof(unsigned long long) * 2 * LBK_LL_COMPS * LBK_LL_SEGS * 2;
        CK(hipMalloc(&c->coop_ll, llb));
        CK(hipMemset(c->coop_ll, 0, llb));  // tag 0: no pass (sequence numbers start at 1)
    }
    {
        const size_t llb = sizeof(unsigned long long) * 2 * LBK_LL_COMPS * LBK_LL_SEGS * 2;
        CK(hipMalloc(&c->wolfe_ll, llb));
        CK(hipMemset(c->wolfe_ll, 0, llb));
    }
    CK(hipHostMalloc((void**)&c->wolfe_out_h, sizeof(lbk_search), hipHostMallocMapped | hipHostMallocCoherent));
    memset(c->wolfe_out_h, 0, sizeof(lbk_search));
    CK(hipHostGetDevicePointer((void**)&c->wolfe_out_d, c->wolfe_out_h, 0));
    {
        const size_t llb = sizeof(unsigned long long) * 2 * LBK_KMAX * LBK_SEGS;  // regular slots only
        CK(hipMalloc(&c->coll_ll, llb));
        CK(hipMemset(c->coll_ll, 0, llb));  // tag 0: no launch (tags start at 1)
    }
    CK(hipHostMalloc((void**)&c->coop_err_h, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
    *c->coop_err_h = 0;
    CK(hipHostGetDevicePointer((void**)&c->coop_err_d, c->coop_err_h, 0));
    CK(hipHostMalloc((void**)&c->h_xchg, sizeof(double) * LBK_WSLOT, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&c->dh_xchg, c->h_xchg, 0));
    CK(hipHostMalloc((void**)&c->sp_h, sizeof(unsigned long long) * 20, hipHostMallocMapped | hipHostMallocCoherent));
    memset(c->sp_h, 0, sizeof(unsigned long long) * 20);
    CK(hipHostGetDevicePointer((void**)&c->sp_dh, c->sp_h, 0));
    CK(hipMalloc(&c->sp_vd, sizeof(unsigned long long) * 4));
    CK(hipMemset(c->sp_vd, 0, sizeof(unsigned long long) * 4));
    {
        int khz = 0;
        CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
        c->wall_khz = khz > 0 ? khz : 100000.0;
    }
    {
        // the cooperative iteration's grid barrier needs every workgroup resident at once: cap its
        // segment count by what this device holds (fewer CUs, or a kernel grown past 2 per CU)
        int cus = 0, occ = 1 << 30;
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        int o = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_coop_iter<LBK_OBJ_ROSENBROCK>, LB_BLOCK, 0));
        occ = std::min(occ, o);
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_coop_iter<LBK_OBJ_QUAD_TRIDIAG>, LB_BLOCK, 0));
        occ = std::min(occ, o);
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_coop_iter<LBK_OBJ_QUAD_SEPARABLE>, LB_BLOCK, 0));
        occ = std::min(occ, o);
        if (c->cu_part) cus = c->cu_count;  // the stream sees only its own CUs
        c->coop_max = (int)std::min<int64_t>(c->coop_max, (int64_t)occ * cus);
        // the device-resident line searches have grid barriers of their own: their own occupancy caps
        // them (a register footprint above k_coop_iter's would otherwise over-commit the
        // grid)
        int wocc = 1 << 30;
#define SEARCH_OCC(O)                                                                                   \
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (k_coop_search<O, 0>), LB_BLOCK, 0));           \
    wocc = std::min(wocc, o);                                                                           \
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (k_coop_search<O, 1>), LB_BLOCK, 0));           \
    wocc = std::min(wocc, o);                                                                           \
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (k_coop_search<O, 2>), LB_BLOCK, 0));           \
    wocc = std::min(wocc, o);                                                                           \
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (k_coop_search<O, 3>), LB_BLOCK, 0));           \
    wocc = std::min(wocc, o);
        SEARCH_OCC(LBK_OBJ_ROSENBROCK)
        SEARCH_OCC(LBK_OBJ_QUAD_TRIDIAG)
        SEARCH_OCC(LBK_OBJ_QUAD_SEPARABLE)
#undef SEARCH_OCC
        c->wolfe_max = (int)std::min<int64_t>(c->coop_max, (int64_t)wocc * cus);
        // the persistent forms: every workgroup of their grid resident, at most `cap` per CU (the
        // occupancy answer is VGPR-bound here, where the API and the hardware agree;
        // MI355X_MICROARCH.md's one-short case is SGPR-bound, 82-98 SGPRs at 7-8 per CU). A grid that
        // does not fit still ends: every flagged wait times out (2 s).
        int cap = 4;  // workgroups per CU (A/B: LBFGS_PERSIST_WG)
        if (const char* e = getenv("LBFGS_PERSIST_WG")) cap = std::max(1, atoi(e));
        // LDS per CU from the device (160 KiB on gfx950): the reservation below and the occupancy
        // queries use the same figure
        int lds_cu = 0;
        CK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device));
        // (an A/B without the reservation changed nothing: -DLBK_PERSIST_LDS=0 in variant builds)
#ifdef LBK_PERSIST_LDS
        const int lds_on = LBK_PERSIST_LDS;
#else
        const int lds_on = 1;
#endif
        c->persist_lds = lds_on && lds_cu > 0 ? lds_cu / (cap + 1) + 1024 : 0;
        c->persist_gmax = 0;
#if LBK_PERSIST_ITER
        // the whole iteration (LBFGS_PERSIST=1, variant builds only; 165 VGPRs: 3 per CU)
        int po = 1 << 30;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (k_persist_iter<LBK_OBJ_ROSENBROCK, true>), LB_BLOCK, c->persist_lds));
        po = std::min(po, o);
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (k_persist_iter<LBK_OBJ_QUAD_TRIDIAG, true>), LB_BLOCK, c->persist_lds));
        po = std::min(po, o);
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (k_persist_iter<LBK_OBJ_QUAD_SEPARABLE, true>), LB_BLOCK, c->persist_lds));
        po = std::min(po, o);
        c->persist_gmax = std::min(po, cap) * cus;
#else
        int po = 0;
#endif
        // the persistent two-loop (LBFGS_PERSIST=2) without the commit's registers; its LDS
        // reservation lets exactly `cap` workgroups onto a CU, so the dispatcher spreads the resident
        // grid evenly (without it two workgroups can share a CU while another idles; A/B
        // LBFGS_PERSIST_LDS=0). A kernel the reservation cannot be granted to turns the mode off.
        bool lds_ok = true;
        if (c->persist_lds) {
            lds_ok &= hipFuncSetAttribute((const void*)k_persist_twoloop<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          c->persist_lds) == hipSuccess;
            lds_ok &= hipFuncSetAttribute((const void*)k_persist_twoloop<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          c->persist_lds) == hipSuccess;
#if LBK_PERSIST_ITER
#define PSET(O)                                                                                                            \
    lds_ok &= hipFuncSetAttribute((const void*)k_persist_iter<O, true>, hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                  c->persist_lds) == hipSuccess;                                                           \
    lds_ok &= hipFuncSetAttribute((const void*)k_persist_iter<O, false>, hipFuncAttributeMaxDynamicSharedMemorySize,        \
                                  c->persist_lds) == hipSuccess
            PSET(LBK_OBJ_ROSENBROCK);
            PSET(LBK_OBJ_QUAD_TRIDIAG);
            PSET(LBK_OBJ_QUAD_SEPARABLE);
#undef PSET
#endif
            (void)hipGetLastError();
        }
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_persist_twoloop<true>, LB_BLOCK, c->persist_lds));
        po = o;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_persist_twoloop<false>, LB_BLOCK, c->persist_lds));
        po = std::min(po, o);
        c->persist2_gmax = lds_ok ? std::min(po, cap) * cus : 0;
        if (!lds_ok) c->persist_gmax = 0;
    }
    c->persist_on = 0;
    if (const char* e = getenv("LBFGS_PERSIST")) c->persist_on = atoi(e);  // 1: whole iteration, 2: two-loop
    // strided segment ownership and walks without the alternation measured slower:
    // variant builds only (-DLBK_PERSIST_STRIDE=1, -DLBK_PERSIST_ALT=0)
#ifdef LBK_PERSIST_STRIDE
    c->persist_stride = LBK_PERSIST_STRIDE;
#else
    c->persist_stride = 0;
#endif
#ifdef LBK_PERSIST_ALT
    c->persist_alt = LBK_PERSIST_ALT;
#else
    c->persist_alt = 1;
#endif
    CK(hipMalloc(&c->fold_wait, sizeof(unsigned long long)));
    CK(hipMemset(c->fold_wait, 0, sizeof(unsigned long long)));
    CK(hipMalloc(&c->persist_cnt, sizeof(unsigned long long) * LBK_GROUPS));
    CK(hipMemset(c->persist_cnt, 0, sizeof(unsigned long long) * LBK_GROUPS));
    CK(hipMalloc(&c->persist_gflag, sizeof(unsigned long long) * 2 * 8 * 8 * 2));
    CK(hipMemset(c->persist_gflag, 0, sizeof(unsigned long long) * 2 * 8 * 8 * 2));
    CK(hipDeviceSynchronize());
#undef CK
    if (world > 1 && !grp) {
        // the peer mailbox is an optional accelerator when an RCCL id is given: without it the
        // context still runs on RCCL all-gathers
        const int xrc = lbk_xgmi_create(&c->xg, device, rank, world, LBK_WSLOT, c->err, sizeof c->err);
        if (xrc != 0) {
            if (!nccl_id) return xrc;
            fprintf(stderr, "lbfgs: %s; exchanges stay on RCCL\n", c->err);
            c->xg = nullptr;
            c->err[0] = 0;
        }
        if (hipMalloc(&c->d_ckslot, sizeof(uint64_t) * LBK_GROUPS * 2) != hipSuccess) return -2;
    }
    // one rank with an RCCL id: a 1-rank communicator, and every reduction goes through the
    // sharded path's in-place all-gather (diagnostic: the RCCL leg executed on a one-GPU box,
    // bit-identical to the unsharded run; the one-rank shortcuts - cooperative / single-workgroup
    // iteration, deferred stage 2, host-mirrored stage 2 - are off so the slot order is the
    // sharded one)
    if (world == 1 && !grp && nccl_id) {
        c->direct = 0;
        c->coop_max = 0;
        c->wolfe_max = 0;
    }
    if (!grp && nccl_id) return rccl_init(c, nccl_id);
    return 0;
}

// The RCCL communicator of a sharded context, created on a helper thread and waited for with a
// bound (LBFGS_RCCL_TIMEOUT, 60 s): a rank that never joins, or a bootstrap that stalls, costs this
// call one timeout, not a hang. (A non-blocking ncclCommInitRankConfig alone is not enough: on this
// RCCL the call itself blocked in its bootstrap when a peer never joined, profiles/r05/rccl_leg/.)
// On a timeout the thread is abandoned, still waiting inside RCCL, and ends with the process.
namespace {
// One state word decides who owns the finished communicator and the job: the helper thread moves
// RUNNING -> DONE when the init returns (the caller then takes both), the caller moves RUNNING ->
// ABANDONED when its wait runs out (the thread then aborts the communicator and frees the job).
// Exactly one of the two compare-exchanges succeeds.
enum { RCCL_JOB_RUNNING = 0, RCCL_JOB_DONE = 1, RCCL_JOB_ABANDONED = 2 };
struct RcclInitJob {
    ncclUniqueId id;
    int device, world, rank;
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclInProgress;
    std::atomic<int> state{RCCL_JOB_RUNNING};
};
}  // namespace

static int rccl_init(lbk_ctx* c, const void* nccl_id) {
    RcclInitJob* job = new (std::nothrow) RcclInitJob();
    if (!job) return -4;
    memcpy(&job->id, nccl_id, sizeof job->id);
    job->device = c->device;
    job->world = c->geo.world;
    job->rank = c->geo.rank;
    try {
        std::thread([job] {
            (void)hipSetDevice(job->device);
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 1;
            ncclComm_t comm = nullptr;
            const ncclResult_t r = ncclCommInitRankConfig(&comm, job->world, job->id, job->rank, &cfg);
            job->comm = comm;
            job->r = r;
            int expect = RCCL_JOB_RUNNING;
            if (!job->state.compare_exchange_strong(expect, RCCL_JOB_DONE, std::memory_order_acq_rel)) {
                // the caller gave up (ABANDONED): this thread owns the communicator and the job
                if (comm) (void)ncclCommAbort(comm);
                delete job;
            }
        }).detach();
    } catch (...) {
        delete job;
        snprintf(c->err, sizeof c->err, "RCCL init: cannot start its thread");
        return -3;
    }
    const double t_end = mono_s() + c->rccl_timeout_s;
    while (job->state.load(std::memory_order_acquire) == RCCL_JOB_RUNNING && mono_s() < t_end) usleep(200);
    int expect = RCCL_JOB_RUNNING;
    if (job->state.compare_exchange_strong(expect, RCCL_JOB_ABANDONED, std::memory_order_acq_rel)) {
        snprintf(c->err, sizeof c->err, "ncclCommInitRankConfig: no progress in %.0f s (RCCL communicator abandoned)",
                 c->rccl_timeout_s);
        fprintf(stderr, "lbfgs rank %d: %s\n", c->geo.rank, c->err);
        c->rccl_hung = 1;
        return -3;  // the thread owns the job now; a late communicator is aborted there
    }
    const ncclResult_t r = job->r;  // DONE: the thread has let go of the job
    ncclComm_t comm = job->comm;
    delete job;
    if (r != ncclSuccess) {
        snprintf(c->err, sizeof c->err, "ncclCommInitRankConfig: %s", ncclGetErrorString(r));
        if (comm) (void)ncclCommAbort(comm);
        return -3;
    }
    c->comm = comm;
    return 0;
}

// A context created without an RCCL id (the mailboxes alone) takes a communicator afterwards
// (bench.py: after the headline measurement, for the RCCL comparison leg)
int lbk_rccl_attach(lbk_ctx* c, const void* nccl_id) {
    if (!c || !nccl_id || c->grp || c->geo.world < 2) return -1;
    if (c->comm) return 0;
    if (c->rccl_hung) {
        snprintf(c->err, sizeof c->err, "an earlier RCCL communicator of this context was aborted");
        return -3;
    }
    HIPCHK(c, hipSetDevice(c->device));
    int rc = rccl_init(c, nccl_id);
    if (rc) return rc;
    // one all-gather through it, waited for with the same bound, before anything relies on it
    double* buf = nullptr;
    HIPCHK(c, hipMalloc(&buf, sizeof(double) * LBK_WSLOT));
    if (hipMemsetAsync(buf, 0, sizeof(double) * LBK_WSLOT, c->stream) != hipSuccess) rc = -2;
    const int saved = c->xg_on;
    c->xg_on = 0;
    if (rc == 0) rc = exchange_buf(c, buf, LBK_KMAX);
    c->xg_on = saved;
    if (rc == 0) rc = rccl_stream_wait(c, "RCCL self-test all-gather");
    if (!c->rccl_hung) (void)hipFree(buf);  // else a collective may still address it
    return rc;
}

void lbk_destroy(lbk_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream && !c->rccl_hung) (void)hipStreamSynchronize(c->stream);
    if (!c->rccl_hung) prof_flush(c);
    for (auto e : c->ev_free) (void)hipEventDestroy(e);
    for (auto e : c->xfer_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->dq_A) (void)hipFree(c->dq_A);
    if (c->dq_b) (void)hipFree(c->dq_b);
    if (c->dq_t) (void)hipFree(c->dq_t - LBK_FRONT);
    lbk_xgmi_destroy(c->xg);
    if (c->d_ckslot) (void)hipFree(c->d_ckslot);
    (void)hipFree(c->partials);
    (void)hipFree(c->coop_ll);
    (void)hipFree(c->wolfe_ll);
    if (c->wolfe_out_h) (void)hipHostFree(c->wolfe_out_h);
    (void)hipFree(c->coll_ll);
    xfer_pool_free(c);
    (void)hipFree(c->persist_cnt);
    (void)hipFree(c->fold_wait);
    (void)hipFree(c->persist_gflag);
    if (c->coop_err_h) (void)hipHostFree(c->coop_err_h);
    if (c->stall_release_h && !c->rccl_hung) (void)hipHostFree(c->stall_release_h);  // else a stall may still read it
    if (c->sp_h) (void)hipHostFree(c->sp_h);
    if (c->h_xchg) (void)hipHostFree(c->h_xchg);
    if (c->sp_vd) (void)hipFree(c->sp_vd);
    if (c->mark_ev) (void)hipEventDestroy(c->mark_ev);
    (void)hipFree(c->cnt);
    (void)hipFree(c->slots);
    (void)hipHostFree(c->h_slots);
    (void)hipFree(c->wslots);
    (void)hipHostFree(c->h_wslots);
    (void)hipFree(c->d_ck);
    (void)hipHostFree(c->h_ck);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const lbk_geo* lbk_geometry(const lbk_ctx* c) { return &c->geo; }
const char* lbk_last_error(const lbk_ctx* c) { return c ? c->err : "no context"; }

// Vector allocation (LBFGS_VEC_ALLOC, read at context creation):
//   pool (default)  vectors of 64 MiB .. 2 GiB are physically contiguous allocations
//                   (hipDeviceMallocContiguous) that are never returned to the driver: a freed one
//                   goes to a process-wide pool and the next vector of the same size and device takes
//                   it (at most LBFGS_VEC_POOL_GB = 32 GiB held per process, then plain); other
//                   sizes are plain hipMalloc
//   plain           every vector a plain hipMalloc
//   contiguous      every vector contiguous, freed with hipFree (A/B only: not safe, below)
// Contiguous vectors stream faster at n = 1e8 (profiles/r06/alloc_ab/, alternating contexts in one
// process: 88.5-89.0 it/s against 85.4-87.1, k_axpy_dot 534-540 us against 546-551, the commit
// 1060-1082 against 1150-1184): a plain allocation's rate depends on the physical pages it gets.
// But on this ROCm stack freeing a contiguous allocation corrupts the process's next allocations:
// tools/repeat_stress.py (profiles/r06/alloc_reuse/) found wrong results in the first solve of
// contexts created after contiguous vectors had been freed - 131 of 200 when only the destroyed
// contexts' vectors were contiguous, 50 of 200 the other way round (the freed ones contiguous, the
// failing new ones plain), 0 of 400 with plain allocations throughout. The pool never frees one:
// 0 of 900 with every vector pooled (LBFGS_VEC_POOL_MIN_MB=0), and 88.0 / 88.3 it/s against plain
// 86.8 / 86.8 alternating at n = 1e8 (profiles/r06/pool/).
namespace {
struct VecPool {
    std::mutex mu;
    std::vector<std::pair<std::pair<int, size_t>, void*>> idle;  // ((device, bytes), base)
    std::unordered_set<void*> mine;                                // every base the pool owns
    size_t held = 0;                                              // bytes owned (idle + in use)
};
VecPool& vec_pool() {
    static VecPool* p = new VecPool();  // never destroyed: its memory is never given back
    return *p;
}
constexpr size_t kPoolMax = size_t(2) << 30;
}  // namespace

double* lbk_vec_alloc(lbk_ctx* c) {
    const size_t bytes = sizeof(double) * (size_t)c->vec_doubles;
    double* p = nullptr;
    if (c->vec_mode == LBK_VEC_POOL && bytes >= c->vec_pool_min && bytes <= kPoolMax) {
        VecPool& P = vec_pool();
        std::lock_guard<std::mutex> lk(P.mu);
        for (size_t i = 0; i < P.idle.size(); ++i)
            if (P.idle[i].first == std::make_pair(c->device, bytes)) {
                p = static_cast<double*>(P.idle[i].second);
                P.idle[i] = P.idle.back();
                P.idle.pop_back();
                c->vec_pooled++;
                break;
            }
        if (!p && P.held + bytes <= c->vec_pool_cap) {
            if (hipExtMallocWithFlags((void**)&p, bytes, hipDeviceMallocContiguous) == hipSuccess) {
                P.mine.insert(p);
                P.held += bytes;
                c->vec_pooled++;
            } else {
                (void)hipGetLastError();
                p = nullptr;
                c->vec_plain_fallbacks++;
            }
        }
    } else if (c->vec_mode == LBK_VEC_CONTIGUOUS) {
        if (hipExtMallocWithFlags((void**)&p, bytes, hipDeviceMallocContiguous) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            c->vec_plain_fallbacks++;
        }
    }
    if (!p && hipMalloc(&p, bytes) != hipSuccess) {
        snprintf(c->err, sizeof c->err, "hipMalloc of %lld doubles failed", (long long)c->vec_doubles);
        return nullptr;
    }
    if (hipMemsetAsync(p, 0, bytes, c->stream) != hipSuccess) {
        lbk_vec_free(c, p + LBK_FRONT);
        return nullptr;
    }
    return p + LBK_FRONT;
}

void lbk_vec_free(lbk_ctx* c, double* v) {
    if (!v) return;
    void* base = v - LBK_FRONT;
    VecPool& P = vec_pool();
    {
        std::lock_guard<std::mutex> lk(P.mu);
        if (!P.mine.count(base)) {
            (void)hipFree(base);  // (synchronises the device: no kernel of this context still uses it)
            return;
        }
    }
    // a pooled vector: the context's queued work on it finishes before another context can take it
    // (a stream that may hold a hung RCCL collective keeps it: it stays owned and idle forever)
    if (c->rccl_hung || hipStreamSynchronize(c->stream) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(P.mu);
    P.idle.push_back({{c->device, sizeof(double) * (size_t)c->vec_doubles}, base});
}

int lbk_vec_pool_stats(const lbk_ctx* c, int* pooled, double* held_gb) {
    VecPool& P = vec_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    if (pooled) *pooled = c ? c->vec_pooled : 0;
    if (held_gb) *held_gb = (double)P.held / double(size_t(1) << 30);
    return c ? c->vec_mode : -1;
}

void* lbk_host_alloc(size_t bytes) {
    void* p = nullptr;
    return hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}

void lbk_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

// ---- whole-vector copies between the caller's (pageable) memory and HBM: x0 in, x out ----------
// (configs[3]'s time to solution pays both; parallel-implementation/L-BFGS.cu:176, 360-365 too).
// LBFGS_XFER selects how a copy of >= 16 MB travels:
//   pageable  one hipMemcpyAsync from / to the caller's buffer (the runtime stages it)
//   register  the caller's pages pinned for the copy (hipHostRegister), one DMA, unpinned
//   staged    LBFGS_XFER_THREADS host threads, each with its own stream and two pinned 8 MB
//             buffers, copy their slice through them while the DMA engines move the previous chunk
// (tools/xferprobe.hip measures the three on the box; the default is the measured best).
namespace {
constexpr size_t kXferMin = 16u << 20, kXferChunk = 8u << 20;

struct XferPool {
    int threads = 0;
    std::vector<hipStream_t> st;
    std::vector<char*> buf;        // 2 per thread
    std::vector<hipEvent_t> ev;    // 2 per thread
};
XferPool* xfer_pool(lbk_ctx* c) {
    if (c->xfer_pool) return static_cast<XferPool*>(c->xfer_pool);
    XferPool* P = new (std::nothrow) XferPool();
    if (!P) return nullptr;
    int T = 8;
    if (const char* e = getenv("LBFGS_XFER_THREADS")) T = std::max(1, std::min(32, atoi(e)));
    P->threads = T;
    P->st.resize(T);
    P->buf.resize(2 * T);
    P->ev.resize(2 * T);
    bool ok = true;
    for (int t = 0; t < T && ok; ++t) {
        ok = hipStreamCreateWithFlags(&P->st[t], hipStreamNonBlocking) == hipSuccess;
        for (int b = 0; b < 2 && ok; ++b) {
            ok = hipHostMalloc((void**)&P->buf[2 * t + b], kXferChunk, hipHostMallocDefault) == hipSuccess &&
                 hipEventCreateWithFlags(&P->ev[2 * t + b], hipEventDisableTiming) == hipSuccess;
        }
    }
    c->xfer_pool = P;  // freed by xfer_pool_free (also a partial one)
    return ok ? P : nullptr;
}

// one worker: its slice [off, off + len) of the copy, through its two pinned buffers
int xfer_slice(lbk_ctx* c, XferPool* P, int t, char* dst, const char* src, size_t len, bool h2d) {
    if (hipSetDevice(c->device) != hipSuccess) return -2;
    hipStream_t s = P->st[t];
    const size_t nch = (len + kXferChunk - 1) / kXferChunk;
    if (h2d) {
        for (size_t i = 0; i < nch; ++i) {
            const int b = (int)(i & 1);
            const size_t o = i * kXferChunk, l = std::min(kXferChunk, len - o);
            if (i >= 2 && hipEventSynchronize(P->ev[2 * t + b]) != hipSuccess) return -2;  // the DMA that read it
            memcpy(P->buf[2 * t + b], src + o, l);
            if (hipMemcpyAsync(dst + o, P->buf[2 * t + b], l, hipMemcpyHostToDevice, s) != hipSuccess ||
                hipEventRecord(P->ev[2 * t + b], s) != hipSuccess)
                return -2;
        }
    } else {
        auto issue = [&](size_t i) {
            const int b = (int)(i & 1);
            const size_t o = i * kXferChunk, l = std::min(kXferChunk, len - o);
            return hipMemcpyAsync(P->buf[2 * t + b], src + o, l, hipMemcpyDeviceToHost, s) == hipSuccess &&
                   hipEventRecord(P->ev[2 * t + b], s) == hipSuccess;
        };
        if (nch > 0 && !issue(0)) return -2;
        for (size_t i = 0; i < nch; ++i) {
            const int b = (int)(i & 1);
            if (hipEventSynchronize(P->ev[2 * t + b]) != hipSuccess) return -2;
            if (i + 1 < nch && !issue(i + 1)) return -2;  // the other buffer, freed one step ago
            const size_t o = i * kXferChunk, l = std::min(kXferChunk, len - o);
            memcpy(dst + o, P->buf[2 * t + b], l);
        }
    }
    return hipStreamSynchronize(s) == hipSuccess ? 0 : -2;
}

int xfer_mode() {  // read per copy (two getenv calls per solve): tests and tools switch it in-process
    int mode = 0;
    if (const char* e = getenv("LBFGS_XFER")) {
        if (!strcmp(e, "register")) mode = 1;
        else if (!strcmp(e, "staged")) mode = 2;
    }
    return mode;
}

// dst / src: one device, one host pointer; bytes; h2d direction
int xfer(lbk_ctx* c, void* dst, const void* src, size_t bytes, bool h2d) {
    const int mode = bytes >= kXferMin ? xfer_mode() : 0;
    if (mode == 1) {  // pin the caller's pages for this copy
        void* host = h2d ? const_cast<void*>(src) : dst;
        const uintptr_t a = (uintptr_t)host & ~(uintptr_t)4095;
        const size_t len = (((uintptr_t)host + bytes + 4095) & ~(uintptr_t)4095) - a;
        if (hipHostRegister((void*)a, len, hipHostRegisterDefault) == hipSuccess) {
            hipError_t e = hipMemcpyAsync(dst, src, bytes, h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, c->stream);
            const int wrc = e == hipSuccess ? stream_wait(c, "vector transfer") : 0;
            (void)hipHostUnregister((void*)a);
            HIPCHK(c, e);
            return wrc;
        }
        (void)hipGetLastError();  // not registrable (already pinned, ...): the pageable copy
    } else if (mode == 2) {
        XferPool* P = xfer_pool(c);
        if (P) {
            const int wrc = stream_wait(c, "vector transfer");  // the solver stream's work on the vector is done
            if (wrc) return wrc;
            const int T = P->threads;
            const size_t per = ((bytes / T) + 4095) & ~(size_t)4095;
            std::vector<std::thread> th;
            std::vector<int> rc(T, 0);
            for (int t = 0; t < T; ++t) {
                const size_t o = std::min(bytes, per * t), l = std::min(bytes, per * (t + 1)) - o;
                if (!l) continue;
                th.emplace_back([=, &rc] {
                    rc[t] = xfer_slice(c, P, t, (char*)dst + o, (const char*)src + o, l, h2d);
                });
            }
            for (auto& x : th) x.join();
            for (int t = 0; t < T; ++t)
                if (rc[t]) {
                    snprintf(c->err, sizeof c->err, "staged transfer failed (worker %d)", t);
                    return -2;
                }
            return 0;
        }
    }
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, c->stream));
    return stream_wait(c, "vector transfer");
}
}  // namespace

void xfer_pool_free(lbk_ctx* c) {
    XferPool* P = static_cast<XferPool*>(c->xfer_pool);
    if (!P) return;
    for (auto s : P->st)
        if (s) (void)hipStreamDestroy(s);
    for (auto b : P->buf)
        if (b) (void)hipHostFree(b);
    for (auto e : P->ev)
        if (e) (void)hipEventDestroy(e);
    delete P;
    c->xfer_pool = nullptr;
}

int lbk_upload(lbk_ctx* c, double* dst, const double* host_global) {
    // local range plus the ghosts that exist globally
    const int64_t lo = c->geo.elem_lo > 0 ? c->geo.elem_lo - 1 : 0;
    const int64_t hi = std::min<int64_t>(c->geo.elem_lo + c->geo.n_loc + 1, c->geo.n);
    if (hi <= lo) return 0;
    return xfer(c, dst + (lo - c->geo.elem_lo), host_global + lo, sizeof(double) * (hi - lo), true);
}

int lbk_upload_local(lbk_ctx* c, double* dst, const double* host_local) {
    if (c->geo.n_loc == 0) return 0;
    HIPCHK(c, hipMemcpyAsync(dst, host_local, sizeof(double) * c->geo.n_loc, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

// asynchronous transfers of the local range on the solver stream; event `tag` (0..3) marks the
// copy's completion for lbk_xfer_wait (host-callback objectives: double-buffered pinned buffers)
int lbk_download_local_async(lbk_ctx* c, double* host_local, const double* src, int tag) {
    if (tag < 0 || tag >= 4) return -1;
    if (!c->xfer_ev[tag]) HIPCHK(c, hipEventCreateWithFlags(&c->xfer_ev[tag], hipEventDisableTiming));
    if (c->geo.n_loc > 0)
        HIPCHK(c, hipMemcpyAsync(host_local, src, sizeof(double) * c->geo.n_loc, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(c->xfer_ev[tag], c->stream));
    return 0;
}

int lbk_upload_local_async(lbk_ctx* c, double* dst, const double* host_local, int tag) {
    if (tag < 0 || tag >= 4) return -1;
    if (!c->xfer_ev[tag]) HIPCHK(c, hipEventCreateWithFlags(&c->xfer_ev[tag], hipEventDisableTiming));
    if (c->geo.n_loc > 0)
        HIPCHK(c, hipMemcpyAsync(dst, host_local, sizeof(double) * c->geo.n_loc, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipEventRecord(c->xfer_ev[tag], c->stream));
    return 0;
}

int lbk_xfer_wait(lbk_ctx* c, int tag) {
    if (tag < 0 || tag >= 4) return -1;
    if (c->xfer_ev[tag]) HIPCHK(c, hipEventSynchronize(c->xfer_ev[tag]));
    return 0;
}

int lbk_download(lbk_ctx* c, double* host_global, const double* src) {
    return lbk_download_local(c, host_global + c->geo.elem_lo, src);
}

int lbk_download_local(lbk_ctx* c, double* host_local, const double* src) {
    if (c->geo.n_loc == 0) return 0;
    return xfer(c, host_local, src, sizeof(double) * c->geo.n_loc, false);
}

int lbk_copy(lbk_ctx* c, double* dst, const double* src) {
    HIPCHK(c, hipMemcpyAsync(dst - 1, src - 1, sizeof(double) * (c->geo.n_loc + 2), hipMemcpyDeviceToDevice,
                             c->stream));
    return 0;
}


int lbk_dot(lbk_ctx* c, const double* a, const double* b, int slot) {
    Geo g = kgeo(c);
    Red r = kred_deferrable(c, slot);
    fold_producer(c, r, false);
    return launch(c, LBK_K_DOT, 2, slot, [&] {
        if (r.fp.peers)
            NT_DISPATCH(c, hipLaunchKernelGGL((k_dot<NT_, true>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, a, b, g, r));
        else
            NT_DISPATCH(c, hipLaunchKernelGGL(k_dot<NT_>, dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, a, b, g, r));
    });
}

int lbk_axpy_dot(lbk_ctx* c, double* qout, const double* qin, const double* y, const double* s, double rho,
                 int ref_alpha, int slot) {
    Geo g = kgeo(c);
    g.ppart = take_pending(c, ref_alpha);
    const FoldSrc fs = take_fold(c, ref_alpha);
    Red r = kred_deferrable(c, slot);
    fold_producer(c, r, false);
    const double* pa = sref(c, ref_alpha);
    return launch(c, LBK_K_AXPY_DOT, 4, slot, [&] {
        if (r.fp.peers || fs.mbx)
            NT_DISPATCH(c, hipLaunchKernelGGL((k_axpy_dot<NT_, true>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, qout, qin, y, s, rho, pa, g, r, fs));
        else
            NT_DISPATCH(c, hipLaunchKernelGGL(k_axpy_dot<NT_>, dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, qout, qin, y, s, rho, pa, g, r, fs));
    });
}

int lbk_mid(lbk_ctx* c, double* rout, const double* qin, const double* y0, double rho0, double gamma,
            int ref_alpha, int slot) {
    Geo g = kgeo(c);
    g.ppart = take_pending(c, ref_alpha);
    const FoldSrc fs = take_fold(c, ref_alpha);
    Red r = kred_deferrable(c, slot);
    fold_producer(c, r, true);
    const double* pa = sref(c, ref_alpha);
    if (c->geo.world > 1) g.edge_slot = r.slot;
    return launch(c, LBK_K_MID, 3, slot, [&] {
        if (r.fp.peers || fs.mbx)
            NT_DISPATCH(c, hipLaunchKernelGGL((k_mid<NT_, true>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, rout, qin, y0, rho0, gamma, pa, g, r, fs));
        else
            NT_DISPATCH(c, hipLaunchKernelGGL(k_mid<NT_>, dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, rout, qin, y0, rho0, gamma, pa, g, r, fs));
    });
}

int lbk_axpy2_dot(lbk_ctx* c, double* rr, const double* rin, const double* s, const double* ynext, double rho,
                  int ref_beta, int ref_alpha, int slot) {
    Geo g = kgeo(c);
    g.ppart = take_pending(c, ref_beta);
    const FoldSrc fs = take_fold(c, ref_beta);
    Red r = kred_deferrable(c, slot);
    fold_producer(c, r, true);
    const double* pb = sref(c, ref_beta);
    const double* pa = sref(c, ref_alpha);
    if (c->geo.world > 1) g.edge_slot = r.slot;
    return launch(c, LBK_K_AXPY2_DOT, 4, slot, [&] {
        if (r.fp.peers || fs.mbx)
            NT_DISPATCH(c, hipLaunchKernelGGL((k_axpy2_dot<NT_, true>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, rr, rin, s, ynext, rho, pb, pa, g, r, fs));
        else
            NT_DISPATCH(c, hipLaunchKernelGGL(k_axpy2_dot<NT_>, dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, rr, rin, s, ynext, rho, pb, pa, g, r, fs));
    });
}

int lbk_last(lbk_ctx* c, double* dout, const double* rr, const double* s, const double* gg, double rho,
             int ref_beta, int ref_alpha, int slot) {
    Geo g = kgeo(c);
    g.ppart = take_pending(c, ref_beta);
    Red r = kred(c, slot);
    const double* pb = sref(c, ref_beta);
    const double* pa = sref(c, ref_alpha);
    if (c->geo.world > 1) g.edge_slot = r.slot;
    return launch(c, LBK_K_LAST, 4, slot, [&] {
        NT_DISPATCH(c, hipLaunchKernelGGL(k_last<NT_>, dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, dout, rr, s, gg, rho, pb, pa, g, r));
    });
}

int lbk_negdot(lbk_ctx* c, double* dout, const double* gg, int slot) {
    Geo g = kgeo(c);
    Red r = kred(c, slot);
    if (c->geo.world > 1) g.edge_slot = r.slot;
    return launch(c, LBK_K_NEGDOT, 2, slot, [&] {
        NT_DISPATCH(c, hipLaunchKernelGGL(k_negdot<NT_>, dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, dout, gg, g, r));
    });
}


int lbk_eval(lbk_ctx* c, int obj, const double* x, double* gout, int slot) {
    Geo g = kgeo(c);
    Red r = kred(c, slot, 2);
    DirArgs da = {nullptr, nullptr, nullptr, 0.0, nullptr, nullptr, 0.0, nullptr, c->geo.g_lo, c->geo.g_hi};
    return launch(c, LBK_K_EVAL, gout ? 2 : 1, slot, [&] {
        OBJ_DISPATCH(obj, hipLaunchKernelGGL((k_objective<O_, true, true, NT_>), dim3(nblocks(c)), dim3(LB_BLOCK), 0,
                                             c->stream, x, da, 0.0, gout, g, r));
        return 0;
    }, 2);
}

int lbk_trial(lbk_ctx* c, int obj, const double* x, const double* d, double alpha, double* gout, int slot) {
    Geo g = kgeo(c);
    Red r = kred(c, slot, 2);
    DirArgs da = {d, nullptr, nullptr, 0.0, nullptr, nullptr, 0.0, ghost_ptr(c), c->geo.g_lo, c->geo.g_hi};
    const int kind = gout ? LBK_K_TRIAL_FG : LBK_K_TRIAL_F;
    return launch(c, kind, gout ? 3 : 2, slot, [&] {
        if (gout) {
            OBJ_DISPATCH(obj, hipLaunchKernelGGL((k_objective<O_, false, true, NT_>), dim3(nblocks(c)), dim3(LB_BLOCK),
                                                 0, c->stream, x, da, alpha, gout, g, r));
        } else {
            OBJ_DISPATCH(obj, hipLaunchKernelGGL((k_objective<O_, false, false, NT_>), dim3(nblocks(c)), dim3(LB_BLOCK),
                                                 0, c->stream, x, da, alpha, gout, g, r));
        }
        return 0;
    }, 2);
}

int lbk_dense_set(lbk_ctx* c, const double* A, const double* b) {
    const int64_t n = c->geo.n;
    if (c->geo.world != 1 || n > LBK_DENSE_NMAX || !A || !b) {
        snprintf(c->err, sizeof c->err, "dense quadratic: one rank and n <= %d only", LBK_DENSE_NMAX);
        return -1;
    }
    if (!c->dq_A) {
        HIPCHK(c, hipMalloc(&c->dq_A, sizeof(double) * (size_t)(n * n)));
        HIPCHK(c, hipMalloc(&c->dq_b, sizeof(double) * (size_t)n));
        double* t = lbk_vec_alloc(c);
        if (!t) return -2;
        c->dq_t = t;
    }
    HIPCHK(c, hipMemcpyAsync(c->dq_A, A, sizeof(double) * (size_t)(n * n), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->dq_b, b, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

int lbk_dense_eval(lbk_ctx* c, const double* x, double* gout, int slot) {
    if (!c->dq_A) {
        snprintf(c->err, sizeof c->err, "dense quadratic: no matrix (lbfgs_set_dense_quadratic)");
        return -1;
    }
    const int64_t n = c->geo.n;
    const int nb = (int)((n + 3) / 4);
    // the row pass reads A once (n^2 doubles) and x; its bytes are counted with the terms pass
    hipLaunchKernelGGL(k_dense_rows, dim3(nb), dim3(256), 0, c->stream, c->dq_A, c->dq_b, x, gout, c->dq_t, n);
    HIPCHK(c, hipGetLastError());
    Geo g = kgeo(c);
    Red r = kred(c, slot, 2);
    return launch(c, LBK_K_EVAL, (double)n + 3.0 + (gout ? 2.0 : 0.0), slot, [&] {
        NT_DISPATCH(c, hipLaunchKernelGGL(k_terms_dot<NT_>, dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, c->dq_t,
                                          gout, g, r));
    }, 2);
}

int lbk_point(lbk_ctx* c, double* z, const double* x, const double* d, double alpha) {
    const int64_t lo = -1, hi = c->geo.n_loc + 1;
    const int64_t cnt = hi - lo;
    const int nb = (int)((cnt + 255) / 256);
    return launch(c, LBK_K_POINT, 3, -1, [&] {
        hipLaunchKernelGGL(k_point, dim3(nb), dim3(256), 0, c->stream, z, x, d, alpha, lo, hi);
    });
}

int lbk_elementwise(lbk_ctx* c, int op, double* out, const double* a, const double* b, double alpha) {
    const int nb = (int)std::min<int64_t>((c->geo.n_loc + 255) / 256, 4096);
    return launch(c, LBK_K_POINT, op == 1 || op == 3 ? 3 : 2, -1, [&] {
        if (nb > 0) hipLaunchKernelGGL(k_elementwise, dim3(nb), dim3(256), 0, c->stream, op, out, a, b, alpha, c->geo.n_loc);
    });
}

// ---- vector-free mode -------------------------------------------------------------------
// the persistent iteration's segments per workgroup (1..16, dividing a group's 1024) for this n,
// or 0 when it is off or the grid would not be resident
// the persistent forms' grid (resident workgroups, each owning every G-th segment) when `mode` is
// on for this context, else 0
static int persist_grid(const lbk_ctx* c, int mode, int gmax) {
    if (c->persist_on != mode || c->geo.world != 1 || c->comm || !c->direct || c->geo.nseg <= c->coop_max) return 0;
    return (int)std::min<int64_t>(gmax, c->geo.nseg);
}
static int persist_fits(const lbk_ctx* c) { return persist_grid(c, 1, c->persist_gmax); }

int lbk_twoloop_ok(const lbk_ctx* c, int h) {
    return h >= 1 && h <= LBK_SMALL_HMAX && persist_grid(c, 2, c->persist2_gmax) > 0;
}

int lbk_twoloop_persist(lbk_ctx* c, int h, const double* g, double* q, double* r, const double* const* S,
                        const double* const* Y, const double* rho, double gamma, int p0_ref, int slot_p0,
                        int slot_a0, int slot_b0) {
    const int nb = lbk_twoloop_ok(c, h) ? persist_grid(c, 2, c->persist2_gmax) : 0;
    if (!nb) return -1;
    // p0_ref's slot is read directly (slot_total) by the kernel: a stage 2 still pending for it
    // (deferred, or a folded exchange) must land first
    {
        const int rc = flush_pending(c);
        if (rc) return rc;
    }
    SmallArgs a;
    memset(&a, 0, sizeof a);
    a.h = h;
    a.p0_from_slot = p0_ref >= 0;
    a.p0_slot = p0_ref >= 0 ? sref(c, p0_ref) : nullptr;
    a.g = g;
    a.q = q;
    a.r = r;
    for (int i = 0; i < h; ++i) {
        a.S[i] = S[i];
        a.Y[i] = Y[i];
        a.rho[i] = rho[i];
    }
    a.gamma = gamma;
    a.slots = c->slots;
    // written by block 0 of the launch, read on the device by the next passes / the commit
    c->slot_mirror[slot_p0] = 0;
    c->slot_s2[slot_p0] = 0;
    for (int i = 0; i < h; ++i) {
        c->slot_mirror[slot_a0 + i] = c->slot_mirror[slot_b0 + i] = 0;
        c->slot_s2[slot_a0 + i] = c->slot_s2[slot_b0 + i] = 0;
    }
    a.slot_p0 = slot_p0;
    a.slot_a0 = slot_a0;
    a.slot_b0 = slot_b0;
    a.ll = c->coop_ll;
    a.seq_base = (unsigned)c->coop_base;
    a.err = c->coop_err_d;
    a.timeout = (unsigned long long)(2.0 * c->wall_khz * 1e3);  // 2 s: a grid that is not resident ends
    a.partials = c->partials;
    a.pcnt = c->persist_cnt;
    a.gflag = c->persist_gflag;
    a.spw = c->persist_stride ? 0 : (c->geo.nseg + nb - 1) / nb;
    a.alt = c->persist_alt;
    c->coop_base += (unsigned long long)((p0_ref >= 0 ? 0 : 1) + 2 * h - 1);
    Geo geo = kgeo(c);
    geo.rev = 0;
    const double vec = (p0_ref >= 0 ? 0.0 : 2.0) + 4.0 * (h - 1) + 3.0 + 4.0 * (h - 1);
    return launch(c, LBK_K_SMALL_ITER, vec, -1, [&] {
        NT_DISPATCH(c, hipLaunchKernelGGL((k_persist_twoloop<NT_>), dim3(nb), dim3(LB_BLOCK), c->persist_lds, c->stream, a, geo));
    });
}

int lbk_small_iter(lbk_ctx* c, int obj, int h, const double* g, double* q, double* r, const double* const* S,
                   const double* const* Y, const double* rho, double gamma, int p0_ref, double a0, const double* x,
                   double* xn, double* gn, double* so, double* yo, int slot_p0, int slot_a0, int slot_b0,
                   int slot_c, double cand, const lbk_spec* spec, unsigned long long* epoch) {
    if (epoch) *epoch = 0;
    if (!lbk_small_ok(c, h) || (spec && !lbk_small_spec_ok(c, h))) return -1;
    SmallArgs a;
    memset(&a, 0, sizeof a);
    a.h = h;
    a.p0_from_slot = p0_ref >= 0;
    a.p0_slot = p0_ref >= 0 ? sref(c, p0_ref) : nullptr;
    a.g = g;
    a.q = q;
    a.r = r;
    for (int i = 0; i < h; ++i) {
        a.S[i] = S[i];
        a.Y[i] = Y[i];
        a.rho[i] = rho[i];
    }
    a.gamma = gamma;
    a.a0 = a0;
    a.cand = cand;
    a.x = x;
    a.xn = xn;
    a.gn = gn;
    a.so = so;
    a.yo = yo;
    a.slots = c->slots;
    a.hslots = c->direct ? c->dh_slots : nullptr;
    c->slot_mirror[slot_p0] = 0;  // single-component passes: device only (see mirrored())
    for (int i = 0; i < h; ++i) c->slot_mirror[slot_a0 + i] = c->slot_mirror[slot_b0 + i] = 0;
    c->slot_mirror[slot_c] = c->direct ? 1 : 0;
    // written here, not by a ticket launch: no ticket completion word stands for them
    c->slot_s2[slot_p0] = c->slot_s2[slot_c] = 0;
    for (int i = 0; i < h; ++i) c->slot_s2[slot_a0 + i] = c->slot_s2[slot_b0 + i] = 0;
    a.slot_p0 = slot_p0;
    a.slot_a0 = slot_a0;
    a.slot_b0 = slot_b0;
    a.slot_c = slot_c;
    Geo geo = kgeo(c);
    // algorithmic bytes: the multi-launch sequence's passes (P0 dot if computed, 4 per pair
    // pass, 3 for mid, 8 for the commit)
    const double vec = (p0_ref >= 0 ? 0.0 : 2.0) + 4.0 * (h - 1) + 3.0 + 4.0 * (h - 1) + 8.0;
    const int persist = persist_fits(c);
    if ((c->coop_max > 0 && c->geo.nseg <= c->coop_max) || persist) {
        // passes of this launch (sequence numbers it tags): [P0] + (h-1) first-loop + mid + (h-1)
        // second-loop + commit
        const int passes = (p0_ref >= 0 ? 0 : 1) + 2 * h;
        a.ll = c->coop_ll;
        a.seq_base = (unsigned)c->coop_base;
        a.err = c->coop_err_d;
        a.timeout = (unsigned long long)(2.0 * c->wall_khz * 1e3);  // 2 s
        if (c->direct) {  // a completion record the host can wait on without a stream sync
            const unsigned long long e = ++c->sp_epoch;
            const int i = (int)(e & 3);
            a.epoch = e;
            a.done = c->sp_dh;
            a.rec = c->sp_dh + 4 + 4 * i;
            c->sp_base[i] = c->coop_base;
            c->sp_bytes[i] = vec * 8.0 * (double)c->geo.n_loc;
            c->sp_spec[i] = spec != nullptr;
            if (spec) {
                a.spec = 1;
                a.spec_ls = spec->ls;
                a.prev_c = c->slots + (int64_t)spec->prev_slot * LBK_SLOT;
                a.spec_fx = spec->fx;
                a.spec_c1 = spec->c1;
                a.spec_c2 = spec->c2;
                a.spec_tol = spec->tol;
                a.vd = c->sp_vd + i;
                if (spec->chain_epoch) {
                    a.chain = c->sp_vd + (spec->chain_epoch & 3);
                    a.chain_want = (spec->chain_epoch << 1) | 1ull;
                }
            }
            if (epoch) *epoch = e;
        }
        c->coop_base += (unsigned long long)passes;
        geo.rev = 0;
#if LBK_PERSIST_ITER
        if (persist) {
            a.partials = c->partials;
            a.pcnt = c->persist_cnt;
            a.gflag = c->persist_gflag;
            const int nb = persist;
            a.spw = c->persist_stride ? 0 : (c->geo.nseg + nb - 1) / nb;
            a.alt = c->persist_alt;
            return launch(c, LBK_K_SMALL_ITER, vec, -1, [&] {
                NT_DISPATCH(c, switch (obj) {
                    case LBK_OBJ_ROSENBROCK: hipLaunchKernelGGL((k_persist_iter<LBK_OBJ_ROSENBROCK, NT_>), dim3(nb), dim3(LB_BLOCK), c->persist_lds, c->stream, a, geo); break;
                    case LBK_OBJ_QUAD_TRIDIAG: hipLaunchKernelGGL((k_persist_iter<LBK_OBJ_QUAD_TRIDIAG, NT_>), dim3(nb), dim3(LB_BLOCK), c->persist_lds, c->stream, a, geo); break;
                    default: hipLaunchKernelGGL((k_persist_iter<LBK_OBJ_QUAD_SEPARABLE, NT_>), dim3(nb), dim3(LB_BLOCK), c->persist_lds, c->stream, a, geo); break;
                });
            });
        }
#endif
        const int nb = (int)c->geo.nseg;
        return launch(c, LBK_K_SMALL_ITER, vec, -1, [&] {
            switch (obj) {
                case LBK_OBJ_ROSENBROCK: hipLaunchKernelGGL(k_coop_iter<LBK_OBJ_ROSENBROCK>, dim3(nb), dim3(LB_BLOCK), 0, c->stream, a, geo); break;
                case LBK_OBJ_QUAD_TRIDIAG: hipLaunchKernelGGL(k_coop_iter<LBK_OBJ_QUAD_TRIDIAG>, dim3(nb), dim3(LB_BLOCK), 0, c->stream, a, geo); break;
                default: hipLaunchKernelGGL(k_coop_iter<LBK_OBJ_QUAD_SEPARABLE>, dim3(nb), dim3(LB_BLOCK), 0, c->stream, a, geo); break;
            }
        });
    }
    snprintf(c->err, sizeof c->err, "lbk_small_iter: no one-launch form for this size");
    return -1;
}

int lbk_small_spec_ok(const lbk_ctx* c, int h) {
    return lbk_small_ok(c, h) && c->direct && c->coop_max > 0 && c->geo.nseg <= c->coop_max;
}

int lbk_search_dev_ok(const lbk_ctx* c, int obj) {
    return c->dev_wolfe && c->geo.world == 1 && !c->comm && c->wolfe_max > 0 && c->geo.nseg <= c->wolfe_max &&
           (obj == LBK_OBJ_ROSENBROCK || obj == LBK_OBJ_QUAD_TRIDIAG || obj == LBK_OBJ_QUAD_SEPARABLE);
}

static int small_wait(lbk_ctx* c, unsigned long long epoch, int word = 0);

int lbk_search_dev(lbk_ctx* c, int obj, int ls, const double* x, const double* d, lbk_search* st,
                   const lbk_search_commit* cm) {
    if (!lbk_search_dev_ok(c, obj) || ls < 0 || ls > 3 || (cm && cm->slot >= 0 && (cm->slot >= LBK_NSLOTS || !cm->g))) {
        snprintf(c->err, sizeof c->err, "lbk_search_dev: not a single-rank cooperative size (or bad arguments)");
        return -1;
    }
    SmallArgs a;
    memset(&a, 0, sizeof a);
    a.ll = c->wolfe_ll;
    a.seq_base = (unsigned)c->wolfe_seq;
    a.err = c->coop_err_d;
    a.timeout = (unsigned long long)(c->search_timeout_s * c->wall_khz * 1e3);  // 2 s per barrier
    a.done = c->sp_dh + 3;  // completion word: the host polls it instead of synchronising the stream
    a.epoch = ++c->search_epoch;
    c->wolfe_seq += LBK_SEARCH_PASSES + 1;                                     // trial passes + the commit
    SearchCommit k;
    memset(&k, 0, sizeof k);
    const bool commit = cm && cm->slot >= 0;
    if (commit) {
        k.g = cm->g;
        k.xn = cm->xn;
        k.gn = cm->gn;
        k.so = cm->so;
        k.yo = cm->yo;
        k.slot = c->slots + (int64_t)cm->slot * LBK_SLOT;
        k.hslot = c->direct ? c->dh_slots + (int64_t)cm->slot * LBK_SLOT : nullptr;
    }
    lbk_search s = *st;
    s.done = s.committed = s.passes_f = s.passes_fg = 0;
    Geo geo = kgeo(c);
    geo.rev = 0;
    const int nb = (int)c->geo.nseg;
    lbk_search* o = c->wolfe_out_d;
    const int rc = launch(c, LBK_K_TRIAL_FG, 0.0, -1, [&] {
#define SEARCH_LAUNCH(O)                                                                                                   \
    switch (ls) {                                                                                                          \
        case 0: hipLaunchKernelGGL((k_coop_search<O, 0>), dim3(nb), dim3(LB_BLOCK), 0, c->stream, a, geo, s, x, d, k, o); break; \
        case 1: hipLaunchKernelGGL((k_coop_search<O, 1>), dim3(nb), dim3(LB_BLOCK), 0, c->stream, a, geo, s, x, d, k, o); break; \
        case 2: hipLaunchKernelGGL((k_coop_search<O, 2>), dim3(nb), dim3(LB_BLOCK), 0, c->stream, a, geo, s, x, d, k, o); break; \
        default: hipLaunchKernelGGL((k_coop_search<O, 3>), dim3(nb), dim3(LB_BLOCK), 0, c->stream, a, geo, s, x, d, k, o); break; \
    }
        switch (obj) {
            case LBK_OBJ_ROSENBROCK: SEARCH_LAUNCH(LBK_OBJ_ROSENBROCK) break;
            case LBK_OBJ_QUAD_TRIDIAG: SEARCH_LAUNCH(LBK_OBJ_QUAD_TRIDIAG) break;
            default: SEARCH_LAUNCH(LBK_OBJ_QUAD_SEPARABLE) break;
        }
#undef SEARCH_LAUNCH
    });
    if (rc) return rc;
    const int wrc = small_wait(c, c->search_epoch, 3);  // polls the word; no runtime thread spins
    if (*(volatile unsigned*)c->coop_err_h) {
        // the grid was not resident together (or a barrier waited past its bound): each workgroup
        // leaves at its first failed barrier (or at the next one, which finds the error flag set)
        // and no trial pass or commit runs after it; a workgroup that passed every barrier may have
        // run the commit pass on its own segments, so the caller goes on with the host loop from the
        // same state and commits again even at the first trial's step (recommit_a0); the device
        // form stays off for this context
        HIPCHK(c, hipStreamSynchronize(c->stream));  // the whole grid has drained
        *(volatile unsigned*)c->coop_err_h = 0;
        c->dev_wolfe = 0;
        c->coop_fallbacks++;
        snprintf(c->err, sizeof c->err, "device line search: grid barrier timed out (search redone on the host loop)");
        return -6;
    }
    if (wrc) return wrc;
    lbk_search r;
    memcpy(&r, (const void*)c->wolfe_out_h, sizeof r);
    *st = r;
    // x and d per trial pass; the commit's x, g, d in and x', g', s, y out
    c->bytes_total += (double)(r.passes_f + r.passes_fg) * 2.0 * 8.0 * (double)c->geo.n_loc;
    if (r.committed) {
        c->bytes_total += 7.0 * 8.0 * (double)c->geo.n_loc;
        c->slot_mirror[cm->slot] = c->direct ? 1 : 0;
        c->slot_s2[cm->slot] = 0;
    }
    return 0;
}

// spin on the pinned completion word; every 64k polls ask the stream whether it still runs (a
// faulted or finished stream with the word unset ends the wait with the stream's error)
// A hipStreamQuery on a busy stream keeps one of the runtime's own threads spinning beside the
// waiting one, and more so the more queries are outstanding (tools/query_probe.hip: 0.6-0.9 of a
// core; profiles/r05/config4_cpu/: eight such ranks on one box exhausted its 16-CPU quota and
// configs[4] ran at half speed). The stream is asked only once a wait has lasted 0.25 s - a
// launch that faulted or never wrote its record - never on the way to a normal completion.
// Spin-then-sleep (LBFGS_WAIT=adaptive, the default; =spin: spin from the start, rounds 2-5): a wait
// whose word's last four waits all lasted more than 0.5 ms first sleeps, in steps of at most 200 us,
// through 80 % of the shortest of them less 100 us, and spins only for the rest. At n = 1e8 an
// iteration's host wait is ~11 ms, of which the polling core then sleeps ~90 %; a wait that ends
// early costs at most one sleep step; short waits (small n: tens of us) spin as before.
static void wait_sleep_phase(lbk_ctx* c, const volatile unsigned long long* done, unsigned long long epoch, int word,
                             double t0) {
    double est = 1e30;
    for (int k = 0; k < 4; ++k) est = std::min(est, c->wait_hist[word][k]);
    if (!(est > 0.5e-3) || est > 1e29) return;
    const double until = t0 + 0.8 * est - 100e-6;
    for (;;) {
        if (__atomic_load_n(const_cast<unsigned long long*>(done), __ATOMIC_ACQUIRE) >= epoch) return;
        const double left = until - mono_s();
        if (left <= 0.0) return;
        timespec ts;
        ts.tv_sec = 0;
        ts.tv_nsec = (long)(std::min(left, 200e-6) * 1e9);
        nanosleep(&ts, nullptr);
        c->wait_slept_s += std::min(left, 200e-6);
    }
}

static int small_wait(lbk_ctx* c, unsigned long long epoch, int word) {
    const volatile unsigned long long* done = c->sp_h + word;
    if (__atomic_load_n(const_cast<unsigned long long*>(done), __ATOMIC_ACQUIRE) >= epoch) return 0;
    const double t0 = mono_s();
    if (c->wait_adaptive) wait_sleep_phase(c, done, epoch, word, t0);
    double t_query = 0.0;
    for (unsigned long it = 1;; ++it) {
        if (__atomic_load_n(const_cast<unsigned long long*>(done), __ATOMIC_ACQUIRE) >= epoch) {
            c->wait_hist[word][c->wait_pos[word]++ & 3] = mono_s() - t0;
            c->waits++;
            return 0;
        }
        if ((it & 0xffff) == 0) {
            if (*(volatile unsigned*)c->coop_err_h) break;
            const double now = mono_s();
            if (t_query == 0.0) t_query = now + 0.25;
            if (now < t_query) continue;
            t_query = now + 0.25;
            const hipError_t q = hipStreamQuery(c->stream);
            if (q == hipErrorNotReady) continue;
            if (__atomic_load_n(const_cast<unsigned long long*>(done), __ATOMIC_ACQUIRE) >= epoch) return 0;
            if (q != hipSuccess) {
                snprintf(c->err, sizeof c->err, "cooperative iteration: %s", hipGetErrorString(q));
                return -2;
            }
            snprintf(c->err, sizeof c->err, "cooperative iteration %llu: stream idle, no completion record", epoch);
            return -2;
        }
        __builtin_ia32_pause();
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    snprintf(c->err, sizeof c->err, "cooperative iteration: grid barrier timed out");
    return -2;
}

int lbk_small_fetch(lbk_ctx* c, unsigned long long epoch, int slot, int ncomp, double* totals, int* went,
                    double* rho, double* gamma) {
    if (went) *went = 1;
    if (epoch == 0) return lbk_fetch(c, slot, ncomp, totals);
    if (epoch > c->sp_epoch || epoch + 4 <= c->sp_epoch) {
        snprintf(c->err, sizeof c->err, "lbk_small_fetch: epoch %llu not outstanding", epoch);
        return -1;
    }
    int rc = small_wait(c, epoch);
    if (rc) return rc;
    const int i = (int)(epoch & 3);
    const unsigned long long* r = c->sp_h + 4 + 4 * i;
    const unsigned long long v = __atomic_load_n(r, __ATOMIC_ACQUIRE);
    if ((v >> 1) != epoch) {
        snprintf(c->err, sizeof c->err, "cooperative iteration %llu: record of %llu", epoch, v >> 1);
        return -2;
    }
    double rg[2];
    memcpy(&rg[0], &r[1], sizeof(double));
    memcpy(&rg[1], &r[2], sizeof(double));
    if (rho) *rho = rg[0];
    if (gamma) *gamma = rg[1];
    if (!(v & 1)) {
        // nothing written: release the launch's sequence numbers and bytes. Launches queued
        // behind it are speculative and chained to it, so they did not go either: the counter
        // rolls back to this launch's base
        c->coop_base = c->sp_base[i];
        for (unsigned long long e = epoch; e <= c->sp_epoch; ++e) c->bytes_total -= c->sp_bytes[e & 3];
        if (went) *went = 0;
        return 0;
    }
    double* h = c->h_slots + (int64_t)slot * LBK_SLOT;
    for (int k = 0; k < ncomp; ++k) {
        double t = h[k];
        for (int g = 1; g < LBK_GROUPS; ++g) t = t + h[g * LBK_KMAX + k];
        totals[k] = t;
    }
    return 0;
}

int lbk_mark(lbk_ctx* c) {
    if (!c->mark_ev) HIPCHK(c, hipEventCreateWithFlags(&c->mark_ev, hipEventDisableTiming));
    if (c->pend_slot >= 0) {  // a deferred stage 2 completes before the mark
        const int rc = flush_pending(c);
        if (rc) return rc;
    }
    HIPCHK(c, hipEventRecord(c->mark_ev, c->stream));
    return 0;
}

int lbk_fetch_marked(lbk_ctx* c, int slot, int ncomp, double* totals) {
    if (!c->mark_ev || slot < 0 || slot >= LBK_NSLOTS || !c->slot_mirror[slot] || ncomp > LBK_KMAX ||
        c->slot_s2[slot])  // no mark needed: the slot's launch writes a completion word
        return lbk_fetch(c, slot, ncomp, totals);
    HIPCHK(c, hipEventSynchronize(c->mark_ev));
    if (*(volatile unsigned*)c->coop_err_h) {
        snprintf(c->err, sizeof c->err, "cooperative iteration: grid barrier timed out");
        return -2;
    }
    const double* h = c->h_slots + (int64_t)slot * LBK_SLOT;
    for (int k = 0; k < ncomp; ++k) {
        double t = h[k];
        for (int g = 1; g < LBK_GROUPS; ++g) t = t + h[g * LBK_KMAX + k];
        totals[k] = t;
    }
    return 0;
}

int lbk_small_ok(const lbk_ctx* c, int h) {
    if (c->geo.world != 1 || c->comm || h < 1 || h > LBK_SMALL_HMAX) return 0;
    if (c->coop_max > 0 && c->geo.nseg <= c->coop_max) return 1;
    return persist_fits(c) ? 1 : 0;
}

int lbk_update(lbk_ctx* c, int op, double* out, const double* a, const double* b, double rho, int slot_a,
               int slot_b, double scal) {
    const int64_t npair = c->geo.n_loc / 2;
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((npair + 255) / 256, 16384));
    const double* pa = slot_a >= 0 ? c->slots + (int64_t)slot_a * LBK_SLOT : nullptr;
    const double* pb = slot_b >= 0 ? c->slots + (int64_t)slot_b * LBK_SLOT : nullptr;
    const bool has_b = op == LBK_U_AXPY_Q || op == LBK_U_AXPY_R || op == LBK_U_SUB || op == LBK_U_POINT;
    if (op < 0 || op > LBK_U_POINT || ((op == LBK_U_AXPY_Q || op == LBK_U_AXPY_R) && !pa) ||
        (op == LBK_U_AXPY_R && !pb)) {
        snprintf(c->err, sizeof c->err, "lbk_update: bad op %d / slots", op);
        return -1;
    }
    return launch(c, LBK_K_UPDATE, has_b ? 3 : 2, -1, [&] {
        if (c->geo.n_loc <= 0) return;
#define UPD_CASE(OPC)                                                                                    \
    case OPC:                                                                                            \
        if (c->nt)                                                                                       \
            hipLaunchKernelGGL((k_update<OPC, true>), dim3(nb), dim3(256), 0, c->stream, out, a, b, rho, pa, pb, \
                               scal, c->geo.n_loc);                                                      \
        else                                                                                             \
            hipLaunchKernelGGL((k_update<OPC, false>), dim3(nb), dim3(256), 0, c->stream, out, a, b, rho, pa,   \
                               pb, scal, c->geo.n_loc);                                                  \
        break;
        switch (op) {
            UPD_CASE(LBK_U_AXPY_Q)
            UPD_CASE(LBK_U_AXPY_R)
            UPD_CASE(LBK_U_SCALE)
            UPD_CASE(LBK_U_NEG)
            UPD_CASE(LBK_U_SUB)
            UPD_CASE(LBK_U_POINT)
        }
#undef UPD_CASE
    });
}

int lbk_checksum(lbk_ctx* c, const double* x, uint64_t* c1, uint64_t* c2) {
    HIPCHK(c, hipMemsetAsync(c->d_ck, 0, 2 * sizeof(unsigned long long), c->stream));
    if (c->geo.n_loc > 0) {
        int nb = (int)std::min<int64_t>((c->geo.n_loc + 255) / 256, 2048);
        hipLaunchKernelGGL(k_checksum, dim3(nb), dim3(256), 0, c->stream, x, c->geo.n_loc, c->geo.elem_lo, c->d_ck);
        HIPCHK(c, hipGetLastError());
    }
    if (c->geo.world > 1 && !c->grp && c->xg_on) {
        // integer sums: gather every rank's pair through the peer mailboxes, add on the host
        const int frc = flush_fold(c);  // epochs in order
        if (frc) return frc;
        uint64_t w[LBK_GROUPS * 2];
        HIPCHK(c, hipMemsetAsync(c->d_ckslot, 0, sizeof w, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->d_ckslot + 2 * c->geo.g_lo, c->d_ck, 2 * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                                 c->stream));
        if (lbk_xgmi_exchange_u64(c->xg, c->stream, c->d_ckslot, 2, c->geo.g_lo, c->geo.g_hi) != 0) return -3;
        if (kcopy(c, c->dh_xchg, (const double*)c->d_ckslot, LBK_GROUPS * 2)) return -2;
        HIPCHK(c, hipStreamSynchronize(c->stream));
        memcpy(w, (const void*)c->h_xchg, sizeof w);
        if (lbk_xgmi_failed(c->xg)) {
            snprintf(c->err, sizeof c->err, "xgmi exchange timed out waiting for a peer");
            return -3;
        }
        uint64_t a = 0, b = 0;
        for (int g = 0; g < LBK_GROUPS; ++g) {
            a += w[2 * g];
            b += w[2 * g + 1];
        }
        *c1 = a;
        *c2 = b;
        return 0;
    }
    if ((c->geo.world > 1 || c->comm) && !c->grp) {
        if (!c->comm) {
            snprintf(c->err, sizeof c->err, "sharded context has no exchange backend");
            return -3;
        }
        rccl_debug_stall(c);
        const int rrc = rccl_settle(c, ncclAllReduce(c->d_ck, c->d_ck, 2, ncclUint64, ncclSum, c->comm, c->stream),
                                    "ncclAllReduce");
        if (rrc) return rrc;
    }
    if (kcopy(c, c->dh_xchg, (const double*)c->d_ck, 2)) return -2;  // a kernel's stores, not a DMA
    {
        const int wrc = stream_wait(c, "trajectory checksum (ncclAllReduce)");
        if (wrc) return wrc;
    }
    memcpy(c->h_ck, (const void*)c->h_xchg, 2 * sizeof(unsigned long long));
    *c1 = c->h_ck[0];
    *c2 = c->h_ck[1];
    if (c->grp) {  // integer sums: exact in any order
        lbk_group* G = c->grp;
        G->ck[c->geo.rank][0] = *c1;
        G->ck[c->geo.rank][1] = *c2;
        pthread_barrier_wait(&G->bar);
        unsigned long long a = 0, b = 0;
        for (int k = 0; k < G->world; ++k) {
            a += G->ck[k][0];
            b += G->ck[k][1];
        }
        pthread_barrier_wait(&G->bar);
        *c1 = a;
        *c2 = b;
    }
    return 0;
}

double lbk_total(const double* groups64, int comp) {
    double t = groups64[comp];
    for (int g = 1; g < LBK_GROUPS; ++g) t = t + groups64[g * LBK_KMAX + comp];
    return t;
}

int lbk_fetch_groups(lbk_ctx* c, int slot, double* groups64) {
    const int frc = flush_pending(c);
    if (frc) return frc;
    double* h = slot_host(c, slot);
    const size_t bytes = sizeof(double) * LBK_GROUPS * slot_stride(slot);
    const int si = slot < LBK_NSLOTS ? slot : LBK_NSLOTS + slot - LBK_WSLOT0;
    if (c->slot_s2[si] && c->slot_mirror[si]) {  // a ticket launch's completion word, no stream sync
        const int rc = small_wait(c, c->slot_s2[si], 1);
        if (rc) return rc;
        memcpy(groups64, h, bytes);
        return 0;
    }
    // The slot reaches its host mirror through k_slot_publish's stores (a kernel on the solver
    // stream, behind everything queued so far), never through a copy engine: a DMA into pinned
    // memory returned stale groups here (an emulated 4-rank vector-free solve fetched a wrong
    // f(x0) in 3 of 4 suite runs with that copy, none since; tools/contig_probe.hip).
    double* hd = slot < LBK_NSLOTS ? c->dh_slots + (int64_t)slot * LBK_SLOT
                                   : c->dh_wslots + (int64_t)(slot - LBK_WSLOT0) * LBK_WSLOT;
    if (!c->comm && !c->grp) {
        // polled on the completion word (no stream synchronisation: no runtime thread spins)
        hipLaunchKernelGGL(k_slot_publish, dim3(1), dim3(256), 0, c->stream, (const double*)slot_base(c, slot), hd,
                           (int)(LBK_GROUPS * slot_stride(slot)), c->sp_dh + 2, ++c->pub_epoch);
        HIPCHK(c, hipGetLastError());
        const int rc = small_wait(c, c->pub_epoch, 2);
        if (rc) return rc;
    } else {
        if (!c->slot_mirror[si]) {
            hipLaunchKernelGGL(k_slot_publish, dim3(1), dim3(256), 0, c->stream, (const double*)slot_base(c, slot), hd,
                               (int)(LBK_GROUPS * slot_stride(slot)), c->sp_dh + 2, ++c->pub_epoch);
            HIPCHK(c, hipGetLastError());
        }
        const int wrc = stream_wait(c, "result slot (ncclAllGather)");
        if (wrc) return wrc;
    }
    if (c->xg_on && lbk_xgmi_failed(c->xg)) {
        snprintf(c->err, sizeof c->err, "xgmi exchange timed out waiting for a peer");
        return -3;
    }
    if (*(volatile unsigned*)c->coop_err_h) {
        snprintf(c->err, sizeof c->err, "cooperative iteration: grid barrier timed out");
        return -2;
    }
    memcpy(groups64, h, bytes);
    return 0;
}

// fixed-order total Q0 + Q1 + ... + Q7 of each component (regular or wide slot)
int lbk_fetch(lbk_ctx* c, int slot, int ncomp, double* totals) {
    double gw[LBK_WSLOT];
    int rc = lbk_fetch_groups(c, slot, gw);
    if (rc) return rc;
    const int ks = slot_stride(slot);
    for (int k = 0; k < ncomp; ++k) {
        double t = gw[k];
        for (int g = 1; g < LBK_GROUPS; ++g) t = t + gw[g * ks + k];
        totals[k] = t;
    }
    return 0;
}

int lbk_sync(lbk_ctx* c) {
    const int wrc = stream_wait(c, "stream synchronisation");
    if (wrc) return wrc;
    if (c->xg_on && lbk_xgmi_failed(c->xg)) {
        snprintf(c->err, sizeof c->err, "xgmi exchange timed out waiting for a peer");
        return -3;
    }
    return 0;
}

int lbk_peer_handle(lbk_ctx* c, void* out) {
    if (!c->xg) return -1;
    return lbk_xgmi_handle(c->xg, out);
}

int lbk_peer_connect(lbk_ctx* c, const void* handles) {
    if (!c->xg) return -1;
    HIPCHK(c, hipSetDevice(c->device));
    return lbk_xgmi_connect(c->xg, handles, c->stream, c->err, sizeof c->err);
}

int lbk_peer_enable(lbk_ctx* c, int on) {
    if (on && !lbk_xgmi_connected(c->xg)) return -5;
    if (!on && !c->comm && !c->grp) return -5;  // nothing else to exchange through
    if (!on) {  // a folded exchange in flight is collected through the mailboxes first
        const int rc = flush_fold(c);
        if (rc) return rc;
    }
    c->xg_on = on ? 1 : 0;
    c->xf_on = 0;
    if (on && c->fold_env && c->geo.world > 1 && !c->grp && lbk_xgmi_fold_info(c->xg, &c->xf) == 0 &&
        (c->fold_env == 2 || !c->xf.shared_device || c->cu_part))
        c->xf_on = 1;
    return 0;
}

int lbk_cu_partition(const lbk_ctx* c) { return c->cu_part ? c->cu_count : 0; }

int lbk_vec_fallbacks(const lbk_ctx* c) { return c->vec_plain_fallbacks; }

int lbk_wait_stats(const lbk_ctx* c, double* slept_s, unsigned long long* waits, int* adaptive) {
    if (slept_s) *slept_s = c->wait_slept_s;
    if (waits) *waits = c->waits;
    if (adaptive) *adaptive = c->wait_adaptive;
    return 0;
}

int lbk_coop_info(const lbk_ctx* c, int* coop_max, int* search_max, int* fallbacks) {
    if (coop_max) *coop_max = c->coop_max;
    if (search_max) *search_max = c->dev_wolfe ? c->wolfe_max : 0;
    if (fallbacks) *fallbacks = c->coop_fallbacks;
    return 0;
}

int lbk_stream_probe(lbk_ctx* c, double* q, const double* const* ys, const double* const* ss, int npairs,
                     int launches, double* us, int variant, double* const* outs) {
    if (launches < 1 || !us || !q || !ys || !ss || npairs < 1) return -1;
    for (int k = 0; k < npairs; ++k)
        if (!ys[k] || !ss[k]) return -1;
    HIPCHK(c, hipSetDevice(c->device));
    {
        const int rc = flush_pending(c);
        if (rc) return rc;
    }
    if (nblocks(c) <= 0) {
        *us = 0.0;
        return 0;
    }
    hipEvent_t a = ev_get(c), b = ev_get(c);
    if (!a || !b) {
        snprintf(c->err, sizeof c->err, "hipEventCreate failed");
        return -2;
    }
    // variants (gap analysis against k_axpy_dot): 0 the box probe (alpha = 0, no
    // reduction); 1 the same with alpha != 0; 2 + the pass's segment reduction stored plainly (no
    // stage 2); 3 + the collect stage 2 into a scratch slot; 4 / 5 the product's own k_axpy_dot
    // launch (lbk_axpy_dot: source slot read, collect stage 2), alpha = 0 / != 0, chained through
    // two scratch slots as the passes chain theirs
    constexpr int kProbeSlot = LBK_NSLOTS - 2;  // scratch slots no solver path uses
    if (variant == 4 || variant == 5) {  // the chained source slot starts at 0.0
        HIPCHK(c, hipMemsetAsync(c->slots + (int64_t)kProbeSlot * LBK_SLOT, 0, 2 * LBK_SLOT * sizeof(double),
                                 c->stream));
    }
    HIPCHK(c, hipEventRecord(a, c->stream));
    const int par = c->rev_par;  // the solver's walk parity is left as it was
    const double bytes_before = c->bytes_total;
    for (int i = 0; i < launches; ++i) {
        const double* y = ys[(i + 1) % npairs];
        const double* s = ss[i % npairs];
        hipError_t e = hipSuccess;
        if (variant == 4 || variant == 5) {
            const int src = kProbeSlot + (i & 1), dst = kProbeSlot + ((i + 1) & 1);
            const int rc = lbk_axpy_dot(c, q, q, y, s, variant == 5 ? 1e-12 : 0.0, src * LBK_KMAX, dst);
            if (rc) {
                c->rev_par = par;
                return rc;
            }
            continue;  // launch() flips the walk
        }
        const Geo g = kgeo(c);  // alternating walk, as the passes
        const double alpha = variant == 1 ? 1e-3 : 0.0;
        if (variant == 6) {  // the commit's 4 R + 4 W: x = q, g = y, r and s from the pool; 4 scratch outputs
            if (!outs || !outs[0] || !outs[1] || !outs[2] || !outs[3]) {
                c->rev_par = par;
                return -1;
            }
            const double* rr = ys[(i + 2) % npairs];
            NT_DISPATCH(c, hipLaunchKernelGGL(k_probe_commit<NT_>, dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream,
                                              OpProbeCommit<NT_>{q, y, rr, s, outs[0], outs[1], outs[2], outs[3], 1e-3,
                                                                 0.5},
                                              g, c->partials));
        } else if (variant <= 1) {
            NT_DISPATCH(c, hipLaunchKernelGGL(k_probe_stream<NT_>, dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, q, y,
                                              s, alpha, g, c->partials));
        } else {
            Red r = kred(c, kProbeSlot);
            if (variant == 2) {
                r.ll = nullptr;
                r.ticket = 0;
            }
            NT_DISPATCH(c, hipLaunchKernelGGL(k_probe_stream2<NT_>, dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, q, y,
                                              s, alpha, g, r));
        }
        c->rev_par ^= 1;
        e = hipGetLastError();
        if (e != hipSuccess) c->rev_par = par;
        HIPCHK(c, e);
    }
    c->rev_par = par;
    c->bytes_total = bytes_before;  // probe launches are not solver traffic
    HIPCHK(c, hipEventRecord(b, c->stream));
    HIPCHK(c, hipEventSynchronize(b));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, a, b));
    c->ev_free.push_back(a);
    c->ev_free.push_back(b);
    *us = (double)ms * 1e3 / launches;
    return 0;
}

int lbk_exchange_bench(lbk_ctx* c, int backend, int ks, int iters, double* us) {
    if ((c->geo.world <= 1 && !c->comm) || c->grp || ks < 1 || ks > LBK_KW || iters < 1) return -1;
    if (backend == 2 && !lbk_xgmi_connected(c->xg)) return -5;
    if (backend == 1 && !c->comm) return -5;
    if (backend != 1 && backend != 2) return -1;
    {
        const int rc = flush_fold(c);
        if (rc) return rc;
    }
    const int saved = c->xg_on;
    c->xg_on = backend == 2;
    double* buf = nullptr;
    HIPCHK(c, hipMalloc(&buf, sizeof(double) * LBK_WSLOT));
    HIPCHK(c, hipMemsetAsync(buf, 0, sizeof(double) * LBK_WSLOT, c->stream));
    // an RCCL wait is bounded (rccl_stream_wait); the mailbox kernels bound their own waits
    auto wait = [&]() { return backend == 1 ? rccl_stream_wait(c, "RCCL exchange timing")
                                            : (hipStreamSynchronize(c->stream) == hipSuccess ? 0 : -2); };
    int rc = exchange_buf(c, buf, ks);  // warm-up, also lines the ranks up
    if (rc == 0) rc = wait();
    timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < iters && rc == 0; ++i) rc = exchange_buf(c, buf, ks);
    if (rc == 0) rc = wait();
    clock_gettime(CLOCK_MONOTONIC, &t1);
    c->xg_on = saved;
    if (!c->rccl_hung) (void)hipFree(buf);
    if (rc == 0 && backend == 2 && lbk_xgmi_failed(c->xg)) rc = -3;
    *us = ((double)(t1.tv_sec - t0.tv_sec) * 1e6 + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-3) / iters;
    return rc;
}

int lbk_exchange_fold(const lbk_ctx* c) { return c->xf_on; }

int lbk_exchange_backend(const lbk_ctx* c) {
    if (c->geo.world <= 1) return c->comm ? 1 : 0;
    if (c->grp) return 3;
    if (c->xg_on) return 2;
    return c->comm ? 1 : 0;
}

void lbk_prof_enable(lbk_ctx* c, int on) { c->prof_on = on; }

int lbk_prof_get(lbk_ctx* c, int kind, double* ms, int64_t* launches, double* bytes) {
    if (prof_flush(c) != 0) return -2;
    if (kind < 0 || kind >= LBK_K_COUNT) return -1;
    *ms = c->prof_ms[kind];
    *launches = c->prof_n[kind];
    *bytes = c->prof_bytes[kind];
    if (kind == LBK_K_EXCHANGE && c->fold_wait) {
        // folded exchanges have no launch of their own: their wait, as the consuming pass's first
        // workgroup measured it in its prologue, counts as exchange time
        unsigned long long ticks = 0;
        HIPCHK(c, hipMemcpy(&ticks, c->fold_wait, sizeof ticks, hipMemcpyDeviceToHost));
        *ms += (double)ticks / c->wall_khz;
    }
    return 0;
}

void lbk_prof_reset(lbk_ctx* c) {
    prof_flush(c);
    if (c->fold_wait) (void)hipMemset(c->fold_wait, 0, sizeof(unsigned long long));
    for (int k = 0; k < LBK_K_COUNT; ++k) {
        c->prof_ms[k] = 0;
        c->prof_n[k] = 0;
        c->prof_bytes[k] = 0;
    }
}

double lbk_bytes_moved(const lbk_ctx* c) { return c->bytes_total; }

void lbk_set_ghost_slot(lbk_ctx* c, int slot) { c->ghost_slot = slot; }

lbk_group* lbk_group_create(int world) {
    if (world < 1 || world > LBK_GROUPS) return nullptr;
    lbk_group* G = new (std::nothrow) lbk_group();
    if (!G) return nullptr;
    G->world = world;
    if (pthread_barrier_init(&G->bar, nullptr, (unsigned)world) != 0) {
        delete G;
        return nullptr;
    }
    return G;
}

void lbk_group_destroy(lbk_group* G) {
    if (!G) return;
    pthread_barrier_destroy(&G->bar);
    delete G;
}

}  // extern "C"

