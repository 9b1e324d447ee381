// lbfgs_xgmi.hip — xGMI peer exchange of result-slot group partials for sharded runs
// (interface and wire format: lbfgs_xgmi.h; where it sits in the solver: DESIGN.md §5).
//
// Why not the collective library for this: a sharded iteration needs ~2h + 3 dependent
// all-gathers of 64-768 bytes (every two-loop pass waits for the previous pass's global dot).
// At that size an RCCL all-gather is pure latency: a multi-stage ring protocol launched as its
// own kernel. Here one workgroup stores this rank's values into each peer's mailbox (posted
// xGMI writes, one hop on MI355X's fully connected 8-GPU topology) and polls its own local
// mailbox: the exchange costs one kernel boundary plus one xGMI write latency.
#include "lbfgs_xgmi.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#define XG_GROUPS 8
#define XG_MAXW 8

struct XPeers {
    unsigned long long* mb[XG_MAXW];  // each rank's mailbox as mapped in this process
};

struct lbk_xgmi {
    int device, rank, world, positions;
    unsigned long long* mb;  // own mailbox: [2 parities][positions][2 words], uncached
    XPeers peers;
    hipIpcMemHandle_t handle;
    unsigned* err_h;  // pinned, written by the kernel on a timeout
    unsigned* err_d;
    unsigned* err_dev;  // the same flag in device memory: what the waiting polls read
    unsigned epoch;
    unsigned long long timeout_ticks;  // wall-clock ticks (hipDeviceAttributeWallClockRate)
    double wall_khz;
    int connected;
    std::vector<unsigned long long*> opened;  // peer mappings to close
    unsigned long long** peers_dev;           // device copy of peers.mb (folded exchanges)
    int shared_device;                        // a peer's mailbox is on this GPU (or unknown)
};

namespace {

// a wait ends past `timeout` ticks, or after 1/65536 of it once the error flag (device copy) shows
// an earlier timeout of this rank (one timeout per solve on a broken channel, not one per exchange)
__device__ __forceinline__ bool wait_over(unsigned long long t0, unsigned long long timeout, const unsigned* errd) {
    const unsigned long long el = wall_clock64() - t0;
    if (el > timeout) return true;
    return el > (timeout >> 16) && __hip_atomic_load(errd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}
__device__ __forceinline__ void set_failed(unsigned* err, unsigned* errd) {
    __hip_atomic_store(errd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One workgroup. Push: own positions [lo, hi) to every peer's mailbox (two LL words per 64-bit
// value). Poll: every other position of the own mailbox until both of its words carry this
// epoch, then write the value into the slot. A peer that never arrives ends the wait after
// `timeout` wall-clock ticks with *err set and the value NaN (the host reports the failure at its
// next synchronisation) instead of a hung queue.
__global__ __launch_bounds__(256) void k_xgmi_exchange(unsigned long long* __restrict__ slot, int ks, int g_lo,
                                                        int g_hi, XPeers P, int rank, int world, int positions,
                                                        unsigned epoch, unsigned* err, unsigned* errd,
                                                        unsigned long long timeout,
                                                        unsigned long long* __restrict__ hm) {
    const int lo = g_lo * ks, hi = g_hi * ks, own = hi - lo, npos = XG_GROUPS * ks;
    const size_t par = (size_t)(epoch & 1u) * (size_t)positions * 2;
    const unsigned long long tag = (unsigned long long)epoch << 32;
    for (int i = threadIdx.x; i < own * world; i += blockDim.x) {
        const int p = i / own, j = lo + i % own;
        const unsigned long long v = slot[j];
        if (p == rank) {
            if (hm) hm[j] = v;
            continue;
        }
        unsigned long long* dst = P.mb[p] + par + 2 * (size_t)j;
        __hip_atomic_store(dst, tag | (v & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dst + 1, tag | (v >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const unsigned long long* mine = P.mb[rank] + par;
    const unsigned long long t0 = wall_clock64();
    for (int j = threadIdx.x; j < npos; j += blockDim.x) {
        if (j >= lo && j < hi) continue;
        unsigned long long a, b;
        for (;;) {
            a = __hip_atomic_load(mine + 2 * (size_t)j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            b = __hip_atomic_load(mine + 2 * (size_t)j + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((unsigned)(a >> 32) == epoch && (unsigned)(b >> 32) == epoch) break;
            if (wait_over(t0, timeout, errd)) {
                set_failed(err, errd);
                a = 0;
                b = 0x7ff80000ull;  // quiet NaN
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const unsigned long long v = (a & 0xffffffffull) | ((b & 0xffffffffull) << 32);
        slot[j] = v;
        if (hm) hm[j] = v;
    }
}

// Folded exchanges (lbk_xgmi_fold): wait for the positions the peers' passes pushed for `epoch`
// (component 0 of every group of the other ranks; with `edges`, the rank-edge components 1 of each
// rank's first group and 2 of its last) and write them into the slot.
__global__ __launch_bounds__(64) void k_xgmi_collect(unsigned long long* __restrict__ slot, int ks, int g_lo,
                                                     int g_hi, const unsigned long long* mine, int world,
                                                     unsigned epoch, int edges, unsigned* err, unsigned* errd,
                                                     unsigned long long timeout) {
    const int per = XG_GROUPS / world;
    const int j = threadIdx.x;  // 0..7 group values, 8..15 first-group edges, 16..23 last-group edges
    if (j >= 3 * XG_GROUPS || (j >= XG_GROUPS && !edges)) return;
    const int g = j % XG_GROUPS, kind = j / XG_GROUPS;
    if (g >= g_lo && g < g_hi) return;
    if (kind == 1 && g % per != 0) return;
    if (kind == 2 && g % per != per - 1) return;
    const int pos = g * ks + kind;
    unsigned long long a, b;
    const unsigned long long t0 = wall_clock64();
    for (;;) {
        a = __hip_atomic_load(mine + 2 * (size_t)pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        b = __hip_atomic_load(mine + 2 * (size_t)pos + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((unsigned)(a >> 32) == epoch && (unsigned)(b >> 32) == epoch) break;
        if (wait_over(t0, timeout, errd)) {
            set_failed(err, errd);
            a = 0;
            b = 0x7ff80000ull;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    slot[pos] = (a & 0xffffffffull) | ((b & 0xffffffffull) << 32);
}

unsigned long long ticks(const lbk_xgmi* x, double seconds) {
    return (unsigned long long)(seconds * x->wall_khz * 1e3);
}

int launch(lbk_xgmi* x, hipStream_t s, unsigned long long* slot, int ks, int g_lo, int g_hi,
           unsigned long long timeout, unsigned long long* hm = nullptr) {
    if (ks < 1 || XG_GROUPS * ks > x->positions || g_lo < 0 || g_hi > XG_GROUPS || g_lo >= g_hi) return -1;
    lbk_xgmi_next_epoch(x);
    hipLaunchKernelGGL(k_xgmi_exchange, dim3(1), dim3(256), 0, s, slot, ks, g_lo, g_hi, x->peers, x->rank,
                       x->world, x->positions, x->epoch, x->err_d, x->err_dev, timeout, hm);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// a value with pseudo-random bits in both 32-bit halves, known to every rank
double pattern(int owner, int round, int j) {
    unsigned long long h = (unsigned long long)(owner * 131 + round * 17 + j + 1) * 0x9E3779B97F4A7C15ull;
    h = 0x3ff0000000000000ull | (h >> 12);
    double v;
    memcpy(&v, &h, sizeof v);
    return v;
}

}  // namespace

int lbk_xgmi_create(lbk_xgmi** out, int device, int rank, int world, int positions, char* err, size_t cap) {
    *out = nullptr;
    if (world < 1 || world > XG_MAXW || rank < 0 || rank >= world || positions < XG_GROUPS) return -1;
    lbk_xgmi* x = new (std::nothrow) lbk_xgmi();
    if (!x) return -4;
    x->device = device;
    x->rank = rank;
    x->world = world;
    x->positions = positions;
    const size_t bytes = sizeof(unsigned long long) * 2 * 2 * (size_t)positions;
    // uncached: the owner's polls and the peers' xGMI stores meet in HBM, never in a stale L2
    // line; fine-grained memory (coherent, cached per access) is the fallback
    hipError_t e = hipExtMallocWithFlags((void**)&x->mb, bytes, hipDeviceMallocUncached);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        e = hipExtMallocWithFlags((void**)&x->mb, bytes, hipDeviceMallocFinegrained);
    }
    if (e == hipSuccess) e = hipMemset(x->mb, 0, bytes);
    if (e == hipSuccess) e = hipIpcGetMemHandle(&x->handle, x->mb);
    if (e == hipSuccess) e = hipMalloc((void**)&x->err_dev, sizeof(unsigned));
    if (e == hipSuccess) e = hipMemset(x->err_dev, 0, sizeof(unsigned));
    if (e == hipSuccess) e = hipHostMalloc((void**)&x->err_h, sizeof(unsigned), hipHostMallocMapped);
    if (e == hipSuccess) {
        *x->err_h = 0;
        e = hipHostGetDevicePointer((void**)&x->err_d, x->err_h, 0);
    }
    int khz = 0;
    if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        snprintf(err, cap, "xgmi mailbox: %s", hipGetErrorString(e));
        lbk_xgmi_destroy(x);
        return -2;
    }
    x->wall_khz = khz > 0 ? khz : 100000.0;
    double tmo = 60.0;  // a peer that has not arrived after this long is gone
    if (const char* s = getenv("LBFGS_XGMI_TIMEOUT")) tmo = atof(s);
    x->timeout_ticks = ticks(x, tmo);
    for (int p = 0; p < XG_MAXW; ++p) x->peers.mb[p] = nullptr;
    x->peers.mb[rank] = x->mb;
    *out = x;
    return 0;
}

void lbk_xgmi_destroy(lbk_xgmi* x) {
    if (!x) return;
    (void)hipSetDevice(x->device);
    (void)hipDeviceSynchronize();
    for (auto* p : x->opened) (void)hipIpcCloseMemHandle(p);
    if (x->peers_dev) (void)hipFree(x->peers_dev);
    if (x->mb) (void)hipFree(x->mb);
    if (x->err_h) (void)hipHostFree(x->err_h);
    if (x->err_dev) (void)hipFree(x->err_dev);
    delete x;
}

int lbk_xgmi_handle(const lbk_xgmi* x, void* out) {
    static_assert(sizeof(hipIpcMemHandle_t) <= LBK_PEER_HANDLE_BYTES, "handle size");
    memset(out, 0, LBK_PEER_HANDLE_BYTES);
    memcpy(out, &x->handle, sizeof(hipIpcMemHandle_t));
    return 0;
}

int lbk_xgmi_connected(const lbk_xgmi* x) { return x && x->connected; }
int lbk_xgmi_failed(const lbk_xgmi* x) { return x && x->err_h && *(volatile unsigned*)x->err_h != 0; }

int lbk_xgmi_connect(lbk_xgmi* x, const void* handles, hipStream_t stream, char* err, size_t cap) {
    if (x->connected) return 0;
    const unsigned char* hb = static_cast<const unsigned char*>(handles);
    for (int p = 0; p < x->world; ++p) {
        if (p == x->rank) continue;
        hipIpcMemHandle_t h;
        memcpy(&h, hb + (size_t)p * LBK_PEER_HANDLE_BYTES, sizeof h);
        void* ptr = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            snprintf(err, cap, "xgmi: hipIpcOpenMemHandle(rank %d): %s", p, hipGetErrorString(e));
            return -2;
        }
        x->peers.mb[p] = static_cast<unsigned long long*>(ptr);
        x->opened.push_back(x->peers.mb[p]);
        // which GPU holds the peer's mailbox: ranks sharing this GPU (one-card rehearsals and
        // tests) must not fold their exchanges into the passes (a pass's spinning
        // workgroups could hold every CU the peer's producing kernel needs)
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, ptr) != hipSuccess || at.device == x->device) x->shared_device = 1;
        (void)hipGetLastError();
    }
    // self-test: 4 exchanges (both mailbox parities twice) of the widest slot, checked bit for
    // bit on the host; a short timeout so that a broken path fails fast and the caller can
    // fall back to the collective library
    const int ks = x->positions / XG_GROUPS, npos = XG_GROUPS * ks, per = XG_GROUPS / x->world;
    const int g_lo = x->rank * per, g_hi = g_lo + per;
    double selftest_s = 30.0;
    if (const char* s = getenv("LBFGS_XGMI_SELFTEST_TIMEOUT")) selftest_s = atof(s);
    std::vector<double> h(npos);
    unsigned long long* d = nullptr;
    if (hipMalloc((void**)&d, sizeof(double) * npos) != hipSuccess) {
        snprintf(err, cap, "xgmi: self-test buffer");
        return -2;
    }
    int rc = 0;
    for (int t = 0; t < 4 && rc == 0; ++t) {
        for (int j = 0; j < npos; ++j) h[j] = (j >= g_lo * ks && j < g_hi * ks) ? pattern(x->rank, t, j) : -1.0;
        hipError_t e = hipMemcpyAsync(d, h.data(), sizeof(double) * npos, hipMemcpyHostToDevice, stream);
        if (e == hipSuccess && launch(x, stream, d, ks, g_lo, g_hi, ticks(x, selftest_s)) != 0) e = hipErrorLaunchFailure;
        if (e == hipSuccess) e = hipMemcpyAsync(h.data(), d, sizeof(double) * npos, hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        if (e != hipSuccess) {
            snprintf(err, cap, "xgmi: self-test: %s", hipGetErrorString(e));
            rc = -2;
            break;
        }
        if (lbk_xgmi_failed(x)) {
            snprintf(err, cap, "xgmi: self-test round %d timed out waiting for a peer", t);
            rc = -3;
            break;
        }
        for (int j = 0; j < npos; ++j) {
            const int owner = (j / ks) / per;
            const double want = pattern(owner, t, j);
            if (memcmp(&h[j], &want, sizeof want) != 0) {
                snprintf(err, cap, "xgmi: self-test round %d: position %d (rank %d) wrong", t, j, owner);
                rc = -3;
                break;
            }
        }
    }
    (void)hipFree(d);
    if (rc == 0 && !x->peers_dev) {  // the mapped mailboxes for the passes that push themselves
        hipError_t e = hipMalloc((void**)&x->peers_dev, sizeof(unsigned long long*) * XG_MAXW);
        if (e == hipSuccess)
            e = hipMemcpy(x->peers_dev, x->peers.mb, sizeof(unsigned long long*) * XG_MAXW, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            snprintf(err, cap, "xgmi: peer table: %s", hipGetErrorString(e));
            rc = -2;
        }
    }
    if (rc == 0) x->connected = 1;
    return rc;
}

int lbk_xgmi_fold_info(const lbk_xgmi* x, lbk_xgmi_fold* out) {
    if (!x || !x->connected || !x->peers_dev) return -5;
    out->peers = x->peers_dev;
    out->own = x->mb;
    out->err = x->err_d;
    out->errd = x->err_dev;
    out->timeout = x->timeout_ticks;
    out->positions = x->positions;
    out->rank = x->rank;
    out->world = x->world;
    out->shared_device = x->shared_device;
    return 0;
}

unsigned lbk_xgmi_next_epoch(lbk_xgmi* x) {
    ++x->epoch;
    if (x->epoch == 0) ++x->epoch;  // 0 marks an empty mailbox word
    return x->epoch;
}

int lbk_xgmi_collect(lbk_xgmi* x, hipStream_t stream, double* slot, int ks, int g_lo, int g_hi, unsigned epoch,
                     int edges) {
    if (!x->connected) return -5;
    const unsigned long long* mine = x->mb + (size_t)(epoch & 1u) * (size_t)x->positions * 2;
    hipLaunchKernelGGL(k_xgmi_collect, dim3(1), dim3(64), 0, stream, reinterpret_cast<unsigned long long*>(slot), ks,
                       g_lo, g_hi, mine, x->world, epoch, edges, x->err_d, x->err_dev, x->timeout_ticks);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lbk_xgmi_exchange(lbk_xgmi* x, hipStream_t stream, double* slot, int ks, int g_lo, int g_hi,
                      double* host_mirror) {
    if (!x->connected) return -5;
    return launch(x, stream, reinterpret_cast<unsigned long long*>(slot), ks, g_lo, g_hi, x->timeout_ticks,
                  reinterpret_cast<unsigned long long*>(host_mirror));
}

int lbk_xgmi_exchange_u64(lbk_xgmi* x, hipStream_t stream, uint64_t* slot, int ks, int g_lo, int g_hi) {
    if (!x->connected) return -5;
    return launch(x, stream, reinterpret_cast<unsigned long long*>(slot), ks, g_lo, g_hi, x->timeout_ticks);
}
