#pragma once
// lbfgs_kernels_impl.h — MI355X (gfx950, CDNA4) device layer of the L-BFGS solver: the kernels,
// the context and the launch helpers, shared by the three translation units that define the
// lbk_* entry points (lbfgs_kernels.hip: lifecycle, two-loop passes, objectives, results;
// lbfgs_kernels_commit.hip: commit and batched trials; lbfgs_kernels_vf.hip: vector-free mode),
// compiled in parallel. Everything here has internal linkage.
//
//
// Every kernel is one streaming pass over fp64 n-vectors that fuses the elementwise work of
// one step of the reference algorithm with the dot products that depend on it:
//
//   k_axpy_dot   q = q_in - alpha_{i+1} y_{i+1};  s_i . q        (lbfgs.cpp:124-138, one i)
//   k_mid        r = (q - alpha_0 y_0) * gamma;   y_0 . r        (:134-137, :141-154, :160)
//   k_axpy2_dot  r += s_i (alpha_i - beta_i);      y_{i+1} . r    (:157-165)
//   k_last       d = -(r + s (alpha - beta));      g . d          (:163-171)
//   k_commit     d (any mode), x_new = x + a d, f(x_new), g_new, s, y and the five dots
//                g.d, s.y, y.y, g_new.g_new, s.g_new, g_new.d in ONE pass  (:171-205)
//   k_trial      f(x + a d) [, g_t and g_t . d]  without materialising x + a d
//                (line_search.cpp:19-30, :125-189)
//
// The scalar that a pass needs from the previous pass (alpha_i = rho_i (s_i . q), beta_i) is
// never sent to the host: the producing kernel leaves 8 group partials in a device result
// slot and the consuming kernel forms the fixed-order total in its prologue.
//
// Canonical reduction order (restated in oracle/lbfgs_oracle.c for checking):
//   segment s = [s L, min((s+1) L, n)), L = max(512, roundup(ceil(n/8192), 128)), one 256-thread
//   workgroup per segment; thread (w, lane) visits rows 4u + w (128 elements each), two
//   elements per lane (one 16-B load), accumulating with v_fma_f64 (dots) / v_add_f64 (sums);
//   wave butterfly (shfl_xor 1..32) -> ((w0 + w1) + (w2 + w3)) = segment partial;
//   group g = segments 1024g..1024g+1023, reduced by the workgroup that arrives last at the
//   group's ticket (write-through sc1 partials, agent-scope atomic ticket) into a balanced
//   tree; total = Q0 + Q1 + ... + Q7 in order. The order depends on n only, so results are
//   identical for any grid, any launch timing and any number of GPUs that divides 8.
//
// Elementwise arithmetic is compiled with -ffp-contract=off so every expression below rounds
// exactly like the reference's C++ (x86-64, no FMA); the only FMAs are the explicit fma() of
// the dot accumulations.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <pthread.h>
#include <unistd.h>
#include <cstring>
#include <ctime>
#include <new>
#include <vector>

#include "lbfgs_device.h"
#include "lbfgs_xgmi.h"

#define LB_BLOCK 256
#define LBK_FRONT 32

namespace {

struct Geo {
    int64_t n, L, nseg, seg_lo, elem_lo, n_loc;
    int g_lo, g_hi;
    int spg;            // segments per group (1024; fewer, longer segments in the vector-free commit)
    int rev;            // 1: workgroup b takes the rank's segment nblocks-1-b (see LBFGS_REV)
    const double* ppart;  // deferred stage 2: the producer's partials of this launch's first source
    double* edge_slot;  // sharded: where d[0] / d[n_loc-1] of this rank are published
};

// Folded exchange, consumer side (sharded over the xGMI mailboxes): the other
// ranks' group values of this launch's first source arrive in this rank's mailbox (parity of
// mepoch applied), pushed there by the producing pass itself; src_total polls them. A separate
// kernel argument of the fold-capable passes, so the other kernels' Geo stays as it was.
struct FoldSrc {
    const unsigned long long* mbx;  // nullptr: the source is an ordinary slot
    unsigned mepoch;
    unsigned* merr;   // pinned error flag (the host reads it)
    unsigned* merrd;  // its device copy (the waiting polls read it)
    unsigned long long mtmo;
    unsigned long long* wait;  // profiling: workgroup 0 adds its prologue's wall-clock ticks here
};

// Folded exchange, producer side: where a pass pushes its group values (stage 2's last arriver,
// or k_group_reduce) and its rank-edge values (publish_edges) - every peer's mailbox at `epoch`,
// in the exchange kernel's wire format (lbfgs_xgmi.h). peers == nullptr: no push.
struct FoldPush {
    unsigned long long* const* peers;
    int positions, world, rank;
    unsigned epoch;
};

__device__ __forceinline__ void fold_push(const FoldPush& fp, int pos, double v) {
    const size_t par = (size_t)(fp.epoch & 1u) * (size_t)fp.positions * 2;
    const unsigned long long tag = (unsigned long long)fp.epoch << 32;
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    for (int p = 0; p < fp.world; ++p) {
        if (p == fp.rank) continue;
        unsigned long long* dst = fp.peers[p] + par + 2 * (size_t)pos;
        __hip_atomic_store(dst, tag | (u & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dst + 1, tag | (u >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

struct Red {
    double* partials;  // [LBK_KW][LBK_SEGS], local segment index
    unsigned* cnt;     // [LBK_GROUPS] tickets
    double* slot;      // this launch's result slot [LBK_GROUPS][kstride]
    double* hslot;     // its pinned host mirror, written alongside (one rank), or nullptr
    int ticket;        // 1: in-launch last-arriver stage 2; 0: k_group_reduce after the launch
    int kstride;       // LBK_KMAX (regular slots) or LBK_KW (wide slots)
    // tickets, one rank, host-read slot: the last arriver stores `epoch` into this pinned word
    // after the slot's mirror, so the host waits on it instead of synchronising the stream
    unsigned long long* done;
    unsigned long long epoch;
    FoldPush fp;  // folded exchange: the last arriver pushes the group value (K == 1)
    // collect: segment partials as flagged words, stage 2 by each group's last-dispatched workgroup
    unsigned long long* ll;  // [LBK_KMAX][LBK_SEGS][2] flagged partials, or nullptr (other modes)
    unsigned seq;            // this launch's tag
    unsigned* err;           // pinned: set on a timeout
    unsigned long long timeout;
};

// Streaming loads/stores; NT = non-temporal (the vectors are touched once per pass and, at
// the benchmark sizes, are far larger than the 256 MiB Infinity Cache): +6 % on the 3-read /
// 1-write pass mix on MI355X (profiles/r01/bwprobe_v2.txt).
typedef double dvec2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ double2 ldv(const double* p) {
    if (NT) {
        const dvec2 v = __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(p));
        return make_double2(v.x, v.y);
    }
    return *reinterpret_cast<const double2*>(p);
}
template <bool NT>
__device__ __forceinline__ void stv(double* p, double2 v) {
    if (NT) {
        dvec2 w;
        w.x = v.x;
        w.y = v.y;
        __builtin_nontemporal_store(w, reinterpret_cast<dvec2*>(p));
    } else {
        *reinterpret_cast<double2*>(p) = v;
    }
}
__device__ __forceinline__ void st2m(double* p, double2 v, bool v0, bool v1) {
    if (v1) {
        *reinterpret_cast<double2*>(p) = v;
    } else if (v0) {
        p[0] = v.x;
    }
}

// Work vectors (q / r / d: rewritten pass after pass, read again by the next) may keep the
// temporal policy under NT so that, at per-rank sizes a few times below the Infinity Cache, they
// stay resident while the history streams past (A/B variant: LBK_WORK_TEMPORAL).
#ifndef LBK_WORK_TEMPORAL
#define LBK_WORK_TEMPORAL 1
#endif
// A/B levels: 0 all NT; 1 q/r/d temporal; 2 + x, g; 3 + new s, y; 4 / 5 q/r/d loads / stores only
#define LBK_WLD_T (LBK_WORK_TEMPORAL >= 1 && LBK_WORK_TEMPORAL <= 4)
#define LBK_WST_T (LBK_WORK_TEMPORAL >= 1 && LBK_WORK_TEMPORAL != 4)
#define LBK_XG_T (LBK_WORK_TEMPORAL == 2 || LBK_WORK_TEMPORAL == 3)
#define LBK_SY_T (LBK_WORK_TEMPORAL == 3)
template <bool NT>
__device__ __forceinline__ double2 ldw(const double* p) {
    return ldv<NT && !LBK_WLD_T>(p);
}
// level 2: the iterate and gradient (x, g; read by the trials, the last second-loop pass and
// the commit) as well
template <bool NT>
__device__ __forceinline__ double2 ldx(const double* p) {
    return ldv<NT && !LBK_XG_T>(p);
}

// fixed-order total of the 8 group partials of one slot component
__device__ __forceinline__ double slot_total(const double* p) {
    double t = p[0];
#pragma unroll
    for (int g = 1; g < LBK_GROUPS; ++g) t = t + p[g * LBK_KMAX];
    return t;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = v + __shfl_xor(v, m, 64);
    return v;
}

__device__ __forceinline__ unsigned long long dbits(double v) {
    return (unsigned long long)__double_as_longlong(v);
}
__device__ __forceinline__ double bitsd(unsigned long long u) {
    return __longlong_as_double((long long)u);
}

// Flagged partials of the cooperative iteration ("LL" words): a double travels as two 64-bit
// words, each half tagged with the pass's sequence number in its upper 32 bits. Every 64-bit
// store is single-copy atomic, so a reader that sees both tags has both halves: no separate
// arrival counter, no drain between the data and the flag. Agent-scope (sc1) stores and loads,
// coherent across the XCDs' L2s.
#define LBK_LL_SEGS 8192  // >= LBK_COOP_SEGMAX; every segment for the persistent iteration (LBFGS_PERSIST)
#define LBK_LL_COMPS 10   // up to 8 reduction components + the 2 edge values of an r pass
__device__ __forceinline__ void ll_store(unsigned long long* p, double v, unsigned seq) {
    const unsigned long long u = dbits(v), tag = (unsigned long long)seq << 32;
    __hip_atomic_store(p, tag | (u & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p + 1, tag | (u >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// spins until both halves carry `seq`; past `timeout` wall-clock ticks sets *err and returns NaN.
// Once a wait has lasted 1/1024 of the timeout it also ends (NaN) as soon as *err shows that another
// workgroup's wait already timed out: a launch whose grid broke apart drains in about one timeout,
// not one per remaining barrier. `failed` is set whenever NaN comes from either exit.
__device__ __forceinline__ double ll_load(const unsigned long long* p, unsigned seq, unsigned* err,
                                          unsigned long long timeout, bool& failed) {
    unsigned long long w0 = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long w1 = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(w0 >> 32) != seq || (unsigned)(w1 >> 32) != seq) {
        const unsigned long long t0 = wall_clock64();
        for (;;) {
            __builtin_amdgcn_s_sleep(1);
            w0 = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            w1 = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned)(w0 >> 32) == seq && (unsigned)(w1 >> 32) == seq) break;
            const unsigned long long el = wall_clock64() - t0;
            if (el > timeout) {
                if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                failed = true;
                return __builtin_nan("");
            }
            if (err && el > (timeout >> 10) && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
                failed = true;
                return __builtin_nan("");
            }
        }
    }
    return bitsd((w1 << 32) | (w0 & 0xffffffffull));
}
__device__ __forceinline__ double ll_load(const unsigned long long* p, unsigned seq, unsigned* err,
                                          unsigned long long timeout) {
    bool failed = false;
    return ll_load(p, seq, err, timeout, failed);
}

// Per-workgroup view of its segment.
struct Seg {
    int64_t sbeg;   // global index of segment start
    int64_t lb;     // local index of segment start
    int64_t len;    // valid elements in this segment
    int nrows;      // rows (of 128) this wave visits
    int lane, w;
};

// this workgroup's segment, relative to the rank's first: launch order or reversed
__device__ __forceinline__ int64_t seg_block(const Geo& geo) {
    return geo.rev ? (int64_t)gridDim.x - 1 - blockIdx.x : (int64_t)blockIdx.x;
}

__device__ __forceinline__ Seg seg_setup(const Geo& geo) {
    Seg s;
    const int64_t sg = geo.seg_lo + seg_block(geo);
    s.sbeg = sg * geo.L;
    const int64_t send = min(s.sbeg + geo.L, geo.n);
    s.len = send - s.sbeg;
    s.lb = s.sbeg - geo.elem_lo;
    s.lane = threadIdx.x & 63;
    s.w = threadIdx.x >> 6;
    const int nrow_tot = (int)((s.len + 127) / 128);
    s.nrows = nrow_tot > s.w ? (nrow_tot - s.w + 3) / 4 : 0;
    return s;
}

// Offset (within the segment) of this lane's first element in row u of its wave.
__device__ __forceinline__ int64_t row_off(const Seg& s, int u) {
    return (int64_t)(4 * u + s.w) * 128 + 2 * s.lane;
}

// Stage 2 of the canonical order for group g: balanced tree over its 1024 segment partials
// (0.0 beyond nseg) = per thread ((p0 + p1) + (p2 + p3)) over 4 consecutive segments, wave
// butterfly, ((w0 + w1) + (w2 + w3)). ATOMIC: the partials are read with agent-scope (sc1)
// loads inside the producing launch (ticket mode); otherwise plain loads after a kernel
// boundary (reduce-kernel mode).
template <int K, bool ATOMIC>
__device__ __forceinline__ void group_tree(const double* partials, int64_t lbase, int64_t gseg0, int64_t nseg,
                                           int spg, double* slot_g, double* hslot_g,
                                           double (&lds)[4][K > 0 ? K : 1]) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // Few valid partials (a group of at most 64 segments: n up to ~6e4, or the tail group): wave w
    // takes components w, w + 4, ..., lane j entry j, every load in one round trip. The wave
    // butterfly is the balanced tree over entries 0..63; the tree's upper levels only add
    // 0.0 subtrees, which is the final "+ 0.0" (bit-identical to the general path below).
    const int64_t nvalid = min((int64_t)spg, nseg - gseg0);
    if (nvalid <= 64) {
        constexpr int KQ = (K + 3) / 4;
        double p[KQ];
#pragma unroll
        for (int i = 0; i < KQ; ++i) {
            const int k = w + 4 * i;
            p[i] = 0.0;
            if (k < K && lane < nvalid) {
                const double* src = partials + (int64_t)k * LBK_SEGS + lbase + lane;
                p[i] = ATOMIC ? bitsd(__hip_atomic_load(reinterpret_cast<const unsigned long long*>(src),
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                              : *src;
            }
        }
#pragma unroll
        for (int i = 0; i < KQ; ++i) {
            const int k = w + 4 * i;
            const double v = wave_sum(p[i]) + 0.0;
            if (k < K && lane == 0) {
                slot_g[k] = v;
                if (hslot_g) hslot_g[k] = v;
            }
        }
        return;
    }
    double q[K];
    // components in chunks of 8 with every load of a chunk issued before the first butterfly:
    // the relaxed atomic loads of the ticket path are not batched by the compiler, and one L2
    // round trip per component cost ~0.7 us each (27.6 us for a 27-component vector-free
    // commit at n = 1e4)
    constexpr int KC = 8;
#pragma unroll
    for (int k0 = 0; k0 < K; k0 += KC) {
        double p[KC][4];
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            if (k0 + kc >= K) break;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t j = 4 * t + i;
                const double* src = partials + (int64_t)(k0 + kc) * LBK_SEGS + lbase + j;
                if (j < spg && gseg0 + j < nseg)
                    p[kc][i] = ATOMIC ? bitsd(__hip_atomic_load(reinterpret_cast<const unsigned long long*>(src),
                                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                                      : *src;
                else
                    p[kc][i] = 0.0;
            }
        }
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            if (k0 + kc >= K) break;
            q[k0 + kc] = wave_sum((p[kc][0] + p[kc][1]) + (p[kc][2] + p[kc][3]));
        }
    }
    __syncthreads();  // lds reuse
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) lds[w][k] = q[k];
    }
    __syncthreads();
    if (t == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double v = (lds[0][k] + lds[1][k]) + (lds[2][k] + lds[3][k]);
            slot_g[k] = v;
            if (hslot_g) hslot_g[k] = v;
        }
    }
}

// Collect mode's stage 2 of group g inside the producing launch: group_tree's arithmetic exactly
// (the same two shapes: <= 64 valid partials, or 4 per thread + butterflies + the wave pairs),
// with the partials read as flagged words (ll_store, tag = the launch's sequence number) that
// every workgroup of the group stored without waiting. Each batch of words is issued at once and
// polled until every tag matches; a wait past `timeout` sets *err and gives NaN.
template <int M>
__device__ __forceinline__ void ll_load_batch(const unsigned long long* const (&p)[M], const bool (&on)[M],
                                              unsigned seq, double (&out)[M], unsigned* err,
                                              unsigned long long timeout) {
    unsigned long long w0[M], w1[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        w0[m] = on[m] ? __hip_atomic_load(p[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        w1[m] = on[m] ? __hip_atomic_load(p[m] + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    }
    unsigned long long t0 = 0;
    for (;;) {
        bool all = true;
#pragma unroll
        for (int m = 0; m < M; ++m)
            if (on[m] && ((unsigned)(w0[m] >> 32) != seq || (unsigned)(w1[m] >> 32) != seq)) all = false;
        if (all) break;
        if (t0 == 0) t0 = wall_clock64();
        if (wall_clock64() - t0 > timeout) {
            if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
            for (int m = 0; m < M; ++m) out[m] = __builtin_nan("");
            return;
        }
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int m = 0; m < M; ++m) {
            if (on[m] && (unsigned)(w0[m] >> 32) != seq)
                w0[m] = __hip_atomic_load(p[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (on[m] && (unsigned)(w1[m] >> 32) != seq)
                w1[m] = __hip_atomic_load(p[m] + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) out[m] = on[m] ? bitsd((w1[m] << 32) | (w0[m] & 0xffffffffull)) : 0.0;
}

template <int K>
__device__ __forceinline__ void collect_tree(const Red& red, int64_t lbase, int64_t gseg0, int64_t nseg, int spg,
                                             double* slot_g, double* hslot_g, double (&lds)[4][K > 0 ? K : 1]) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    auto word = [&](int k, int64_t j) { return red.ll + ((int64_t)k * LBK_SEGS + lbase + j) * 2; };
    const int64_t nvalid = min((int64_t)spg, nseg - gseg0);
    if (nvalid <= 64) {  // group_tree's short shape
        constexpr int KQ = (K + 3) / 4;
        const unsigned long long* pp[KQ];
        bool on[KQ];
        double p[KQ];
#pragma unroll
        for (int i = 0; i < KQ; ++i) {
            const int k = w + 4 * i;
            on[i] = k < K && lane < nvalid;
            pp[i] = on[i] ? word(k, lane) : red.ll;
        }
        ll_load_batch<KQ>(pp, on, red.seq, p, red.err, red.timeout);
#pragma unroll
        for (int i = 0; i < KQ; ++i) {
            const int k = w + 4 * i;
            const double v = wave_sum(p[i]) + 0.0;
            if (k < K && lane == 0) {
                slot_g[k] = v;
                if (hslot_g) hslot_g[k] = v;
            }
        }
        return;
    }
    double q[K];
    constexpr int KC = 2;  // components per batch of polled words (4 words... 8 per component)
#pragma unroll
    for (int k0 = 0; k0 < K; k0 += KC) {
        const unsigned long long* pp[KC * 4];
        bool on[KC * 4];
        double p[KC * 4];
#pragma unroll
        for (int kc = 0; kc < KC; ++kc)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t j = 4 * t + i;
                on[kc * 4 + i] = k0 + kc < K && j < spg && gseg0 + j < nseg;
                pp[kc * 4 + i] = on[kc * 4 + i] ? word(k0 + kc, j) : red.ll;
            }
        ll_load_batch<KC * 4>(pp, on, red.seq, p, red.err, red.timeout);
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            if (k0 + kc >= K) break;
            q[k0 + kc] = wave_sum((p[kc * 4] + p[kc * 4 + 1]) + (p[kc * 4 + 2] + p[kc * 4 + 3]));
        }
    }
    __syncthreads();  // lds reuse
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) lds[w][k] = q[k];
    }
    __syncthreads();
    if (t == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double v = (lds[0][k] + lds[1][k]) + (lds[2][k] + lds[3][k]);
            slot_g[k] = v;
            if (hslot_g) hslot_g[k] = v;
        }
    }
}

// Segment partial (wave butterflies, ((w0 + w1) + (w2 + w3))), then either
//   red.ticket : write-through store + per-group agent-scope ticket; the last-arriving
//                workgroup of the group runs stage 2 (one launch; used for small grids), or
//   otherwise  : a plain store; k_group_reduce runs stage 2 after the kernel boundary. The
//                ticket's vmcnt(0) has to wait for all the wave's outstanding row stores, which
//                costs ~2x on short segments (n = 1e7: 3.0 vs 4.7+ TB/s, profiles/r01).
// Both give the same bits.
template <int K, bool FOLD = false>
__device__ __forceinline__ void reduce_publish(double (&acc)[K], const Geo& geo, const Red& red) {
    __shared__ double lds[4][K];
    __shared__ int last_flag;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = wave_sum(acc[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) lds[w][k] = acc[k];
    }
    __syncthreads();
    const int64_t b = seg_block(geo);
    const int64_t sg = geo.seg_lo + b;
    const int g = (int)(sg / geo.spg);
    // (compiled for regular slots only: the code would cost the wide-slot vector-free commit a
    // wave per SIMD of registers)
    if constexpr (K <= LBK_KMAX) {
    if (red.ll) {
        // collect: the partial as flagged words, no wait; one workgroup per group - the one on
        // the group's last segment in walk order (highest block index of the group: its last
        // segment, or its first when the walk is reversed) - forms the group tree from them.
        // Forward progress does not rest on dispatch order (on a multi-XCD part workgroups go
        // round-robin over the XCDs, so there is none across the grid): a launch has at most
        // LBK_GROUPS = 8 waiting collectors and every other workgroup is wait-free, so the
        // producers always find CUs and every wait ends. On a GPU time-shared with other work the
        // wait is bounded by the collect timeout (LBFGS_COLLECT_TIMEOUT, 10 s), then NaN + error.
        if (t == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                ll_store(red.ll + ((int64_t)k * LBK_SEGS + b) * 2, (lds[0][k] + lds[1][k]) + (lds[2][k] + lds[3][k]),
                         red.seq);
        }
        const int64_t gseg0 = (int64_t)g * geo.spg;
        const int64_t glast = min(geo.nseg, gseg0 + geo.spg) - 1;
        if (sg != (geo.rev ? gseg0 : glast)) return;  // uniform over the workgroup
        collect_tree<K>(red, gseg0 - geo.seg_lo, gseg0, geo.nseg, geo.spg, red.slot + g * red.kstride,
                        red.hslot ? red.hslot + g * red.kstride : nullptr, lds);
        return;
    }
    }
    if (!red.ticket) {
        if (t == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                red.partials[(int64_t)k * LBK_SEGS + b] = (lds[0][k] + lds[1][k]) + (lds[2][k] + lds[3][k]);
        }
        return;
    }
    if (t == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double p = (lds[0][k] + lds[1][k]) + (lds[2][k] + lds[3][k]);
            // write-through (sc1) store: visible to the last arriver's sc1 loads
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(red.partials + (int64_t)k * LBK_SEGS + b),
                               dbits(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int64_t hi = min(geo.nseg, (int64_t)(g + 1) * geo.spg);
        const unsigned expect = (unsigned)(hi - (int64_t)g * geo.spg);
        const unsigned old = __hip_atomic_fetch_add(red.cnt + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_flag = (old + 1u == expect);
    }
    __syncthreads();
    if (!last_flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t gseg0 = (int64_t)g * geo.spg;
    group_tree<K, true>(red.partials, gseg0 - geo.seg_lo, gseg0, geo.nseg, geo.spg, red.slot + g * red.kstride,
                        red.hslot ? red.hslot + g * red.kstride : nullptr, lds);
    // folded exchange: thread 0 stored the group value (K == 1) itself; it goes to every peer now
    if (FOLD && K == 1 && red.fp.peers && t == 0) fold_push(red.fp, g * red.kstride, red.slot[g * red.kstride]);
    if (t == 0) __hip_atomic_store(red.cnt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (red.done) {  // every wave's mirror stores complete before the word
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (t == 0) __hip_atomic_store(red.done, red.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Reduce-kernel mode: one workgroup per group of this rank (stage 2 after the boundary).
template <int K>
__global__ __launch_bounds__(LB_BLOCK) void k_group_reduce(const double* __restrict__ partials, Geo geo,
                                                           double* __restrict__ slot, double* hslot, int kstride,
                                                           FoldPush fp) {
    __shared__ double lds[4][K];
    const int g = geo.g_lo + (int)blockIdx.x;
    const int64_t gseg0 = (int64_t)g * geo.spg;
    group_tree<K, false>(partials, gseg0 - geo.seg_lo, gseg0, geo.nseg, geo.spg, slot + g * kstride,
                         hslot ? hslot + g * kstride : nullptr, lds);
    if (K == 1 && fp.peers && threadIdx.x == 0) fold_push(fp, g * kstride, slot[g * kstride]);
}

// The same stage 2 for a runtime number of components (wide slots): blockIdx.y takes
// components [8 y, 8 y + 8), all their partial loads issued before the first butterfly;
// identical arithmetic per component as group_tree.
__global__ __launch_bounds__(LB_BLOCK) void k_group_reduce_wide(const double* __restrict__ partials, Geo geo,
                                                                double* __restrict__ slot, double* hslot, int K,
                                                                int kstride) {
    constexpr int KC = 8;
    __shared__ double lds[4][KC];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int g = geo.g_lo + (int)blockIdx.x;
    const int k0 = KC * (int)blockIdx.y;
    const int64_t gseg0 = (int64_t)g * geo.spg;
    const int64_t lbase = gseg0 - geo.seg_lo;
    double p[KC][4];
#pragma unroll
    for (int c = 0; c < KC; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t j = 4 * t + i;
            p[c][i] = (k0 + c < K && j < geo.spg && gseg0 + j < geo.nseg) ? partials[(int64_t)(k0 + c) * LBK_SEGS + lbase + j] : 0.0;
        }
#pragma unroll
    for (int c = 0; c < KC; ++c) {
        const double q = wave_sum((p[c][0] + p[c][1]) + (p[c][2] + p[c][3]));
        if (lane == 0) lds[w][c] = q;
    }
    __syncthreads();
    if (t < KC && k0 + t < K) {
        const double v = (lds[0][t] + lds[1][t]) + (lds[2][t] + lds[3][t]);
        slot[g * kstride + k0 + t] = v;
        if (hslot) hslot[g * kstride + k0 + t] = v;
    }
}

// A wait on a peer's mailbox word ends past `timeout` wall-clock ticks, or - once it has waited
// 1/65536 of that (~1 ms of the default 60 s) - as soon as the error flag's device copy shows that
// an earlier wait of this rank already timed out: a broken channel costs one timeout per solve, not
// one per exchange queued before the host's next synchronisation.
__device__ __forceinline__ bool peer_wait_over(unsigned long long t0, unsigned long long timeout, const unsigned* errd) {
    const unsigned long long el = wall_clock64() - t0;
    if (el > timeout) return true;
    return el > (timeout >> 16) && __hip_atomic_load(errd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

// Total of a launch's first source slot (the previous pass's reduction). Normally stage 2 ran
// after the producer (k_group_reduce or tickets) and the slot holds the group values. With a
// deferred stage 2 (geo.ppart, mid n on one rank) every workgroup of the consuming launch forms
// the group trees from the producer's partials itself - the same trees, so the same bits - and
// workgroup 0 stores the group values into the slot for later readers. One kernel boundary and
// the stage-2 launch per pass disappear; the price is each workgroup reading <= 2048 partials.
// Folded exchange, consumer side: the rank's own groups from the slot (its producer's stage 2,
// before this launch's boundary), every other group's value from the mailbox once both words carry
// the exchange's epoch (a wait past the timeout sets *merr and gives NaN, as the exchange kernel);
// workgroup 0 completes the slot for later readers. Same eight values, same fixed-order sum.
__device__ __forceinline__ double src_total_mailbox(const double* slot, const Geo& geo, const FoldSrc& fs) {
    __shared__ double gv[LBK_GROUPS];
    const int t = threadIdx.x;
    const unsigned long long w0 = (fs.wait && blockIdx.x == 0 && t == 0) ? wall_clock64() : 0ull;
    if (t < LBK_GROUPS) {
        double v;
        if (t >= geo.g_lo && t < geo.g_hi) {
            v = slot[t * LBK_KMAX];
        } else {
            const unsigned long long* p = fs.mbx + 2 * (size_t)(t * LBK_KMAX);
            unsigned long long a, b;
            const unsigned long long t0 = wall_clock64();
            for (;;) {
                a = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                b = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if ((unsigned)(a >> 32) == fs.mepoch && (unsigned)(b >> 32) == fs.mepoch) break;
                if (peer_wait_over(t0, fs.mtmo, fs.merrd)) {
                    __hip_atomic_store(fs.merrd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(fs.merr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    a = 0;
                    b = 0x7ff80000ull;  // quiet NaN
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            v = bitsd((a & 0xffffffffull) | ((b & 0xffffffffull) << 32));
            if (blockIdx.x == 0) const_cast<double*>(slot)[t * LBK_KMAX] = v;
        }
        gv[t] = v;
    }
    __syncthreads();
    // the time this launch's first workgroup spent waiting for the peers' values (exchange_share)
    if (fs.wait && blockIdx.x == 0 && t == 0)
        __hip_atomic_fetch_add(fs.wait, wall_clock64() - w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    double tt = gv[0];
#pragma unroll
    for (int g = 1; g < LBK_GROUPS; ++g) tt = tt + gv[g];
    return tt;
}

__device__ __forceinline__ double src_total(const double* slot, const Geo& geo) {
    if (!geo.ppart) return slot_total(slot);
    __shared__ double gv[LBK_GROUPS];
    __shared__ double ldt[4][1];
    const int ng = (int)((geo.nseg + LBK_SEG_PER_GROUP - 1) / LBK_SEG_PER_GROUP);
    // one group tree per group with segments (group_tree's registers only: a form that loads every
    // group at once raised the pass kernels from 68-70 to 74-80 VGPRs, one wave per SIMD fewer, and
    // ran slower); groups without a segment are the slot's 0.0
    if (threadIdx.x < LBK_GROUPS) gv[threadIdx.x] = 0.0;
    __syncthreads();
    for (int g = 0; g < ng; ++g) {
        group_tree<1, false>(geo.ppart, (int64_t)g * LBK_SEG_PER_GROUP, (int64_t)g * LBK_SEG_PER_GROUP, geo.nseg,
                             LBK_SEG_PER_GROUP, &gv[g], nullptr, ldt);
        __syncthreads();
    }
    if (blockIdx.x == 0 && threadIdx.x < ng) const_cast<double*>(slot)[threadIdx.x * LBK_KMAX] = gv[threadIdx.x];
    double t = gv[0];
#pragma unroll
    for (int g = 1; g < LBK_GROUPS; ++g) t = t + gv[g];
    return t;
}

// ---------------------------------------------------------------------------------------
// Objectives (benchmark.cpp:58-81, :16-56; main.cpp:7-21), per element e with neighbours.
// ---------------------------------------------------------------------------------------
template <int OBJ>
__device__ __forceinline__ double obj_term(double zc, double zp, bool has_p) {
    if (OBJ == LBK_OBJ_ROSENBROCK) {
        const double term1 = zp - zc * zc;
        const double term2 = 1.0 - zc;
        return 100.0 * term1 * term1 + term2 * term2;  // valid only when has_p
    } else if (OBJ == LBK_OBJ_QUAD_TRIDIAG) {
        const double dterm = 1000.0 * zc * zc;
        return has_p ? dterm + 100.0 * zc * zp : dterm;
    } else {
        return (zc - 1.0) * (zc - 1.0);
    }
}
// does element e contribute an f term?
template <int OBJ>
__device__ __forceinline__ bool obj_has_term(bool has_p) {
    return OBJ == LBK_OBJ_ROSENBROCK ? has_p : true;
}

template <int OBJ>
__device__ __forceinline__ double obj_grad(double zm, double zc, double zp, bool has_m, bool has_p) {
    if (OBJ == LBK_OBJ_ROSENBROCK) {
        double g = 0.0;
        if (has_m) g = g + 200.0 * (zc - zm * zm);  // grad[i+1] += 200 term2 (first)
        if (has_p) {
            const double term1 = 2.0 * (zc - 1.0);
            const double term2 = zp - zc * zc;
            g = g + (term1 - 400.0 * zc * term2);    // grad[i] += term1 - 400 x term2
        }
        return g;
    } else if (OBJ == LBK_OBJ_QUAD_TRIDIAG) {
        double g = 2000.0 * zc;
        if (has_m) g = g + 100.0 * zm;
        if (has_p) g = g + 100.0 * zp;
        return g;
    } else {
        return 2.0 * (zc - 1.0);
    }
}

// Neighbour exchange inside a row: lane l holds z[2l], z[2l+1]; the halo value zh is
// z[-1] on lane 0 and z[128] on lane 63. Returned by value (selects): a by-reference form
// made hipcc place both outputs in scratch and pick one with a dynamic store.
struct Nb {
    double l, r;
};
__device__ __forceinline__ Nb neighbours(double z0, double z1, double zh, int lane) {
    Nb nb;
    const double up = __shfl_up(z1, 1, 64);
    const double dn = __shfl_down(z0, 1, 64);
    nb.l = (lane == 0) ? zh : up;
    nb.r = (lane == 63) ? zh : dn;
    return nb;
}

// ---------------------------------------------------------------------------------------
// Streaming framework. A kernel is a policy Op with
//   typename Op::Row                      registers of one row (128 elements) of this lane
//   op.load(Row&, int64_t i)              issue the loads of local elements i, i+1 (+ halo)
//   op.apply<MASK>(Row&, i, e0, v0, v1, acc)  compute, store, accumulate (elements < len)
// and every kernel walks its segment as: full segments (all but the last) in groups of
// 4 / 2 / 1 rows with every load of a group issued before any use and no element masks;
// the last, partial segment row by row with masks. The accumulation order (row u
// ascending, v = 0 then 1) is the canonical one in both paths.
// ---------------------------------------------------------------------------------------
template <bool MASK, int UN, int K, class Op>
__device__ __forceinline__ void rows(const Op& op, const Seg& s, int u0, double (&acc)[K]) {
    typename Op::Row r[UN];
#pragma unroll
    for (int j = 0; j < UN; ++j) op.load(r[j], s.lb + row_off(s, u0 + j));
#pragma unroll
    for (int j = 0; j < UN; ++j) {
        const int64_t o = row_off(s, u0 + j);
        const bool v0 = MASK ? o < s.len : true;
        const bool v1 = MASK ? o + 1 < s.len : true;
        op.template apply<MASK>(r[j], s.lb + o, s.sbeg + o, v0, v1, acc);
    }
}

// Software-pipelined full-segment walk: the loads of row group k+1 are issued before group k is
// computed and stored. The in-place passes (q, r) carry no __restrict__ between input and output,
// so the compiler cannot hoist the next group's loads above this group's stores by itself.
template <int UN, int K, class Op>
__device__ __forceinline__ void load_group(const Op& op, const Seg& s, int u0, typename Op::Row (&r)[UN]) {
#pragma unroll
    for (int j = 0; j < UN; ++j) op.load(r[j], s.lb + row_off(s, u0 + j));
}
template <int UN, int K, class Op>
__device__ __forceinline__ void apply_group(const Op& op, const Seg& s, int u0, typename Op::Row (&r)[UN],
                                            double (&acc)[K]) {
#pragma unroll
    for (int j = 0; j < UN; ++j) {
        const int64_t o = row_off(s, u0 + j);
        op.template apply<false>(r[j], s.lb + o, s.sbeg + o, true, true, acc);
    }
}

template <int K, class Op>
__device__ __forceinline__ void stream_pipelined(const Op& op, const Seg& s, double (&acc)[K]) {
    constexpr int G = 2;  // rows per group
    int u0 = 0;
    if (s.nrows >= 2 * G) {
        typename Op::Row a[G], b[G];
        load_group<G, K>(op, s, 0, a);
        for (;;) {
            const bool more_b = u0 + 2 * G <= s.nrows;
            if (more_b) load_group<G, K>(op, s, u0 + G, b);
            apply_group<G, K>(op, s, u0, a, acc);
            u0 += G;
            if (!more_b) break;
            const bool more_a = u0 + 2 * G <= s.nrows;
            if (more_a) load_group<G, K>(op, s, u0 + G, a);
            apply_group<G, K>(op, s, u0, b, acc);
            u0 += G;
            if (!more_a) break;
        }
    }
    for (; u0 < s.nrows; ++u0) rows<false, 1>(op, s, u0, acc);
}

#ifndef LBK_PIPELINE
#define LBK_PIPELINE 0
#endif

// Rows per load group on full segments. A pass with few load streams per row (k_mid: q and y0)
// keeps fewer bytes in flight per wave at 4 rows; op_unroll widens its groups. The groups only
// decide when loads are issued: rows are still applied, and accumulated, in ascending order, so
// every unroll gives the same bits.
#ifndef LBK_MID_UNROLL
#define LBK_MID_UNROLL 8
#endif
template <class Op>
struct op_unroll {
    static constexpr int value = 4;
};
template <bool NT>
struct OpMid;
template <bool NT>
struct op_unroll<OpMid<NT>> {
    static constexpr int value = LBK_MID_UNROLL;
};

template <int K, class Op>
__device__ __forceinline__ void stream(const Op& op, const Seg& s, const Geo& geo, double (&acc)[K], int u0 = 0) {
    if (LBK_PIPELINE && s.len == geo.L && u0 == 0) {
        stream_pipelined(op, s, acc);
        return;
    }
    if (s.len == geo.L) {
        constexpr int U = op_unroll<Op>::value;
        if constexpr (U > 4)
            for (; u0 + U <= s.nrows; u0 += U) rows<false, U>(op, s, u0, acc);
        for (; u0 + 4 <= s.nrows; u0 += 4) rows<false, 4>(op, s, u0, acc);
        if (u0 + 2 <= s.nrows) {
            rows<false, 2>(op, s, u0, acc);
            u0 += 2;
        }
        if (u0 < s.nrows) rows<false, 1>(op, s, u0, acc);
    } else {
        for (; u0 < s.nrows; ++u0) rows<true, 1>(op, s, u0, acc);
    }
}

// Stencil passes (the commit and the trials of the Rosenbrock / tridiagonal objectives need z
// at each row's outer neighbours): over a full segment the waves step through 16 rows at a time
// - wave w takes rows 16k + 4j + w, j = 0..3, which is the canonical visiting order (u = 4k + j)
// - and publish the (x, d) of their rows' first and last elements in LDS, so a row's halo comes
// from the neighbouring wave's registers instead of a second read of x and d (4.23 -> ~4.0
// vector reads per commit launch at n = 1e8). Only the segment's first row's left halo and each
// step's last row's right halo are read from memory. One barrier per step; the LDS edge table is
// double-buffered and the previous step's carry is read before the barrier, so a wave running a
// step ahead never overwrites what a slower one still reads.
template <int K, class Op>
__device__ __forceinline__ void stream_stencil(const Op& op, const Seg& s, double (&acc)[K]) {
    __shared__ double2 E[2][16][2];
    const int nrow = (int)(s.len >> 7);  // full segment: a whole number of rows
    const int nsteps = (nrow + 15) >> 4;
    const bool l0 = s.lane == 0, l63 = s.lane == 63;
    for (int k = 0; k < nsteps; ++k) {
        const int buf = k & 1;
        typename Op::Row r[4];
        double2 hmem[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 16 * k + 4 * j + s.w;
            if (row < nrow) {
                const int64_t i = s.lb + (int64_t)row * 128 + 2 * s.lane;
                op.load_core(r[j], i);
                // memory halos: the segment's first row (left), a step's last row (right)
                hmem[j] = make_double2(0.0, 0.0);
                if (l0 && row == 0) hmem[j] = op.halo_mem(i - 1);
                if (l63 && (4 * j + s.w == 15 || row + 1 == nrow)) hmem[j] = op.halo_mem(i + 2);
            }
        }
        double2 carry = make_double2(0.0, 0.0);
        if (k > 0 && s.w == 0 && l0) carry = E[buf ^ 1][15][1];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 16 * k + 4 * j + s.w;
            if (row < nrow) {
                if (l0) E[buf][4 * j + s.w][0] = op.edge_first(r[j]);
                if (l63) E[buf][4 * j + s.w][1] = op.edge_last(r[j]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int rr = 4 * j + s.w, row = 16 * k + rr;
            if (row < nrow) {
                double2 h = hmem[j];
                if (l0 && row > 0) h = rr > 0 ? E[buf][rr - 1][1] : carry;
                if (l63 && rr < 15 && row + 1 < nrow) h = E[buf][rr + 1][0];
                op.set_halo(r[j], h);
                const int64_t o = (int64_t)row * 128 + 2 * s.lane;
                op.template apply<false>(r[j], s.lb + o, s.sbeg + o, true, true, acc);
            }
        }
    }
}

#ifndef LBK_LDS_HALO
#define LBK_LDS_HALO 1
#endif

// stencil ops over full segments exchange row halos through LDS; everything else streams
template <int K, class Op>
__device__ __forceinline__ void stream_halo(const Op& op, const Seg& s, const Geo& geo, double (&acc)[K]) {
    if constexpr (LBK_LDS_HALO && Op::kStencil) {
        if (s.len == geo.L) {
            stream_stencil(op, s, acc);
            return;
        }
    }
    stream(op, s, geo, acc);
}

template <bool MASK, bool NT>
__device__ __forceinline__ void st2(double* p, double2 v, bool v0, bool v1) {
    if (!MASK || (v0 && v1))
        stv<NT>(p, v);
    else
        st2m(p, v, v0, v1);
}

// acc = fma(a, b, acc) for the valid elements of a lane pair
template <bool MASK, bool NT>
__device__ __forceinline__ void st2w(double* p, double2 v, bool v0, bool v1) {
    st2<MASK, NT && !LBK_WST_T>(p, v, v0, v1);
}

template <bool MASK, bool NT>
__device__ __forceinline__ void st2x(double* p, double2 v, bool v0, bool v1) {
    st2<MASK, NT && !LBK_XG_T>(p, v, v0, v1);
}
// level 3: the new history pair (s, y: the next two-loop's first reads)
template <bool MASK, bool NT>
__device__ __forceinline__ void st2h(double* p, double2 v, bool v0, bool v1) {
    st2<MASK, NT && !LBK_SY_T>(p, v, v0, v1);
}

template <bool MASK>
__device__ __forceinline__ double fma2(double2 a, double2 b, double acc, bool v0, bool v1) {
    if (!MASK || v0) acc = fma(a.x, b.x, acc);
    if (!MASK || v1) acc = fma(a.y, b.y, acc);
    return acc;
}

// ---------------------------------------------------------------------------------------
// Two-loop recursion passes
// ---------------------------------------------------------------------------------------
template <bool NT>
struct OpDot {  // acc += a . b
    const double* __restrict__ a;
    const double* __restrict__ b;
    struct Row {
        double2 a, b;
    };
    __device__ void load(Row& r, int64_t i) const {
        r.a = ldv<NT>(a + i);
        r.b = ldv<NT>(b + i);
    }
    template <bool MASK>
    __device__ void apply(Row& r, int64_t, int64_t, bool v0, bool v1, double (&acc)[1]) const {
        acc[0] = fma2<MASK>(r.a, r.b, acc[0], v0, v1);
    }
};

template <bool NT>
struct OpAxpyDot {  // q = qin - alpha y;  acc += s . q       (lbfgs.cpp:133-137)
    double* qout;
    const double* qin;
    const double* __restrict__ y;
    const double* __restrict__ s;
    double alpha;
    __device__ void set_coef(double a) { alpha = a; }
    struct Row {
        double2 q, y, s;
    };
    __device__ void load(Row& r, int64_t i) const {
        r.q = ldw<NT>(qin + i);
        r.y = ldv<NT>(y + i);
        r.s = ldv<NT>(s + i);
    }
    template <bool MASK>
    __device__ void apply(Row& r, int64_t i, int64_t, bool v0, bool v1, double (&acc)[1]) const {
        double2 qn;
        qn.x = r.q.x - alpha * r.y.x;
        qn.y = r.q.y - alpha * r.y.y;
        st2w<MASK, NT>(qout + i, qn, v0, v1);
        acc[0] = fma2<MASK>(r.s, qn, acc[0], v0, v1);
    }
};

// Sharded runs: the rank's first and last value of a pass's output vector (d, or the r of the
// last second-loop pass) are written into spare components of the pass's result slot (group
// g_lo comp 1, group g_hi-1 comp 2), which the slot exchange delivers to the neighbouring
// ranks as their halo.
__device__ __forceinline__ void publish_edges(double* edge_slot, int64_t i, int64_t n_loc, int g_lo, int g_hi,
                                              double2 d, bool v0, bool v1) {
    if (!edge_slot) return;
    if (i == 0 && v0) edge_slot[g_lo * LBK_KMAX + 1] = d.x;
    if (i + 1 == n_loc - 1 && v1) edge_slot[(g_hi - 1) * LBK_KMAX + 2] = d.y;
    if (i == n_loc - 1 && v0) edge_slot[(g_hi - 1) * LBK_KMAX + 2] = d.x;
}

template <bool NT>
struct OpMid {  // r = (qin - alpha0 y0) * gamma;  acc += y0 . r      (:134-137, :150-154, :160)
    double* __restrict__ rout;
    const double* __restrict__ qin;
    const double* __restrict__ y0;
    double alpha, gamma;
    double* edge_slot;  // sharded: this rank's edge r for the neighbours' commit halo
    int64_t n_loc;
    int g_lo, g_hi;
    __device__ void set_coef(double a) { alpha = a; }
    struct Row {
        double2 q, y;
    };
    __device__ void load(Row& r, int64_t i) const {
        r.q = ldw<NT>(qin + i);
        r.y = ldv<NT>(y0 + i);
    }
    template <bool MASK>
    __device__ void apply(Row& r, int64_t i, int64_t, bool v0, bool v1, double (&acc)[1]) const {
        double2 rr;
        rr.x = (r.q.x - alpha * r.y.x) * gamma;
        rr.y = (r.q.y - alpha * r.y.y) * gamma;
        st2w<MASK, NT>(rout + i, rr, v0, v1);
        publish_edges(edge_slot, i, n_loc, g_lo, g_hi, rr, v0, v1);
        acc[0] = fma2<MASK>(r.y, rr, acc[0], v0, v1);
    }
};

template <bool NT>
struct OpAxpy2Dot {  // r += s (alpha - beta);  acc += ynext . r      (:159-164)
    double* r;        // out (== rin in place, or the other buffer of a ping-pong pair)
    const double* rin;
    const double* __restrict__ s;
    const double* __restrict__ yn;
    double coef;
    double* edge_slot;  // sharded: this rank's edge r for the neighbours' commit halo
    int64_t n_loc;
    int g_lo, g_hi;
    __device__ void set_coef(double c) { coef = c; }
    struct Row {
        double2 r, s, y;
    };
    __device__ void load(Row& w, int64_t i) const {
        w.r = ldw<NT>(rin + i);
        w.s = ldv<NT>(s + i);
        w.y = ldv<NT>(yn + i);
    }
    template <bool MASK>
    __device__ void apply(Row& w, int64_t i, int64_t, bool v0, bool v1, double (&acc)[1]) const {
        double2 rn;
        rn.x = w.r.x + w.s.x * coef;
        rn.y = w.r.y + w.s.y * coef;
        st2w<MASK, NT>(r + i, rn, v0, v1);
        publish_edges(edge_slot, i, n_loc, g_lo, g_hi, rn, v0, v1);
        acc[0] = fma2<MASK>(w.y, rn, acc[0], v0, v1);
    }
};

template <bool NT>
struct OpLast {  // d = -(r + s (alpha - beta));  acc += g . d        (:163-171)
    double* __restrict__ dout;
    const double* __restrict__ r;
    const double* __restrict__ s;
    const double* __restrict__ g;
    double coef;
    double* edge_slot;
    int64_t n_loc;
    int g_lo, g_hi;
    struct Row {
        double2 r, s, g;
    };
    __device__ void load(Row& w, int64_t i) const {
        w.r = ldw<NT>(r + i);
        w.s = ldv<NT>(s + i);
        w.g = ldx<NT>(g + i);
    }
    template <bool MASK>
    __device__ void apply(Row& w, int64_t i, int64_t, bool v0, bool v1, double (&acc)[1]) const {
        double2 d;
        d.x = -(w.r.x + w.s.x * coef);
        d.y = -(w.r.y + w.s.y * coef);
        st2w<MASK, NT>(dout + i, d, v0, v1);
        publish_edges(edge_slot, i, n_loc, g_lo, g_hi, d, v0, v1);
        acc[0] = fma2<MASK>(w.g, d, acc[0], v0, v1);
    }
};

template <bool NT>
struct OpNegDot {  // d = -g;  acc += g . d                          (:90, :151-152)
    double* __restrict__ dout;
    const double* __restrict__ g;
    double* edge_slot;
    int64_t n_loc;
    int g_lo, g_hi;
    struct Row {
        double2 g;
    };
    __device__ void load(Row& w, int64_t i) const { w.g = ldv<NT>(g + i); }
    template <bool MASK>
    __device__ void apply(Row& w, int64_t i, int64_t, bool v0, bool v1, double (&acc)[1]) const {
        double2 d;
        d.x = -w.g.x;
        d.y = -w.g.y;
        st2w<MASK, NT>(dout + i, d, v0, v1);
        publish_edges(edge_slot, i, n_loc, g_lo, g_hi, d, v0, v1);
        acc[0] = fma2<MASK>(w.g, d, acc[0], v0, v1);
    }
};

// Folded exchange of an r pass (sharded): the workgroup holding the rank's first or last element
// pushes that edge value, which one of its waves stored into the slot during the stream, to the
// peers once its waves are past the stream (a workgroup-scope hand-off on one CU).
__device__ __forceinline__ void fold_push_edges(const Geo& geo, const Seg& s, const FoldPush& fp) {
    const bool first = s.lb == 0, last = s.lb + s.len == geo.n_loc;
    if (!first && !last) return;  // uniform over the workgroup
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (threadIdx.x == 0) {
        const volatile double* e = geo.edge_slot;
        if (first) fold_push(fp, geo.g_lo * LBK_KMAX + 1, e[geo.g_lo * LBK_KMAX + 1]);
        if (last) fold_push(fp, (geo.g_hi - 1) * LBK_KMAX + 2, e[(geo.g_hi - 1) * LBK_KMAX + 2]);
    }
}

// FOLD: a folded exchange's producer (sharded, the mailboxes; the kernels of every other run are
// compiled without its code, which costs the pass kernels registers)
template <class Op, int K, bool FOLD = false>
__device__ __forceinline__ void run_pass(const Op& op, const Geo& geo, const Red& red) {
    const Seg s = seg_setup(geo);
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    stream(op, s, geo, acc);
    if (FOLD && red.fp.peers && geo.edge_slot) fold_push_edges(geo, s, red.fp);
    reduce_publish<K, FOLD>(acc, geo, red);
}

// Folded consumer (sharded over the mailboxes): the pass's coefficient waits for the peers' group
// values, so a full segment issues its first row group's loads before it polls; the wait for the
// xGMI hop runs under those loads instead of ahead of them. coef() is called by every thread (it
// synchronises the workgroup). The rows are applied and accumulated in the same order as
// run_pass, so the bits are the same.
#ifndef LBK_FOLD_PREFETCH
#define LBK_FOLD_PREFETCH 1  // A/B: 0 polls before any load, as round 3's first folded consumers
#endif
template <class Op, int K, class Coef>
__device__ __forceinline__ void run_pass_prefetch(Op op, const Geo& geo, const Red& red, Coef coef) {
    const Seg s = seg_setup(geo);
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    constexpr int U = op_unroll<Op>::value;
    if (LBK_FOLD_PREFETCH && s.len == geo.L && s.nrows >= U) {
        typename Op::Row r[U];
        load_group<U, K>(op, s, 0, r);
        op.set_coef(coef());
        apply_group<U, K>(op, s, 0, r, acc);
        stream(op, s, geo, acc, U);
    } else {
        op.set_coef(coef());
        stream(op, s, geo, acc);
    }
    if (red.fp.peers && geo.edge_slot) fold_push_edges(geo, s, red.fp);
    reduce_publish<K, true>(acc, geo, red);
}

template <class Op, int K>
__device__ __forceinline__ void run_pass_halo(const Op& op, const Geo& geo, const Red& red) {
    const Seg s = seg_setup(geo);
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    stream_halo(op, s, geo, acc);
    reduce_publish<K>(acc, geo, red);
}

template <bool NT, bool FOLD = false>
__global__ __launch_bounds__(LB_BLOCK) void k_dot(const double* __restrict__ a, const double* __restrict__ b,
                                                  Geo geo, Red red) {
    run_pass<OpDot<NT>, 1, FOLD>(OpDot<NT>{a, b}, geo, red);
}

// alpha = rho * total(prev)
// FOLD: sharded over the mailboxes, the source arrives folded (src_total polls) and the result is
// pushed folded. A folded producer whose source came through a slot (or the reverse) does not
// occur: the two-loop's passes fold as a chain.
template <bool NT, bool FOLD = false>
__global__ __launch_bounds__(LB_BLOCK) void k_axpy_dot(double* qout, const double* qin, const double* __restrict__ y,
                                                       const double* __restrict__ sv, double rho,
                                                       const double* __restrict__ prev, Geo geo, Red red, FoldSrc fs) {
    if constexpr (FOLD) {
        if (fs.mbx) {
            run_pass_prefetch<OpAxpyDot<NT>, 1>(OpAxpyDot<NT>{qout, qin, y, sv, 0.0}, geo, red,
                                                [&] { return rho * src_total_mailbox(prev, geo, fs); });
            return;
        }
    }
    const double alpha = rho * src_total(prev, geo);
    run_pass<OpAxpyDot<NT>, 1, FOLD>(OpAxpyDot<NT>{qout, qin, y, sv, alpha}, geo, red);
}

template <bool NT, bool FOLD = false>
__global__ __launch_bounds__(LB_BLOCK) void k_mid(double* __restrict__ rout, const double* __restrict__ qin,
                                                  const double* __restrict__ y0, double rho0, double gamma,
                                                  const double* __restrict__ prev, Geo geo, Red red, FoldSrc fs) {
    if constexpr (FOLD) {
        if (fs.mbx) {
            run_pass_prefetch<OpMid<NT>, 1>(OpMid<NT>{rout, qin, y0, 0.0, gamma, geo.edge_slot, geo.n_loc, geo.g_lo,
                                                      geo.g_hi},
                                            geo, red, [&] { return rho0 * src_total_mailbox(prev, geo, fs); });
            return;
        }
    }
    const double alpha = rho0 * src_total(prev, geo);
    run_pass<OpMid<NT>, 1, FOLD>(OpMid<NT>{rout, qin, y0, alpha, gamma, geo.edge_slot, geo.n_loc, geo.g_lo, geo.g_hi},
                                 geo, red);
}

// beta = rho * total(pb), alpha = rho * total(pa)
template <bool NT, bool FOLD = false>
__global__ __launch_bounds__(LB_BLOCK) void k_axpy2_dot(double* r, const double* rin, const double* __restrict__ sv,
                                                        const double* __restrict__ yn, double rho,
                                                        const double* __restrict__ pb, const double* __restrict__ pa,
                                                        Geo geo, Red red, FoldSrc fs) {
    if constexpr (FOLD) {
        if (fs.mbx) {
            run_pass_prefetch<OpAxpy2Dot<NT>, 1>(
                OpAxpy2Dot<NT>{r, rin, sv, yn, 0.0, geo.edge_slot, geo.n_loc, geo.g_lo, geo.g_hi}, geo, red, [&] {
                    const double beta = rho * src_total_mailbox(pb, geo, fs);
                    const double alpha = rho * slot_total(pa);
                    return alpha - beta;
                });
            return;
        }
    }
    const double beta = rho * src_total(pb, geo);
    const double alpha = rho * slot_total(pa);
    run_pass<OpAxpy2Dot<NT>, 1, FOLD>(
        OpAxpy2Dot<NT>{r, rin, sv, yn, alpha - beta, geo.edge_slot, geo.n_loc, geo.g_lo, geo.g_hi}, geo, red);
}

template <bool NT>
__global__ __launch_bounds__(LB_BLOCK) void k_last(double* __restrict__ dout, const double* __restrict__ r,
                                                   const double* __restrict__ sv, const double* __restrict__ g,
                                                   double rho, const double* __restrict__ pb,
                                                   const double* __restrict__ pa, Geo geo, Red red) {
    const double beta = rho * src_total(pb, geo);
    const double alpha = rho * slot_total(pa);
    run_pass<OpLast<NT>, 1>(OpLast<NT>{dout, r, sv, g, alpha - beta, geo.edge_slot, geo.n_loc, geo.g_lo, geo.g_hi},
                             geo, red);
}

template <bool NT>
__global__ __launch_bounds__(LB_BLOCK) void k_negdot(double* __restrict__ dout, const double* __restrict__ g,
                                                     Geo geo, Red red) {
    run_pass<OpNegDot<NT>, 1>(OpNegDot<NT>{dout, g, geo.edge_slot, geo.n_loc, geo.g_lo, geo.g_hi}, geo, red);
}

// ---------------------------------------------------------------------------------------
// Objective passes: evaluation point z = x + alpha d with d given by DMODE.
// ---------------------------------------------------------------------------------------
struct DirArgs {
    const double* dsrc;  // D_BUF: d;  D_TWOLOOP: r
    const double* s;     // D_TWOLOOP: s_{h-1}
    const double* g;     // D_NEG_G / commit: g
    double coef;         // D_TWOLOOP: alpha - beta (formed on the device, see k_commit)
    const double* pa;    // D_TWOLOOP: slot of s_{h-1} . q   (alpha = rho * total)
    const double* pb;    // D_TWOLOOP: slot of y_{h-1} . r   (beta  = rho * total)
    double rho;
    const double* ghost;  // sharded, D_BUF: all-gathered slot holding the neighbours' edge d
    int g_lo, g_hi;
    // cooperative iteration, D_TWOLOOP: the last r pass's flagged words (components 1 / 2: first /
    // last r of every segment), that pass's sequence number, the segment length that indexes them
    const unsigned long long* redge;
    int64_t L;
    unsigned redge_seq;
    unsigned* err;
    unsigned long long tmo;
};

// A/B: LBK_DIR_NT=1 streams the direction source (d, or r of the last second-loop pass) of the
// commit and the trials non-temporal
#ifndef LBK_DIR_NT
#define LBK_DIR_NT 0
#endif
template <bool NT>
__device__ __forceinline__ double2 ldd(const double* p) {
    return LBK_DIR_NT ? ldv<NT>(p) : ldw<NT>(p);
}
template <int DMODE, bool NT>
__device__ __forceinline__ double2 load_dir(const DirArgs& da, int64_t i, double2 gv) {
    double2 d;
    if (DMODE == LBK_D_BUF) {
        d = ldd<NT>(da.dsrc + i);
    } else if (DMODE == LBK_D_NEG_G) {
        d.x = -gv.x;
        d.y = -gv.y;
    } else {
        const double2 rv = ldd<NT>(da.dsrc + i);
        const double2 sv = ldv<NT>(da.s + i);
        d.x = -(rv.x + sv.x * da.coef);
        d.y = -(rv.y + sv.y * da.coef);
    }
    return d;
}
template <int DMODE>
__device__ __forceinline__ double load_dir1(const DirArgs& da, int64_t i) {
    if (DMODE == LBK_D_BUF) return da.dsrc[i];
    if (DMODE == LBK_D_NEG_G) return -da.g[i];
    return -(da.dsrc[i] + da.s[i] * da.coef);
}

// neighbour rank's edge d, from the all-gathered slot (see publish_edges)
__device__ __forceinline__ double ghost_d(const DirArgs& da, int64_t hi, int64_t n_loc) {
    // left ghost = last d of the rank owning group g_lo-1; right ghost = first d of group g_hi
    return hi < 0 ? da.ghost[(da.g_lo - 1) * LBK_KMAX + 2] : da.ghost[da.g_hi * LBK_KMAX + 1];
    (void)n_loc;
}

template <int OBJ>
__device__ __forceinline__ bool needs_halo() {
    return OBJ == LBK_OBJ_ROSENBROCK || OBJ == LBK_OBJ_QUAD_TRIDIAG;
}

// halo value z = x + alpha d at local index i-1 (lane 0) or i+2 (lane 63)
template <int OBJ, bool NO_DIR, int DMODE>
__device__ __forceinline__ double halo_z(const double* __restrict__ x, const DirArgs& da, double alpha,
                                         int64_t i, int64_t n_loc) {
    double zh = 0.0;
    if (needs_halo<OBJ>()) {
        const int lane = threadIdx.x & 63;
        if (lane == 0 || lane == 63) {
            const int64_t hi = (lane == 0) ? i - 1 : i + 2;
            if (hi >= -1 && hi <= n_loc) {
                if (NO_DIR) {
                    zh = x[hi];
                } else {
                    double dh;
                    if (DMODE == LBK_D_BUF && da.ghost && (hi == -1 || hi == n_loc))
                        dh = ghost_d(da, hi, n_loc);
                    else if (DMODE == LBK_D_TWOLOOP && da.ghost && (hi == -1 || hi == n_loc))
                        dh = -(ghost_d(da, hi, n_loc) + da.s[hi] * da.coef);  // neighbour's edge r, s ghost
                    else if (DMODE == LBK_D_TWOLOOP && da.redge && hi >= 0 && hi < n_loc && hi / da.L != i / da.L) {
                        // r of another workgroup's segment, written in this launch: its published
                        // edge (write-through), not the plain-stored vector
                        const int64_t sg = hi / da.L;
                        const double rv = ll_load(da.redge + ((hi == sg * da.L ? 1 : 2) * LBK_LL_SEGS + sg) * 2,
                                                  da.redge_seq, da.err, da.tmo);
                        dh = -(rv + da.s[hi] * da.coef);
                    } else
                        dh = load_dir1<DMODE>(da, hi);
                    zh = x[hi] + alpha * dh;
                }
            }
        }
    }
    return zh;
}

// (x, d) at local element hi (-1 <= hi <= n_loc; zeros outside), d per DMODE: halo operands
template <int DMODE, bool REDGE = false>
__device__ __forceinline__ double2 xd_at(const double* __restrict__ x, const DirArgs& da, int64_t hi, int64_t n_loc) {
    if (hi < -1 || hi > n_loc) return make_double2(0.0, 0.0);
    double dh;
    if (DMODE == LBK_D_BUF && da.ghost && (hi == -1 || hi == n_loc))
        dh = ghost_d(da, hi, n_loc);
    else if (DMODE == LBK_D_TWOLOOP && da.ghost && (hi == -1 || hi == n_loc))
        dh = -(ghost_d(da, hi, n_loc) + da.s[hi] * da.coef);
    else if (REDGE && DMODE == LBK_D_TWOLOOP && da.redge && hi >= 0 && hi < n_loc &&
             (hi == (hi / da.L) * da.L || hi == (hi / da.L) * da.L + da.L - 1)) {
        // persistent iteration (stencil walk): a segment edge's r, written in this launch by the
        // workgroup that owns that segment - its published edge word (as halo_z)
        const int64_t sg = hi / da.L;
        const double rv = ll_load(da.redge + ((hi == sg * da.L ? 1 : 2) * LBK_LL_SEGS + sg) * 2, da.redge_seq,
                                  da.err, da.tmo);
        dh = -(rv + da.s[hi] * da.coef);
    } else
        dh = load_dir1<DMODE>(da, hi);
    return make_double2(x[hi], dh);
}

// (x, d) at the halo element of lane 0 (i-1) / lane 63 (i+2), or zeros: every step's halo
// z = x + a d from one read (the batched trials and the commit's candidate step); the same
// operands and operations as halo_z
template <int OBJ, int DMODE>
__device__ __forceinline__ double2 halo_xd(const double* __restrict__ x, const DirArgs& da, int64_t i, int64_t n_loc) {
    double2 xd = make_double2(0.0, 0.0);
    if (needs_halo<OBJ>()) {
        const int lane = threadIdx.x & 63;
        if (lane == 0 || lane == 63) {
            const int64_t hi = (lane == 0) ? i - 1 : i + 2;
            if (hi >= -1 && hi <= n_loc) {
                double dh;
                if (DMODE == LBK_D_BUF && da.ghost && (hi == -1 || hi == n_loc))
                    dh = ghost_d(da, hi, n_loc);
                else if (DMODE == LBK_D_TWOLOOP && da.ghost && (hi == -1 || hi == n_loc))
                    dh = -(ghost_d(da, hi, n_loc) + da.s[hi] * da.coef);
                else if (DMODE == LBK_D_TWOLOOP && da.redge && hi >= 0 && hi < n_loc && hi / da.L != i / da.L) {
                    // cooperative iteration: another workgroup's r from this launch (as halo_z)
                    const int64_t sg = hi / da.L;
                    const double rv = ll_load(da.redge + ((hi == sg * da.L ? 1 : 2) * LBK_LL_SEGS + sg) * 2,
                                              da.redge_seq, da.err, da.tmo);
                    dh = -(rv + da.s[hi] * da.coef);
                } else
                    dh = load_dir1<DMODE>(da, hi);
                xd = make_double2(x[hi], dh);
            }
        }
    }
    return xd;
}

// f terms of the two elements of a lane at z (right neighbour from the row, lane 63's from zh)
template <int OBJ, bool MASK>
__device__ __forceinline__ void objective_f_pair(double2 z, double zh, int64_t e0, int64_t n, bool v0, bool v1,
                                                 double& facc) {
    const int lane = threadIdx.x & 63;
    const double dn = __shfl_down(z.x, 1, 64);
    const double zr = (lane == 63) ? zh : dn;
    const bool p0 = e0 + 1 < n, p1 = e0 + 2 < n;
    if ((!MASK || v0) && obj_has_term<OBJ>(p0)) facc = facc + obj_term<OBJ>(z.x, z.y, p0);
    if ((!MASK || v1) && obj_has_term<OBJ>(p1)) facc = facc + obj_term<OBJ>(z.y, zr, p1);
}

// f terms and gradient of the two elements of a lane at z (neighbours from the row)
template <int OBJ, bool MASK>
__device__ __forceinline__ double2 objective_pair(double2 z, double zh, int64_t e0, int64_t n, bool v0, bool v1,
                                                  double& facc, bool with_g) {
    const int lane = threadIdx.x & 63;
    const Nb nb = neighbours(z.x, z.y, zh, lane);
    const bool p0 = e0 + 1 < n, p1 = e0 + 2 < n;
    if ((!MASK || v0) && obj_has_term<OBJ>(p0)) facc = facc + obj_term<OBJ>(z.x, z.y, p0);
    if ((!MASK || v1) && obj_has_term<OBJ>(p1)) facc = facc + obj_term<OBJ>(z.y, nb.r, p1);
    double2 g;
    if (with_g) {
        g.x = obj_grad<OBJ>(nb.l, z.x, z.y, e0 > 0, p0);
        g.y = obj_grad<OBJ>(z.x, z.y, nb.r, true, p1);
    }
    return g;
}

// Evaluate f (and optionally g) at z = x (NO_DIR, reductions f, g.g; lbfgs.cpp:29-30) or at
// z = x + alpha d (reductions f, g_t . d; line_search.cpp trials).
template <int OBJ, bool NO_DIR, bool WITH_G, bool NT>
struct OpObjective {
    const double* __restrict__ x;
    DirArgs da;
    double alpha;
    double* __restrict__ gout;
    int64_t n, n_loc;
    struct Row {
        double2 z, d;
        double zh;
    };
    __device__ void load(Row& r, int64_t i) const {
        const double2 xv = ldx<NT>(x + i);
        if (NO_DIR) {
            r.z = xv;
        } else {
            r.d = ldw<NT>(da.dsrc + i);
            r.z.x = xv.x + alpha * r.d.x;
            r.z.y = xv.y + alpha * r.d.y;
        }
        r.zh = halo_z<OBJ, NO_DIR, LBK_D_BUF>(x, da, alpha, i, n_loc);
    }
    template <bool MASK>
    __device__ void apply(Row& r, int64_t i, int64_t e0, bool v0, bool v1, double (&acc)[2]) const {
        const double2 g = objective_pair<OBJ, MASK>(r.z, r.zh, e0, n, v0, v1, acc[0], WITH_G);
        if (WITH_G) {
            if (gout) st2x<MASK, NT>(gout + i, g, v0, v1);
            acc[1] = NO_DIR ? fma2<MASK>(g, g, acc[1], v0, v1) : fma2<MASK>(g, r.d, acc[1], v0, v1);
        }
    }
};

template <int OBJ, bool NO_DIR, bool WITH_G, bool NT>
__global__ __launch_bounds__(LB_BLOCK) void k_objective(const double* __restrict__ x, DirArgs da, double alpha,
                                                        double* __restrict__ gout, Geo geo, Red red) {
    run_pass<OpObjective<OBJ, NO_DIR, WITH_G, NT>, 2>(OpObjective<OBJ, NO_DIR, WITH_G, NT>{x, da, alpha, gout, geo.n, geo.n_loc},
                                                  geo, red);
}

// The commit: d per DMODE, x_new = x + alpha d, f(x_new), g_new = grad f(x_new) (or read
// from gn for OBJ == NONE), s = x_new - x, y = g_new - g, and the dots
//   [GD] g.d  [F] f  [SY] s.y  [YY] y.y  [GG] g_new.g_new  [SG] s.g_new  [DPHI] g_new.d
// CAND: also f(x + cand d) at the line search's next backtracking step [FC] (no extra bytes:
// x and d are in registers), so a rejected first step needs no trial pass for the second.
// REDGE: the persistent iteration's commit (k_persist_iter), whose stencil halos at segment edges
// come from the published edge words
template <int OBJ, int DMODE, bool NT, bool CAND = false, bool REDGE = false>
struct OpCommit {
    static constexpr int K = CAND ? 8 : 7;
    const double* __restrict__ x;
    DirArgs da;
    double alpha;
    double* __restrict__ xn;
    double* __restrict__ gn;
    double* __restrict__ so;
    double* __restrict__ yo;
    int64_t n, n_loc;
    double cand;
    struct Row {
        double2 x, g, d, z, gx;
        double zh, zch;
    };
    static constexpr bool kStencil = OBJ != LBK_OBJ_NONE && (OBJ == LBK_OBJ_ROSENBROCK || OBJ == LBK_OBJ_QUAD_TRIDIAG);
    __device__ void load_core(Row& r, int64_t i) const {
        r.x = ldx<NT>(x + i);
        r.g = ldx<NT>(da.g + i);
        r.d = load_dir<DMODE, NT>(da, i, r.g);
        if (OBJ == LBK_OBJ_NONE) r.gx = ldv<NT>(gn + i);
        r.z.x = r.x.x + alpha * r.d.x;
        r.z.y = r.x.y + alpha * r.d.y;
    }
    __device__ double2 halo_mem(int64_t hi) const { return xd_at<DMODE, REDGE>(x, da, hi, n_loc); }
    __device__ double2 edge_first(const Row& r) const { return make_double2(r.x.x, r.d.x); }
    __device__ double2 edge_last(const Row& r) const { return make_double2(r.x.y, r.d.y); }
    __device__ void set_halo(Row& r, double2 xd) const {
        r.zh = xd.x + alpha * xd.y;
        if (CAND) r.zch = xd.x + cand * xd.y;
    }
    __device__ void load(Row& r, int64_t i) const {
        r.x = ldx<NT>(x + i);
        r.g = ldx<NT>(da.g + i);
        r.d = load_dir<DMODE, NT>(da, i, r.g);
        if (OBJ == LBK_OBJ_NONE) r.gx = ldv<NT>(gn + i);
        r.z.x = r.x.x + alpha * r.d.x;
        r.z.y = r.x.y + alpha * r.d.y;
        if (CAND) {
            const double2 xd = halo_xd<OBJ, DMODE>(x, da, i, n_loc);
            r.zh = xd.x + alpha * xd.y;
            r.zch = xd.x + cand * xd.y;
        } else {
            r.zh = (OBJ == LBK_OBJ_NONE) ? 0.0 : halo_z<OBJ, false, DMODE>(x, da, alpha, i, n_loc);
        }
    }
    template <bool MASK>
    __device__ void apply(Row& r, int64_t i, int64_t e0, bool v0, bool v1, double (&acc)[K]) const {
        if (CAND) {
            double2 zc;
            zc.x = r.x.x + cand * r.d.x;
            zc.y = r.x.y + cand * r.d.y;
            objective_f_pair<OBJ, MASK>(zc, r.zch, e0, n, v0, v1, acc[LBK_C_FC]);
        }
        double2 g2;
        if (OBJ == LBK_OBJ_NONE) {
            g2 = r.gx;
        } else {
            g2 = objective_pair<OBJ, MASK>(r.z, r.zh, e0, n, v0, v1, acc[LBK_C_F], true);
            st2x<MASK, NT>(gn + i, g2, v0, v1);
        }
        st2x<MASK, NT>(xn + i, r.z, v0, v1);
        double2 sv, yv;
        sv.x = r.z.x - r.x.x;
        sv.y = r.z.y - r.x.y;
        yv.x = g2.x - r.g.x;
        yv.y = g2.y - r.g.y;
        st2h<MASK, NT>(so + i, sv, v0, v1);
        st2h<MASK, NT>(yo + i, yv, v0, v1);
        acc[LBK_C_GD] = fma2<MASK>(r.g, r.d, acc[LBK_C_GD], v0, v1);
        acc[LBK_C_SY] = fma2<MASK>(sv, yv, acc[LBK_C_SY], v0, v1);
        acc[LBK_C_YY] = fma2<MASK>(yv, yv, acc[LBK_C_YY], v0, v1);
        acc[LBK_C_GG] = fma2<MASK>(g2, g2, acc[LBK_C_GG], v0, v1);
        acc[LBK_C_SG] = fma2<MASK>(sv, g2, acc[LBK_C_SG], v0, v1);
        acc[LBK_C_DPHI] = fma2<MASK>(g2, r.d, acc[LBK_C_DPHI], v0, v1);
    }
};

#ifndef LBK_COMMIT_WAVES
#define LBK_COMMIT_WAVES 0  // A/B: > 0 asks the register allocation for that many waves per SIMD
#endif
#if LBK_COMMIT_WAVES > 0
#define LBK_COMMIT_ATTR __attribute__((amdgpu_waves_per_eu(LBK_COMMIT_WAVES)))
#else
#define LBK_COMMIT_ATTR
#endif
template <int OBJ, int DMODE, bool NT, bool CAND = false>
__global__ __launch_bounds__(LB_BLOCK) LBK_COMMIT_ATTR void k_commit(const double* __restrict__ x, DirArgs da, double alpha,
                                                     double* __restrict__ xn, double* __restrict__ gn,
                                                     double* __restrict__ so, double* __restrict__ yo,
                                                     Geo geo, Red red, double cand = 0.0) {
    if (DMODE == LBK_D_TWOLOOP) {
        const double beta = da.rho * src_total(da.pb, geo);
        const double alph = da.rho * slot_total(da.pa);
        da.coef = alph - beta;  // r[j] += s[j] * (alpha[i] - beta)  (lbfgs.cpp:137)
    }
    // sharded: keep the x and s ghosts current (x_new = x + alpha d and s = x_new - x at the
    // neighbours' edge elements: the owner's operands, so the owner's bits). The s ghosts let a
    // later TWOLOOP commit form the neighbours' edge d from their published edge r.
    if ((DMODE == LBK_D_BUF || DMODE == LBK_D_TWOLOOP) && da.ghost && threadIdx.x == 0) {
        if (seg_block(geo) == 0 && geo.elem_lo > 0) {
            const double dh = DMODE == LBK_D_BUF ? ghost_d(da, -1, geo.n_loc)
                                                 : -(ghost_d(da, -1, geo.n_loc) + da.s[-1] * da.coef);
            const double z = x[-1] + alpha * dh;
            xn[-1] = z;
            so[-1] = z - x[-1];
        }
        if (seg_block(geo) == gridDim.x - 1 && geo.elem_lo + geo.n_loc < geo.n) {
            const int64_t e = geo.n_loc;
            const double dh = DMODE == LBK_D_BUF ? ghost_d(da, e, geo.n_loc)
                                                 : -(ghost_d(da, e, geo.n_loc) + da.s[e] * da.coef);
            const double z = x[e] + alpha * dh;
            xn[e] = z;
            so[e] = z - x[e];
        }
    }
    using Op = OpCommit<OBJ, DMODE, NT, CAND>;
    run_pass_halo<Op, Op::K>(Op{x, da, alpha, xn, gn, so, yo, geo.n, geo.n_loc, cand}, geo, red);
}

// Batched line-search trials: f at NC steps a[0..NC-1] along d (d per DMODE: a buffer, -g, or the
// last second-loop update -(r + s (alpha - beta)) formed on the fly, so a rejected first step
// needs no materialised d) in one read of x and d; DPHI: also g(x + a[0] d) . d (the Wolfe
// curvature term) from the same pass, the gradient never stored. Components: f_0..f_{NC-1}
// [, dphi_0]. Every f is summed in the order of a single-step evaluation (same bits).
template <int OBJ, int DMODE, int NC, bool DPHI, bool NT>
struct OpTrials {
    static constexpr int K = NC + (DPHI ? 1 : 0);
    const double* __restrict__ x;
    DirArgs da;
    double a[NC];
    int64_t n, n_loc;
    struct Row {
        double2 x, d;
        double xh, dh;
    };
    static constexpr bool kStencil = OBJ == LBK_OBJ_ROSENBROCK || OBJ == LBK_OBJ_QUAD_TRIDIAG;
    __device__ void load_core(Row& r, int64_t i) const {
        r.x = ldx<NT>(x + i);
        double2 gv = make_double2(0.0, 0.0);
        if (DMODE == LBK_D_NEG_G) gv = ldx<NT>(da.g + i);
        r.d = load_dir<DMODE, NT>(da, i, gv);
    }
    __device__ double2 halo_mem(int64_t hi) const { return xd_at<DMODE>(x, da, hi, n_loc); }
    __device__ double2 edge_first(const Row& r) const { return make_double2(r.x.x, r.d.x); }
    __device__ double2 edge_last(const Row& r) const { return make_double2(r.x.y, r.d.y); }
    __device__ void set_halo(Row& r, double2 xd) const {
        r.xh = xd.x;
        r.dh = xd.y;
    }
    __device__ void load(Row& r, int64_t i) const {
        load_core(r, i);
        const double2 xd = halo_xd<OBJ, DMODE>(x, da, i, n_loc);
        r.xh = xd.x;
        r.dh = xd.y;
    }
    template <bool MASK>
    __device__ void apply(Row& r, int64_t, int64_t e0, bool v0, bool v1, double (&acc)[K]) const {
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            double2 z;
            z.x = r.x.x + a[j] * r.d.x;
            z.y = r.x.y + a[j] * r.d.y;
            const double zh = r.xh + a[j] * r.dh;
            if (DPHI && j == 0) {
                const double2 g = objective_pair<OBJ, MASK>(z, zh, e0, n, v0, v1, acc[0], true);
                acc[NC] = fma2<MASK>(g, r.d, acc[NC], v0, v1);
            } else {
                objective_f_pair<OBJ, MASK>(z, zh, e0, n, v0, v1, acc[j]);
            }
        }
    }
};

template <int OBJ, int DMODE, int NC, bool DPHI, bool NT>
__global__ __launch_bounds__(LB_BLOCK) void k_trials(Geo geo, Red red, OpTrials<OBJ, DMODE, NC, DPHI, NT> op) {
    if (DMODE == LBK_D_TWOLOOP) {  // alpha - beta of the last second-loop update (as k_commit)
        const double beta = op.da.rho * src_total(op.da.pb, geo);
        const double alph = op.da.rho * slot_total(op.da.pa);
        op.da.coef = alph - beta;
    }
    run_pass_halo<OpTrials<OBJ, DMODE, NC, DPHI, NT>, OpTrials<OBJ, DMODE, NC, DPHI, NT>::K>(op, geo, red);
}

// ---------------------------------------------------------------------------------------
// Dense quadratic objective f(x) = x'Ax + b'x, grad = 2 A x + b: the known-answer problems of
// the reference's sequential-implementation/matrices.h (mat<n>, linear<n>, minimum<n>;
// SURVEY 8f item 4). Row i of A x is one wave: lane l accumulates fma(A_ij, x_j) over
// j = l, l + 64, ... in ascending order, then the wave butterfly; g_i = 2 r_i + b_i and the f term
// t_i = x_i r_i + b_i x_i, which the pass after it sums in the canonical order. The row order
// is restated by oracle/lbfgs_oracle.c (dense_row).
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_dense_rows(const double* __restrict__ A, const double* __restrict__ b,
                                                    const double* __restrict__ x, double* __restrict__ g,
                                                    double* __restrict__ t, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;  // wave-uniform
    const double* __restrict__ a = A + i * n;
    double v = 0.0;
    for (int64_t j = lane; j < n; j += 64) v = fma(a[j], x[j], v);
    v = wave_sum(v);
    if (lane == 0) {
        const double xi = x[i];
        if (g) g[i] = 2.0 * v + b[i];
        t[i] = xi * v + b[i] * xi;
    }
}

// f = canonical sum of the terms t; with g, also g . g (lbk_eval's components)
template <bool NT>
struct OpTermsDot {
    const double* __restrict__ t;
    const double* __restrict__ g;
    struct Row {
        double2 t, g;
    };
    __device__ void load(Row& r, int64_t i) const {
        r.t = ldv<NT>(t + i);
        if (g) r.g = ldv<NT>(g + i);
    }
    template <bool MASK>
    __device__ void apply(Row& r, int64_t, int64_t, bool v0, bool v1, double (&acc)[2]) const {
        if (!MASK || v0) acc[0] = acc[0] + r.t.x;
        if (!MASK || v1) acc[0] = acc[0] + r.t.y;
        if (g) acc[1] = fma2<MASK>(r.g, r.g, acc[1], v0, v1);
    }
};

template <bool NT>
__global__ __launch_bounds__(LB_BLOCK) void k_terms_dot(const double* __restrict__ t, const double* __restrict__ g,
                                                        Geo geo, Red red) {
    run_pass<OpTermsDot<NT>, 2>(OpTermsDot<NT>{t, g}, geo, red);
}

// ---------------------------------------------------------------------------------------
// Vector-free mode (LBFGS_FLAG_VECTOR_FREE). The two-loop runs on the host in coefficient
// space over the Gram matrix of the basis b = [s_0..s_{h-1}, y_0..y_{h-1}, g]; the device
// pass forms d = sum_l c_l b_l + cg g on the fly (l ascending, then g; each product rounded,
// -ffp-contract=off), evaluates the first trial and commits in one sweep, and reduces the new
// Gram rows. HB is the compile-time capacity (bucket) of h, with uniform runtime guards l < 2h,
// so the basis registers and accumulators have static indices.
// ---------------------------------------------------------------------------------------
template <int HB>
struct VfBasis {
    const double* b[2 * HB > 0 ? 2 * HB : 1];
    double c[2 * HB > 0 ? 2 * HB : 1];
    double cg;
    int h;
};

template <int HB>
__device__ __forceinline__ double vf_dir1(const VfBasis<HB>& B, const double* __restrict__ g, int64_t i) {
    double d = 0.0;
#pragma unroll
    for (int l = 0; l < 2 * HB; ++l)
        if (l < 2 * B.h) d = (l == 0) ? B.c[0] * B.b[0][i] : d + B.c[l] * B.b[l][i];
    return B.h == 0 ? B.cg * g[i] : d + B.cg * g[i];
}

// f terms, gradient, x_new, s, y, and the dots (components LBK_VF_*)
template <int OBJ, int HB, bool NT>
struct OpVfCommit {
    static constexpr int K = LBK_VF_YB + 4 * HB + LBK_VF_NA;
    static constexpr int FC = LBK_VF_YB + 4 * HB;  // f at the candidate steps ac[j]
    static constexpr int NB = 2 * HB;
    const double* __restrict__ x;
    const double* __restrict__ g;
    VfBasis<HB> B;
    double alpha;
    double ac[LBK_VF_NA];  // the line search's next candidate steps (alpha * beta^j)
    double* __restrict__ xn;
    double* __restrict__ gn;
    double* __restrict__ so;
    double* __restrict__ yo;
    int64_t n, n_loc;
    struct Row {
        double2 x, g, z;
        double2 zc[LBK_VF_NA];
        double2 b[2 * HB > 0 ? 2 * HB : 1];
        double zh;
    };
    // x, g, the basis and z = x + alpha d (and x + ac[j] d) of local elements i, i+1
    __device__ void load(Row& r, int64_t i) const {
        r.x = ldx<NT>(x + i);
        r.g = ldx<NT>(g + i);
#pragma unroll
        for (int l = 0; l < 2 * HB; ++l)
            if (l < 2 * B.h) r.b[l] = ldv<NT>(B.b[l] + i);
        form(r);
    }
    // d, z = x + alpha d and the candidate points from the loaded row (every basis product
    // rounded, l ascending, then g: the ORC_CANON_VF order)
    __device__ void form(Row& r) const {
        double2 d = make_double2(0.0, 0.0);
#pragma unroll
        for (int l = 0; l < 2 * HB; ++l) {
            if (l < 2 * B.h) {
                if (l == 0) {
                    d.x = B.c[0] * r.b[0].x;
                    d.y = B.c[0] * r.b[0].y;
                } else {
                    d.x = d.x + B.c[l] * r.b[l].x;
                    d.y = d.y + B.c[l] * r.b[l].y;
                }
            }
        }
        if (B.h == 0) {
            d.x = B.cg * r.g.x;
            d.y = B.cg * r.g.y;
        } else {
            d.x = d.x + B.cg * r.g.x;
            d.y = d.y + B.cg * r.g.y;
        }
        r.z.x = r.x.x + alpha * d.x;
        r.z.y = r.x.y + alpha * d.y;
#pragma unroll
        for (int j = 0; j < LBK_VF_NA; ++j) {
            r.zc[j].x = r.x.x + ac[j] * d.x;
            r.zc[j].y = r.x.y + ac[j] * d.y;
        }
        r.zh = 0.0;
    }
    // lane 63: keep the basis values of its last element for finish()
    __device__ void park(const Row& r, double* pk) const {
#pragma unroll
        for (int l = 0; l < 2 * HB; ++l)
            if (l < 2 * B.h) pk[l] = r.b[l].y;
    }
    // the deferred last element of a row (local i, global e) once its right neighbour zp is
    // known: the second element of apply() for lane 63, in the same operation order
    __device__ void finish(double zm, double zc, double zp, double xv, double gv, const double* pk, int64_t i,
                           int64_t e, const double* pzc, const double* zpc, double (&acc)[K]) const {
        const bool p1 = e + 1 < n;
        if (obj_has_term<OBJ>(p1)) acc[LBK_VF_F] = acc[LBK_VF_F] + obj_term<OBJ>(zc, zp, p1);
        if (obj_has_term<OBJ>(p1)) {
#pragma unroll
            for (int j = 0; j < LBK_VF_NA; ++j) acc[FC + j] = acc[FC + j] + obj_term<OBJ>(pzc[j], zpc[j], p1);
        }
        const double g2 = obj_grad<OBJ>(zm, zc, zp, true, p1);
        gn[i] = g2;
        xn[i] = zc;
        const double sv = zc - xv, yv = g2 - gv;
        so[i] = sv;
        yo[i] = yv;
        acc[LBK_VF_SY] = fma(sv, yv, acc[LBK_VF_SY]);
        acc[LBK_VF_YY] = fma(yv, yv, acc[LBK_VF_YY]);
        acc[LBK_VF_GG] = fma(g2, g2, acc[LBK_VF_GG]);
        acc[LBK_VF_YG] = fma(yv, g2, acc[LBK_VF_YG]);
        acc[LBK_VF_GGO] = fma(g2, gv, acc[LBK_VF_GGO]);
#pragma unroll
        for (int l = 0; l < 2 * HB; ++l) {
            if (l < 2 * B.h) {
                acc[LBK_VF_YB + l] = fma(yv, pk[l], acc[LBK_VF_YB + l]);
                acc[LBK_VF_YB + 2 * HB + l] = fma(g2, pk[l], acc[LBK_VF_YB + 2 * HB + l]);
            }
        }
    }
    // (x, d) at one local element (-1 <= hi <= n_loc) formed from memory (segment edges only);
    // z = x + alpha d for any step alpha
    __device__ double2 xd_at(int64_t hi) const {
        if (!needs_halo<OBJ>() || hi < -1 || hi > n_loc) return make_double2(0.0, 0.0);
        return make_double2(x[hi], vf_dir1<HB>(B, g, hi));
    }
    template <bool MASK>
    __device__ void apply(Row& r, int64_t i, int64_t e0, bool v0, bool v1, double (&acc)[K]) const {
        const double2 g2 = objective_pair<OBJ, MASK>(r.z, r.zh, e0, n, v0, v1, acc[LBK_VF_F], true);
        st2x<MASK, NT>(gn + i, g2, v0, v1);
        st2x<MASK, NT>(xn + i, r.z, v0, v1);
        double2 sv, yv;
        sv.x = r.z.x - r.x.x;
        sv.y = r.z.y - r.x.y;
        yv.x = g2.x - r.g.x;
        yv.y = g2.y - r.g.y;
        st2h<MASK, NT>(so + i, sv, v0, v1);
        st2h<MASK, NT>(yo + i, yv, v0, v1);
        acc[LBK_VF_SY] = fma2<MASK>(sv, yv, acc[LBK_VF_SY], v0, v1);
        acc[LBK_VF_YY] = fma2<MASK>(yv, yv, acc[LBK_VF_YY], v0, v1);
        acc[LBK_VF_GG] = fma2<MASK>(g2, g2, acc[LBK_VF_GG], v0, v1);
        acc[LBK_VF_YG] = fma2<MASK>(yv, g2, acc[LBK_VF_YG], v0, v1);
        acc[LBK_VF_GGO] = fma2<MASK>(g2, r.g, acc[LBK_VF_GGO], v0, v1);
        // f at the candidate steps: the same terms as objective_pair's, right neighbours only
        {
            const bool p0 = e0 + 1 < n, p1 = e0 + 2 < n;
#pragma unroll
            for (int j = 0; j < LBK_VF_NA; ++j) {
                const double nr = __shfl_down(r.zc[j].x, 1, 64);
                if ((!MASK || v0) && obj_has_term<OBJ>(p0))
                    acc[FC + j] = acc[FC + j] + obj_term<OBJ>(r.zc[j].x, r.zc[j].y, p0);
                if ((!MASK || v1) && obj_has_term<OBJ>(p1)) acc[FC + j] = acc[FC + j] + obj_term<OBJ>(r.zc[j].y, nr, p1);
            }
        }
#pragma unroll
        for (int l = 0; l < 2 * HB; ++l) {
            if (l < 2 * B.h) {
                acc[LBK_VF_YB + l] = fma2<MASK>(yv, r.b[l], acc[LBK_VF_YB + l], v0, v1);
                acc[LBK_VF_YB + 2 * HB + l] = fma2<MASK>(g2, r.b[l], acc[LBK_VF_YB + 2 * HB + l], v0, v1);
            }
        }
    }
};

// The segment walk of the vector-free commit. Wave w takes a contiguous run of rows
// [wR, min((w+1)R, nrow)), R = ceil(nrow / 4) (the ORC_CANON_VF order), so a row's left stencil
// neighbour is the previous row's last z, carried in a register, and its right neighbour is the
// next row's first z: lane 63's last element is finished one step later, after the next row is
// loaded (its basis values parked in wave-private LDS). Each lane still accumulates its
// elements in ascending order. Only the ends of a wave's run form z from memory (Op::z_at):
// 2 per wave per segment instead of 2 per row. No barriers: the waves stream independently.
template <int K, class Op>
__device__ __forceinline__ void stream_vf(const Op& op, const Seg& s, const Geo& geo, double (&acc)[K]) {
    constexpr int NB = Op::NB > 0 ? Op::NB : 1;
    __shared__ double park[4][NB];
    const int nrow = (int)((s.len + 127) / 128);
    const int R = (nrow + 3) / 4;
    const int r0 = s.w * R;
    const int r1 = min(r0 + R, nrow);
    if (r0 >= r1) return;
    const bool full = s.len == geo.L;
    const bool last_lane = s.lane == 63;
    // both ends of the run formed up front, branch-free: lane 0 at the left neighbour, every
    // other lane at the right one (lane 63 keeps it for the last deferred element), so their
    // loads overlap the first row's instead of waiting behind a lane-divergent branch
    const double2 xd = op.xd_at(s.lane == 0 ? s.lb + (int64_t)r0 * 128 - 1 : s.lb + (int64_t)r1 * 128);
    const double zedge = xd.x + op.alpha * xd.y;
    double zedge_c[LBK_VF_NA], pzc[LBK_VF_NA], zfc[LBK_VF_NA];
#pragma unroll
    for (int j = 0; j < LBK_VF_NA; ++j) {
        zedge_c[j] = xd.x + op.ac[j] * xd.y;
        pzc[j] = 0.0;
    }
    double zl = zedge;
    double pz_m = 0.0, pz_c = 0.0, px = 0.0, pg = 0.0;  // lane 63: deferred element of the previous row
    int64_t pi = 0, pe = 0;
    bool pvalid = false;
    for (int row = r0; row < r1; ++row) {
        const int64_t o = (int64_t)row * 128 + 2 * s.lane;
        typename Op::Row r;
        op.load(r, s.lb + o);
        const double zfirst = __shfl(r.z.x, 0, 64);
#pragma unroll
        for (int j = 0; j < LBK_VF_NA; ++j) zfc[j] = __shfl(r.zc[j].x, 0, 64);
        if (last_lane && row > r0 && pvalid) op.finish(pz_m, pz_c, zfirst, px, pg, park[s.w], pi, pe, pzc, zfc, acc);
        r.zh = zl;  // lane 0's left neighbour; lane 63's right neighbour is deferred
        const bool v0 = full || o < s.len;
        const bool v1 = !last_lane && (full || o + 1 < s.len);
        op.template apply<true>(r, s.lb + o, s.sbeg + o, v0, v1, acc);
        if (last_lane) {
            pz_m = r.z.x;
            pz_c = r.z.y;
#pragma unroll
            for (int j = 0; j < LBK_VF_NA; ++j) pzc[j] = r.zc[j].y;
            px = r.x.y;
            pg = r.g.y;
            op.park(r, park[s.w]);
            pi = s.lb + o + 1;
            pe = s.sbeg + o + 1;
            pvalid = full || o + 1 < s.len;
        }
        zl = __shfl(r.z.y, 63, 64);
    }
    if (last_lane && pvalid) op.finish(pz_m, pz_c, zedge, px, pg, park[s.w], pi, pe, pzc, zedge_c, acc);
}

// (Two forms that stream the next row's basis by LDS-DMA while the current row computes were
// measured slower, 1.7 % and 7 %, and removed: DESIGN.md §4.4, profiles/r04/vf_dma_ab/.)
template <int OBJ, int HB, bool NT>
__global__ __launch_bounds__(LB_BLOCK) void k_vf_commit(OpVfCommit<OBJ, HB, NT> op, Geo geo, Red red) {
    constexpr int K = OpVfCommit<OBJ, HB, NT>::K;
    const Seg s = seg_setup(geo);
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    stream_vf(op, s, geo, acc);
    reduce_publish<K>(acc, geo, red);
}

// materialised d over [0, n_loc) (the rejected-first-trial path; same formula as the commit)
template <int HB, bool NT>
__global__ __launch_bounds__(256) void k_vf_dir(double* __restrict__ d, const double* __restrict__ g, VfBasis<HB> B,
                                                int64_t n_loc) {
    const int64_t npair = n_loc >> 1;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npair; p += stride) {
        const int64_t i = 2 * p;
        double2 v = make_double2(0.0, 0.0);
#pragma unroll
        for (int l = 0; l < 2 * HB; ++l) {
            if (l < 2 * B.h) {
                const double2 b = ldv<NT>(B.b[l] + i);
                if (l == 0) {
                    v.x = B.c[0] * b.x;
                    v.y = B.c[0] * b.y;
                } else {
                    v.x = v.x + B.c[l] * b.x;
                    v.y = v.y + B.c[l] * b.y;
                }
            }
        }
        const double2 gv = ldv<NT>(g + i);
        if (B.h == 0) {
            v.x = B.cg * gv.x;
            v.y = B.cg * gv.y;
        } else {
            v.x = v.x + B.cg * gv.x;
            v.y = v.y + B.cg * gv.y;
        }
        stv<NT>(d + i, v);
    }
    if ((n_loc & 1) && blockIdx.x == 0 && threadIdx.x == 0) d[n_loc - 1] = vf_dir1<HB>(B, g, n_loc - 1);
    if (blockIdx.x == 0 && threadIdx.x == 1) {  // ghost cells (sharded: the neighbours' d, from basis ghosts)
        d[-1] = vf_dir1<HB>(B, g, -1);
        d[n_loc] = vf_dir1<HB>(B, g, n_loc);
    }
}

// sharded vector-free: publish this rank's edge values of x, g, s, y (s, y may be null) into the
// wide slot's spare components, to be all-gathered with the reductions
__global__ void k_vf_edges(double* __restrict__ slot, const double* __restrict__ x, const double* __restrict__ g,
                           const double* __restrict__ s, const double* __restrict__ y, int64_t n_loc, int g_lo,
                           int g_hi) {
    if (threadIdx.x != 0) return;
    const double* v[4] = {x, g, s, y};
    for (int k = 0; k < 4; ++k) {
        slot[g_lo * LBK_KW + LBK_VF_EDGE0 + k] = v[k] ? v[k][0] : 0.0;
        slot[(g_hi - 1) * LBK_KW + LBK_VF_EDGE1 + k] = v[k] ? v[k][n_loc - 1] : 0.0;
    }
}

// ... and after the all-gather, the neighbours' edges into this rank's ghost cells
__global__ void k_vf_ghosts(const double* __restrict__ slot, double* x, double* g, double* s, double* y, int64_t n_loc,
                            int g_lo, int g_hi, int has_left, int has_right) {
    if (threadIdx.x != 0) return;
    double* v[4] = {x, g, s, y};
    for (int k = 0; k < 4; ++k) {
        if (!v[k]) continue;
        if (has_left) v[k][-1] = slot[(g_lo - 1) * LBK_KW + LBK_VF_EDGE1 + k];
        if (has_right) v[k][n_loc] = slot[g_hi * LBK_KW + LBK_VF_EDGE0 + k];
    }
}

// ---------------------------------------------------------------------------------------
// Arguments of the one-launch iterations (the cooperative iteration k_coop_iter, the device line
// search k_coop_search and the persistent forms): the two-loop recursion and the fused first-trial
// commit of one iteration in ONE launch. (A single-workgroup form for the smallest n measured 1.8x
// slower at n = 1e4 than the launch sequence, profiles/r01/small_persistent.txt, and was removed.)
// ---------------------------------------------------------------------------------------
#define LBK_SMALL_HMAX 16

struct SmallArgs {
    int h, p0_from_slot;
    const double* g;
    double* q;
    double* r;
    const double* S[LBK_SMALL_HMAX];
    const double* Y[LBK_SMALL_HMAX];
    double rho[LBK_SMALL_HMAX];
    double gamma, a0;
    double cand;            // cooperative commit: also f at x + cand d (component FC)
    const double* p0_slot;  // previous commit's slot, component SG (p0_from_slot)
    const double* x;
    double *xn, *gn, *so, *yo;
    double* slots;          // slot base (LBK_SLOT doubles per slot)
    double* hslots;         // host mirror base, or nullptr
    int slot_p0, slot_a0, slot_b0, slot_c;
    // cooperative form (k_coop_iter) only
    unsigned long long* ll;       // flagged partials [pass parity][LBK_LL_COMPS][LBK_LL_SEGS][2]
    unsigned seq_base;            // pass p of this launch is tagged seq_base + p + 1 (monotonic)
    unsigned* err;                // pinned: set on a barrier timeout
    unsigned long long timeout;   // wall-clock ticks
    // completion record for the host (pinned, nullptr: none): rec = [(epoch << 1) | went, rho
    // bits, gamma bits], then *done = epoch once block 0's commit results are in the mirror
    unsigned long long epoch;
    unsigned long long* done;
    unsigned long long* rec;
    // speculative launch (lbk_spec): the prologue's tests (spec_ok) on the previous commit slot
    int spec, spec_ls;
    const double* prev_c;
    double spec_fx, spec_c1, spec_c2, spec_tol;
    unsigned long long* vd;             // device verdict word of this launch ((epoch << 1) | went)
    const unsigned long long* chain;    // the previous speculative launch's verdict word, or nullptr
    unsigned long long chain_want;
    // persistent forms (k_persist_iter, k_persist_twoloop) only: segments per workgroup (chunks;
    // 0: strided ownership), alternate the walk direction by pass, the canonical stage 2's
    // partials and per-group arrival counters (segments, monotonic over passes), the group values
    // as flagged words [pass parity][component][group][2]
    int64_t spw;
    int alt;
    double* partials;
    unsigned long long* pcnt;
    unsigned long long* gflag;
};

__device__ __forceinline__ Seg seg_at(const Geo& geo, int64_t sidx, int tq) {
    Seg s;
    s.sbeg = sidx * geo.L;
    const int64_t send = min(s.sbeg + geo.L, geo.n);
    s.len = send - s.sbeg;
    s.lb = s.sbeg - geo.elem_lo;
    s.lane = tq & 63;
    s.w = tq >> 6;
    const int nrow_tot = (int)((s.len + 127) / 128);
    s.nrows = nrow_tot > s.w ? (nrow_tot - s.w + 3) / 4 : 0;
    return s;
}

#define HS(sl) (a.hslots ? a.hslots + (int64_t)(sl) * LBK_SLOT : nullptr)  // host-fetched slots only
// ---------------------------------------------------------------------------------------
// Cooperative iteration for small n (the persistent-block two-loop of SURVEY §7 step 5): one
// workgroup per canonical segment (nseg <= LBK_COOP_SEGMAX, all resident), the whole two-loop
// and the fused first-trial commit of one iteration in ONE launch, with an in-launch grid
// barrier between passes instead of a kernel boundary plus a stage-2 kernel:
//   * each workgroup streams its segment exactly as the pass kernel would, stores its partial
//     write-through (sc1), drains, and adds to a monotonic agent-scope arrival counter;
//   * after the counter shows every workgroup of the pass, every workgroup loads the <= 64
//     partials with sc1 loads and forms the same fixed-order total (group tree + "+ 0.0"
//     levels, then the 8-group sum) - no last arriver, no second launch;
//   * partials are double-buffered by pass parity (a workgroup can be at most one pass ahead);
//   * vectors stay per segment (pass i+1 of a segment reads what the same waves wrote in pass i);
//     the commit's stencil halo across segments reads the last r pass's published edge values.
// A barrier that waits past its timeout sets *err (pinned host memory) instead of hanging.
// ---------------------------------------------------------------------------------------
#define LBK_COOP_SEGMAX 512  // one group; resident at 2 workgroups per CU
static_assert(LBK_COOP_SEGMAX <= LBK_LL_SEGS, "flagged partials cover every cooperative segment");

// component k of a slot: group 0 holds the total's tree, groups 1..7 are empty (+0.0), written
// explicitly so that every reader - the host's fixed-order sum of the mirror, slot_total() of a
// later launch - sums the same eight values
__device__ __forceinline__ void coop_store_total(double* slot, double* hslot, int k, double q0) {
#pragma unroll
    for (int g = 0; g < LBK_GROUPS; ++g) {
        slot[g * LBK_KMAX + k] = g == 0 ? q0 : 0.0;
        if (hslot) hslot[g * LBK_KMAX + k] = g == 0 ? q0 : 0.0;
    }
}

// The prologue of a speculative launch (lbk_spec): the host decisions between the previous
// iteration and this one, restated on the previous commit's totals with the host's expressions
// (lbfgs_driver.c iterate(), ls_*; -ffp-contract=off on both sides, IEEE division and square
// root), so that the launch runs exactly when the host would have made it:
//   * g.d < 0: no fallback to the gradient direction (lbfgs.cpp:146-153);
//   * the line search takes a0 at its first trial (line_search.cpp:19-30, 57-121, 125-189, 33-55);
//   * a0 >= 1e-10 (no line-search failure, lbfgs.cpp:164-168) and s.y > 0 (the pair is stored,
//     :182-191);
//   * |g_new| >= tol (the next iteration does not stop, :80-84);
//   * rho = 1 / s.y finite and gamma = s.y / y.y finite and > 0 (:102-118).
// rg = {rho, gamma} of the new pair.
__device__ __forceinline__ int spec_ok(const SmallArgs& a, double (&rg)[2]) {
    if (a.chain && __hip_atomic_load(a.chain, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != a.chain_want) return 0;
    const double* p = a.prev_c;
    const double gd = slot_total(p + LBK_C_GD), ft = slot_total(p + LBK_C_F), dphi = slot_total(p + LBK_C_DPHI);
    const double sy = slot_total(p + LBK_C_SY), yy = slot_total(p + LBK_C_YY), gg = slot_total(p + LBK_C_GG);
    const double fx = a.spec_fx, al = a.a0, c1 = a.spec_c1, c2 = a.spec_c2;
    rg[0] = 1.0 / sy;
    rg[1] = sy / yy;
    int take = 1;
    if (a.spec_ls < 0) {  // the previous commit's step was already decided by the host
    } else if (gd >= 0) {
        return 0;
    } else switch (a.spec_ls) {
        case 0: take = !(fx - ft < c1 * al * gd); break;                                 // backtracking
        case 1: take = ft <= fx + c1 * al * gd; break;                                    // interpolation
        case 2: take = !(ft > fx + c1 * al * gd) && fabs(dphi) <= -c2 * gd; break;        // Wolfe
        default: take = !(ft > fx + c1 * al * gd) && !(dphi < c2 * gd); break;           // backtracking Wolfe
    }
    if (!take || (a.spec_ls >= 0 && al < 1e-10) || !(sy > 0)) return 0;
    if (sqrt(gg) < a.spec_tol) return 0;
    if (!isfinite(rg[0]) || rg[1] <= 0 || !isfinite(rg[1])) return 0;
    return 1;
}

// block 0: the host-visible record, then the completion word (every wave's mirror stores are
// complete before the word is written)
__device__ __forceinline__ void coop_publish(const SmallArgs& a, int went, double rho, double gamma) {
    if (blockIdx.x != 0 || !a.done) return;
    if (threadIdx.x == 0) {
        __hip_atomic_store(a.rec + 1, dbits(rho), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.rec + 2, dbits(gamma), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.rec, (a.epoch << 1) | (unsigned long long)went, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(a.done, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Returns false (uniformly over the workgroup) when one of its waits timed out or found another
// workgroup's time-out (ll_load): the totals are then NaN and the caller leaves the launch.
template <int K, class Op>
__device__ __forceinline__ bool coop_pass(const Op& op, const Geo& geo, const SmallArgs& a, int pass,
                                          double* slot, double* hslot, const double* rvec, double (&tot)[K],
                                          double (&lds)[4][8], double (&tl)[8]) {
    static_assert(K + 2 <= LBK_LL_COMPS, "flagged components");
    __shared__ int wg_failed;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) wg_failed = 0;  // read after two barriers below
    bool failed = false;
    const int64_t b = blockIdx.x;
    const Seg s = seg_setup(geo);
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    stream(op, s, geo, acc);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const double v = wave_sum(acc[k]);
        if (lane == 0) lds[w][k] = v;
    }
    // this pass's vector stores are read by other waves of the workgroup in the next pass
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const unsigned seq = a.seq_base + (unsigned)pass + 1u;
    unsigned long long* P = a.ll + (size_t)(pass & 1) * LBK_LL_COMPS * LBK_LL_SEGS * 2;
    if (t == 0) {  // the segment partial(s), and for an r pass the segment's first / last r
#pragma unroll
        for (int k = 0; k < K; ++k)
            ll_store(P + ((int64_t)k * LBK_LL_SEGS + b) * 2, (lds[0][k] + lds[1][k]) + (lds[2][k] + lds[3][k]), seq);
        if (rvec) {
            ll_store(P + ((int64_t)K * LBK_LL_SEGS + b) * 2, rvec[s.lb], seq);
            ll_store(P + ((int64_t)(K + 1) * LBK_LL_SEGS + b) * 2, rvec[s.lb + s.len - 1], seq);
        }
    }
    // every workgroup: the fixed-order totals of this pass (the group tree of stage 2, then the
    // 8-group sum with groups 1..7 empty), each thread waiting for the words it reads
    if (geo.nseg <= 64) {  // wave w: components w, w + 4; lane j: entry j (the small-group form)
#pragma unroll
        for (int k = w; k < K; k += 4) {
            const double p =
                lane < geo.nseg ? ll_load(P + ((int64_t)k * LBK_LL_SEGS + lane) * 2, seq, a.err, a.timeout, failed) : 0.0;
            const double q0 = wave_sum(p) + 0.0;  // group 0: the tree's levels above 64 add 0.0
            if (lane == 0) {
                double tt = q0;
#pragma unroll
                for (int g = 1; g < LBK_GROUPS; ++g) tt = tt + 0.0;
                tl[k] = tt;
                if (b == 0 && slot) coop_store_total(slot, hslot, k, q0);
            }
        }
    } else {  // the general form: thread t entries 4t..4t+3, wave butterfly, ((w0+w1)+(w2+w3))
        double p[K][4];
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int j = 4 * t + i;
                p[k][i] = j < geo.nseg ? ll_load(P + ((int64_t)k * LBK_LL_SEGS + j) * 2, seq, a.err, a.timeout, failed)
                                       : 0.0;
            }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double q = wave_sum((p[k][0] + p[k][1]) + (p[k][2] + p[k][3]));
            if (lane == 0) lds[w][k] = q;
        }
        __syncthreads();
        if (t < K) {
            const double q0 = (lds[0][t] + lds[1][t]) + (lds[2][t] + lds[3][t]);
            double tt = q0;
#pragma unroll
            for (int g = 1; g < LBK_GROUPS; ++g) tt = tt + 0.0;
            tl[t] = tt;
            if (b == 0 && slot) coop_store_total(slot, hslot, t, q0);
        }
    }
    if (failed) wg_failed = 1;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) tot[k] = tl[k];
    const bool ok = wg_failed == 0;
    __syncthreads();  // lds / tl / wg_failed reuse by the next pass
    return ok;
}

#define SL(sl) (a.slots + (int64_t)(sl) * LBK_SLOT)
template <int OBJ>
__global__ __launch_bounds__(LB_BLOCK) void k_coop_iter(SmallArgs a, Geo geo) {
    __shared__ double lds[4][8];
    __shared__ double tl[8];
    __shared__ double TA[LBK_SMALL_HMAX], TB[LBK_SMALL_HMAX];
    __shared__ double spec_rg[2];
    __shared__ int spec_went;
    const int h = a.h;
    int pass = 0;
    double t1[1];
    double rho_top = a.rho[h - 1], gamma = a.gamma;
    if (a.spec) {  // every workgroup evaluates the same tests on the same slot: all go or none
        if (threadIdx.x == 0) {
            double rg[2];
            spec_went = spec_ok(a, rg);
            spec_rg[0] = rg[0];
            spec_rg[1] = rg[1];
            if (blockIdx.x == 0)
                __hip_atomic_store(a.vd, (a.epoch << 1) | (unsigned long long)spec_went, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!spec_went) {
            coop_publish(a, 0, spec_rg[0], spec_rg[1]);
            return;
        }
        rho_top = spec_rg[0];
        gamma = spec_rg[1];
    }
    // alpha_{h-1} = rho_{h-1} (s_{h-1} . g): from the previous commit (SG) or a dot pass
    if (a.p0_from_slot)
        t1[0] = slot_total(a.p0_slot);
    else
        coop_pass<1>(OpDot<false>{a.S[h - 1], a.g}, geo, a, pass++, SL(a.slot_p0), nullptr, nullptr, t1, lds, tl);
    if (threadIdx.x == 0) TA[h - 1] = t1[0];
    double alpha = rho_top * t1[0];
    const double* qsrc = a.g;
    for (int i = h - 2; i >= 0; --i) {  // q = q - alpha_{i+1} y_{i+1};  s_i . q
        coop_pass<1>(OpAxpyDot<false>{a.q, qsrc, a.Y[i + 1], a.S[i], alpha}, geo, a, pass++, SL(a.slot_a0 + i),
                     nullptr, nullptr, t1, lds, tl);
        if (threadIdx.x == 0) TA[i] = t1[0];
        alpha = a.rho[i] * t1[0];
        qsrc = a.q;
    }
    coop_pass<1>(OpMid<false>{a.r, qsrc, a.Y[0], alpha, gamma}, geo, a, pass++, SL(a.slot_b0), nullptr,
                 h == 1 ? a.r : nullptr, t1, lds, tl);
    if (threadIdx.x == 0) TB[0] = t1[0];
    __syncthreads();
    for (int i = 0; i + 1 < h; ++i) {  // r += s_i (alpha_i - beta_i);  y_{i+1} . r
        const double beta = a.rho[i] * TB[i];
        const double alph = a.rho[i] * TA[i];
        coop_pass<1>(OpAxpy2Dot<false>{a.r, a.r, a.S[i], a.Y[i + 1], alph - beta}, geo, a, pass++,
                     SL(a.slot_b0 + i + 1), nullptr, i + 2 == h ? a.r : nullptr, t1, lds, tl);
        if (threadIdx.x == 0) TB[i + 1] = t1[0];
        __syncthreads();
    }
    // the last second-loop update, the first trial at a0 and the commit (k_commit TWOLOOP)
    // the halo of d across segments: the last r pass's (pass - 1) flagged edge words
    const int rp = pass - 1;
    DirArgs da = {a.r, a.S[h - 1], a.g, 0.0, nullptr, nullptr, rho_top, nullptr, geo.g_lo, geo.g_hi,
                  a.ll + (size_t)(rp & 1) * LBK_LL_COMPS * LBK_LL_SEGS * 2, geo.L, a.seq_base + (unsigned)rp + 1u, a.err,
                  a.timeout};
    {
        const double beta = rho_top * TB[h - 1];
        const double alph = rho_top * TA[h - 1];
        da.coef = alph - beta;
    }
    double t8[8];
    coop_pass<8>(OpCommit<OBJ, LBK_D_TWOLOOP, false, true>{a.x, da, a.a0, a.xn, a.gn, a.so, a.yo, geo.n, geo.n_loc,
                                                           a.cand},
                 geo, a, pass++, SL(a.slot_c), HS(a.slot_c), nullptr, t8, lds, tl);
    coop_publish(a, 1, rho_top, gamma);
}
#undef SL

// ---------------------------------------------------------------------------------------
// Device-resident line searches for small n (lbfgs_driver.c ls_backtracking,
// ls_interpolation, ls_wolfe, ls_backtracking_wolfe = line_search.cpp:19-30, 57-121, 125-189,
// 33-55): once the host's search needs a trial pass, the rest of the search runs in ONE cooperative
// launch - one workgroup per canonical segment, all resident, each trial a grid-wide pass of the
// k_trials arithmetic (the f-only searches: f at the host's batched halving chain of
// LBK_TRIALS_NC steps; the Wolfe searches: f and g(x + a d) . d at one step) whose fixed-order
// totals every workgroup forms (coop_pass), and the search's decisions restated on them in every
// workgroup with the host's expressions (-ffp-contract=off on both sides; IEEE division and square
// root), so all workgroups take the same branches and the step is the host's bit for bit. The
// host's caches are restated too (the commit's first trial, the backtracking commit's f at the
// next step, the last trial pass), so the launch evaluates exactly the passes the host loop would
// and leaves the same cache behind. A search that ends at another step than the commit's first
// trial is followed, in the same launch, by the commit at that step (the D_BUF commit of k_commit,
// into the host-read commit slot): no second launch and no host round trip for the recommit.
// Its flagged partials have their own buffer and sequence numbers, apart from the cooperative
// iteration's, whose counter a dropped speculative launch rolls back.
// ---------------------------------------------------------------------------------------
struct SearchCommit {
    const double* g;
    double *xn, *gn, *so, *yo;
    double* slot;   // device slot, or nullptr: no commit
    double* hslot;  // its host mirror (direct fetch), or nullptr
};

__device__ __forceinline__ double wolfe_cubic(double a0, double a1, double p0, double dp0, double p1, double dp1) {
    const double d1 = dp0 + dp1 - 3 * (p1 - p0) / (a1 - a0);  // line_search.cpp:8-12
    const double d2 = copysign(sqrt(d1 * d1 - dp0 * dp1), a1 - a0);
    return a0 + (a1 - a0) * (dp0 + d2 - d1) / (dp0 - dp1 + 2 * d2);
}
__device__ __forceinline__ double search_quad(double a0, double p0, double dp0, double p1) {  // :14-16
    return a0 - 0.5 * dp0 * a0 * a0 / (p1 - p0 - dp0 * a0);
}

template <int OBJ, int LS>
__global__ __launch_bounds__(LB_BLOCK) void k_coop_search(SmallArgs a, Geo geo, lbk_search s, const double* x,
                                                          const double* d, SearchCommit cm, lbk_search* out) {
    __shared__ double lds[4][8];
    __shared__ double tl[8];
    constexpr bool FG = LS == 2 || LS == 3;  // Wolfe searches: f and g.d per pass (want_dphi)
    constexpr int NC = LBK_TRIALS_NC;
    DirArgs da = {d, nullptr, nullptr, 0.0, nullptr, nullptr, 0.0, nullptr, geo.g_lo, geo.g_hi};
    int pass = 0;
    // a grid barrier of this workgroup timed out (or found another's time-out): no further pass and
    // no commit; the host sees the error flag, ignores *out and redoes the search on its loop
    bool broken = false;
    // lbfgs_driver.c trial() / trial_batched() for a device objective: the caches, else one pass;
    // false: the launch's pass budget is spent (the state stays at the top of this iteration), or
    // the grid broke apart
    auto trial = [&](double alpha, bool need_g, double& f, double& dphi) -> bool {
        if (s.have_spec && alpha == s.spec_a) {
            f = s.spec_f;
            dphi = s.spec_dphi;
            return true;
        }
        if (!need_g && s.have_cand && alpha == s.cand_a) {
            f = s.cand_f;
            return true;
        }
        for (int j = 0; j < s.tc_n; ++j)
            if (alpha == s.tc_a[j] && (!need_g || (j == 0 && s.tc_dphi_ok))) {
                f = s.tc_f[j];
                dphi = s.tc_dphi;
                return true;
            }
        if (pass >= LBK_SEARCH_PASSES || broken) return false;
        if (FG) {
            OpTrials<OBJ, LBK_D_BUF, 1, true, false> op{x, da, {alpha}, geo.n, geo.n_loc};
            double t[2];
            if (!coop_pass<2>(op, geo, a, pass++, nullptr, nullptr, nullptr, t, lds, tl)) {
                broken = true;
                return false;
            }
            s.tc_n = 1;
            s.tc_a[0] = alpha;
            s.tc_f[0] = t[0];
            s.tc_dphi = t[1];
            s.tc_dphi_ok = 1;
            s.passes_fg++;
            f = t[0];
            dphi = t[1];
        } else {
            const double ratio = LS == 0 ? s.beta : 0.5;  // the search's halving chain
            OpTrials<OBJ, LBK_D_BUF, NC, false, false> op{x, da, {}, geo.n, geo.n_loc};
            op.a[0] = alpha;
#pragma unroll
            for (int j = 1; j < NC; ++j) op.a[j] = op.a[j - 1] * ratio;
            double t[NC];
            if (!coop_pass<NC>(op, geo, a, pass++, nullptr, nullptr, nullptr, t, lds, tl)) {
                broken = true;
                return false;
            }
            s.tc_n = NC;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                s.tc_a[j] = op.a[j];
                s.tc_f[j] = t[j];
            }
            s.tc_dphi = 0.0;
            s.tc_dphi_ok = 0;
            s.passes_f++;
            f = t[0];
        }
        return true;
    };
    auto finish = [&](double step) {
        s.done = 1;
        s.step = step;
    };
    double alpha = s.alpha;
    if (LS == 0) {  // ls_backtracking
        for (;;) {
            double ft, dd;
            if (!trial(alpha, false, ft, dd)) break;
            if (!(s.f_x - ft < s.c1 * alpha * s.gd)) {
                finish(alpha);
                break;
            }
            alpha *= s.beta;
            if (alpha < s.tol) {
                finish(alpha);
                break;
            }
        }
    } else if (LS == 1) {  // ls_interpolation (iter: the loop counter before its `it++ < 20` test)
        double alpha_prev = s.alpha_prev, f_prev = s.f_prev;
        int it = s.iter;
        for (;;) {
            if (!(it++ < 20)) {
                finish(alpha);
                break;
            }
            double f_new, dd;
            if (!trial(alpha, false, f_new, dd)) {
                --it;
                break;
            }
            if (f_new <= s.f_x + s.c1 * alpha * s.gd) {
                finish(alpha);
                break;
            }
            if (alpha < s.amin) {
                finish(s.amin);
                break;
            }
            if (alpha_prev > 0) {
                const double delta = alpha - alpha_prev;
                if (fabs(delta) < 1e-10) {
                    alpha *= 0.5;
                } else {
                    const double ga = (f_new - s.f_x - s.gd * alpha) / (alpha * alpha);
                    alpha = wolfe_cubic(alpha_prev, alpha, f_prev, s.gd, f_new, ga);
                    if (alpha < 0.1 * alpha_prev || alpha > 0.9 * alpha_prev) alpha = alpha_prev * 0.5;
                }
            } else {
                alpha = search_quad(alpha, f_new, s.gd, s.f_x);
                if (alpha < 0.1 * s.init || alpha > 0.9 * s.init) alpha = s.init * 0.5;
            }
            alpha_prev = alpha;
            f_prev = f_new;
        }
        s.alpha_prev = alpha_prev;
        s.f_prev = f_prev;
        s.iter = it;
    } else if (LS == 2) {  // ls_wolfe
        double lo = s.alpha_lo, hi = s.alpha_hi, f_lo = s.f_lo, dphi_lo = s.dphi_lo;
        int iter = s.iter;
        for (;;) {
            if (iter >= 20) {
                finish(alpha);
                break;
            }
            double f_new, dphi_new;
            if (!trial(alpha, false, f_new, dphi_new)) break;
            if (f_new > s.f_x + s.c1 * alpha * s.gd || (f_new >= f_lo && iter > 0)) {
                hi = alpha;
                alpha = wolfe_cubic(lo, hi, f_lo, dphi_lo, f_new, (f_new - s.f_x - s.gd * alpha) / (alpha * alpha));
                ++iter;
                continue;
            }
            trial(alpha, true, f_new, dphi_new);  // the same pass's g.d (cached: want_dphi)
            if (fabs(dphi_new) <= -s.c2 * s.gd) {
                finish(alpha);
                break;
            }
            if (dphi_new >= 0) {
                hi = alpha;
                alpha = wolfe_cubic(lo, hi, f_lo, dphi_lo, f_new, dphi_new);
            } else {
                lo = alpha;
                f_lo = f_new;
                dphi_lo = dphi_new;
                if (hi == INFINITY)
                    alpha *= 2;
                else
                    alpha = wolfe_cubic(lo, hi, f_lo, dphi_lo, f_new, dphi_new);
            }
            if (alpha < s.amin) {
                finish(s.amin);
                break;
            }
            ++iter;
        }
        s.alpha_lo = lo;
        s.alpha_hi = hi;
        s.f_lo = f_lo;
        s.dphi_lo = dphi_lo;
        s.iter = iter;
    } else {  // ls_backtracking_wolfe
        for (;;) {
            double fn, dphi;
            if (!trial(alpha, true, fn, dphi)) break;
            if (fn > s.f_x + s.c1 * alpha * s.gd) {
                alpha *= s.beta;
            } else if (dphi < s.c2 * s.gd) {
                alpha *= 1.1;
            } else {
                finish(alpha);
                break;
            }
            if (alpha < s.tol) {
                finish(alpha);
                break;
            }
        }
    }
    s.alpha = alpha;
    // the commit at the decided step (lbfgs_driver.c commit(), D_BUF, cand 0), unless the commit
    // already taken was at that step
    // (a workgroup whose barriers all completed can still reach this pass while another one timed
    // out at the last trial barrier; it then writes its own segments of xn, gn, s and y, which is
    // why the host's redo commits again even at the first trial's step, recommit_a0)
    if (!broken && s.done && cm.slot && !(s.have_spec && s.step == s.spec_a)) {
        DirArgs dc = {d, nullptr, cm.g, 0.0, nullptr, nullptr, 0.0, nullptr, geo.g_lo, geo.g_hi};
        double t7[7];
        coop_pass<7>(OpCommit<OBJ, LBK_D_BUF, false>{x, dc, s.step, cm.xn, cm.gn, cm.so, cm.yo, geo.n, geo.n_loc,
                                                      0.0},
                     geo, a, pass++, cm.slot, cm.hslot, nullptr, t7, lds, tl);
        s.committed = 1;
    }
    // block 0: the search state, then the completion word the host polls (lbk_search_dev): block 0
    // leaves only after every barrier of the launch completed or failed, and a failure has set the
    // error flag before this word
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) *out = s;
        if (a.done) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_store(a.done, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ---------------------------------------------------------------------------------------
// Persistent forms for large n (LBFGS_PERSIST=1: the whole iteration, k_persist_iter;
// LBFGS_PERSIST=2: the two-loop, k_persist_twoloop; VERDICT r02 item 8, the north star's
// "persistent-block fused two-loop" at configs[2]'s size): one resident grid of G workgroups
// instead of one workgroup per segment. Workgroup b owns a contiguous chunk of spw canonical
// segments of every vector (LBFGS_PERSIST_OWN=stride: the segments b, b + G, b + 2G, ..., so the
// live segments form one window as in the launch sequence; measured slower) and walks them in
// every pass exactly as the pass kernels walk one segment (the same waves the same rows), storing
// each segment partial write-through; a workgroup only ever reads back rows it wrote itself.
// Passes with odd sequence numbers walk the owned segments last to first, so a workgroup starts
// on the segment it touched last, still in the Infinity Cache (the LBFGS_REV effect; A/B
// LBFGS_PERSIST_ALT=0). After its segments, thread g < 8 of the workgroup adds its
// segment count in group g to the group's agent-scope counter (monotonic: after pass seq it
// holds seq * segments-in-group); the arrival that completes a group forms its canonical stage-2
// tree (group_tree, the same bits as k_group_reduce) and publishes the group values as flagged
// words. Every workgroup then waits for the 8 group words of each component and forms the
// fixed-order total. The pass boundaries and stage-2 launches of the launch sequence become one
// counter round trip plus one flagged hop per pass.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t ceil_pos(int64_t x, int64_t y) { return x <= 0 ? 0 : (x + y - 1) / y; }
// persist_pass: one workgroup barrier per pass instead of two per owned segment (A/B: -DLBK_PERSIST_SEGBAR=1)
#ifndef LBK_PERSIST_SEGBAR
#define LBK_PERSIST_SEGBAR 0
#endif
constexpr int kPersistSegMax = 64;

template <int K, bool HALO, class Op>
__device__ __forceinline__ void persist_pass(const Op& op, const Geo& geo, const SmallArgs& a, int pass, double* slot,
                                             double* hslot, const double* rvec, double (&tot)[K],
                                             double (&lds)[4][8], double (&gv)[8][8], int (&last)[8]) {
    static_assert(K + 2 <= LBK_LL_COMPS && K <= 8, "flagged components");
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t G = gridDim.x, b = blockIdx.x;
    // owned segments: chunk [c0, c0 + cnt) (a.spw > 0), or b, b + G, ... (a.spw == 0)
    const int64_t c0 = a.spw > 0 ? min(geo.nseg, b * a.spw) : 0;
    const int64_t cnt = a.spw > 0 ? min(geo.nseg, c0 + a.spw) - c0 : (b < geo.nseg ? (geo.nseg - 1 - b) / G + 1 : 0);
    const unsigned seq = a.seq_base + (unsigned)pass + 1u;
    const bool down = (seq & 1u) != 0 && a.alt;
    unsigned long long* P = a.ll + (size_t)(pass & 1) * LBK_LL_COMPS * LBK_LL_SEGS * 2;
    // a single-component pass without halos or edges: each wave keeps its segment sums in LDS and
    // the workgroup meets once after all its segments, instead of twice per segment (the waves read
    // back only rows they wrote themselves); the same partials, the same bits
    __shared__ double segp[kPersistSegMax][4];
    const bool one_bar = !LBK_PERSIST_SEGBAR && K == 1 && !HALO && rvec == nullptr && cnt <= kPersistSegMax;
    for (int64_t k = 0; k < cnt; ++k) {
        const int64_t kk = down ? cnt - 1 - k : k;
        const int64_t sidx = a.spw > 0 ? c0 + kk : b + kk * G;
        const Seg s = seg_at(geo, sidx, t);
        double acc[K];
#pragma unroll
        for (int k2 = 0; k2 < K; ++k2) acc[k2] = 0.0;
        if constexpr (HALO)
            stream_halo(op, s, geo, acc);
        else
            stream(op, s, geo, acc);
        if (one_bar) {
            const double v = wave_sum(acc[0]);
            if (lane == 0) segp[kk][w] = v;
            continue;
        }
#pragma unroll
        for (int k2 = 0; k2 < K; ++k2) {
            const double v = wave_sum(acc[k2]);
            if (lane == 0) lds[w][k2] = v;
        }
        // this segment's vector stores are read by other waves of the workgroup (its edge r below,
        // the next pass)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (t == 0) {
#pragma unroll
            for (int k2 = 0; k2 < K; ++k2)
                __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.partials + (int64_t)k2 * LBK_SEGS + sidx),
                                   dbits((lds[0][k2] + lds[1][k2]) + (lds[2][k2] + lds[3][k2])), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            if (rvec) {  // the segment's first / last r for the commit's halo across segments
                ll_store(P + ((int64_t)K * LBK_LL_SEGS + sidx) * 2, rvec[s.lb], seq);
                ll_store(P + ((int64_t)(K + 1) * LBK_LL_SEGS + sidx) * 2, rvec[s.lb + s.len - 1], seq);
            }
        }
        __syncthreads();  // lds reuse
    }
    if (one_bar) {
        __syncthreads();
        if (t < cnt) {  // (cnt <= 64: wave 0)
            const int64_t sidx = a.spw > 0 ? c0 + t : b + (int64_t)t * G;
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.partials + sidx),
                               dbits((segp[t][0] + segp[t][1]) + (segp[t][2] + segp[t][3])), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // wave 0 stored the partials: drained before its counter adds
    if (t < 64) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (t < LBK_GROUPS) {
        const int64_t glo = (int64_t)t * LBK_SEG_PER_GROUP, ghi = min(geo.nseg, glo + LBK_SEG_PER_GROUP);
        const int64_t c = ghi <= glo       ? 0
                          : a.spw > 0      ? max((int64_t)0, min(c0 + cnt, ghi) - max(c0, glo))
                                           : ceil_pos(ghi - b, G) - ceil_pos(glo - b, G);
        int fl = 0;
        if (c > 0) {
            const unsigned long long old =
                __hip_atomic_fetch_add(a.pcnt + t, (unsigned long long)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            fl = old + (unsigned long long)c == (unsigned long long)seq * (unsigned long long)(ghi - glo);
        }
        last[t] = fl;
    }
    __syncthreads();
    for (int g = 0; g < LBK_GROUPS; ++g) {
        if (!last[g]) continue;  // uniform: shared
        // stage 2 of group g, then its values as flagged words
        __shared__ double glds[4][K];
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double* sg = slot + g * LBK_KMAX;
        group_tree<K, true>(a.partials, (int64_t)g * LBK_SEG_PER_GROUP, (int64_t)g * LBK_SEG_PER_GROUP, geo.nseg,
                            LBK_SEG_PER_GROUP, sg, hslot ? hslot + g * LBK_KMAX : nullptr, glds);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (t < K) ll_store(a.gflag + ((size_t)((pass & 1) * 8 + t) * 8 + g) * 2, sg[t], seq);
    }
    // every workgroup: the group values (groups without segments are the slot's 0.0), then the
    // fixed-order total of slot_total()
    const int ng = (int)((geo.nseg + LBK_SEG_PER_GROUP - 1) / LBK_SEG_PER_GROUP);
    if (t < K * 8) {
        const int k2 = t >> 3, gg = t & 7;
        gv[k2][gg] = gg < ng ? ll_load(a.gflag + ((size_t)((pass & 1) * 8 + k2) * 8 + gg) * 2, seq, a.err, a.timeout)
                             : 0.0;
    }
    __syncthreads();
    if (t < K) {
        double tt = gv[t][0];
#pragma unroll
        for (int q = 1; q < LBK_GROUPS; ++q) tt = tt + gv[t][q];
        if (blockIdx.x == 0) {
#pragma unroll
            for (int q = 0; q < LBK_GROUPS; ++q) {
                slot[q * LBK_KMAX + t] = gv[t][q];
                if (hslot) hslot[q * LBK_KMAX + t] = gv[t][q];
            }
        }
        lds[0][t] = tt;
    }
    __syncthreads();
#pragma unroll
    for (int k2 = 0; k2 < K; ++k2) tot[k2] = lds[0][k2];
    __syncthreads();  // lds / gv reuse by the next pass
}

// the persistent passes stream k_mid's pass in op_unroll's default 4-row groups: the launch form's
// 8-row groups would set the whole persistent kernel's register budget
template <bool NT>
struct OpMid4 : OpMid<NT> {};

#define SL(sl) (a.slots + (int64_t)(sl) * LBK_SLOT)
// The two-loop recursion of k_persist_iter (passes P0, the h - 1 first-loop passes, mid and the
// h - 1 second-loop passes); EDGES: the r passes also publish the segments' edge r for an
// in-launch commit. Returns the number of passes run; TA / TB hold the two loops' dots.
template <bool NT, bool EDGES>
__device__ __forceinline__ int persist_twoloop(const SmallArgs& a, const Geo& geo, double (&lds)[4][8],
                                               double (&gv)[8][8], double* TA, double* TB, int (&last_flag)[8]) {
    const int h = a.h;
    int pass = 0;
    double t1[1];
    const double rho_top = a.rho[h - 1], gamma = a.gamma;
    if (a.p0_from_slot)
        t1[0] = slot_total(a.p0_slot);
    else
        persist_pass<1, false>(OpDot<NT>{a.S[h - 1], a.g}, geo, a, pass++, SL(a.slot_p0), nullptr, nullptr, t1, lds,
                               gv, last_flag);
    if (threadIdx.x == 0) TA[h - 1] = t1[0];
    double alpha = rho_top * t1[0];
    const double* qsrc = a.g;
    for (int i = h - 2; i >= 0; --i) {  // q = q - alpha_{i+1} y_{i+1};  s_i . q
        persist_pass<1, false>(OpAxpyDot<NT>{a.q, qsrc, a.Y[i + 1], a.S[i], alpha}, geo, a, pass++, SL(a.slot_a0 + i),
                               nullptr, nullptr, t1, lds, gv, last_flag);
        if (threadIdx.x == 0) TA[i] = t1[0];
        alpha = a.rho[i] * t1[0];
        qsrc = a.q;
    }
    persist_pass<1, false>(OpMid4<NT>{{a.r, qsrc, a.Y[0], alpha, gamma}}, geo, a, pass++, SL(a.slot_b0), nullptr,
                           EDGES && h == 1 ? a.r : nullptr, t1, lds, gv, last_flag);
    if (threadIdx.x == 0) TB[0] = t1[0];
    __syncthreads();
    for (int i = 0; i + 1 < h; ++i) {  // r += s_i (alpha_i - beta_i);  y_{i+1} . r
        const double beta = a.rho[i] * TB[i];
        const double alph = a.rho[i] * TA[i];
        persist_pass<1, false>(OpAxpy2Dot<NT>{a.r, a.r, a.S[i], a.Y[i + 1], alph - beta}, geo, a, pass++,
                               SL(a.slot_b0 + i + 1), nullptr, EDGES && i + 2 == h ? a.r : nullptr, t1, lds, gv,
                               last_flag);
        if (threadIdx.x == 0) TB[i + 1] = t1[0];
        __syncthreads();
    }
    return pass;
}

// The whole iteration in one persistent launch (LBFGS_PERSIST=1) lost its A/B at every size
// (0.95-0.97x the launch sequence at n = 1e8): compiled only into A/B variant
// builds (-DLBK_PERSIST_ITER=1, tools/build_variant.sh), not into the shipped library.
#ifndef LBK_PERSIST_ITER
#define LBK_PERSIST_ITER 0
#endif
#if LBK_PERSIST_ITER
template <int OBJ, bool NT>
__global__ __launch_bounds__(LB_BLOCK) void k_persist_iter(SmallArgs a, Geo geo) {
    __shared__ double lds[4][8];
    __shared__ double gv[8][8];
    __shared__ double TA[LBK_SMALL_HMAX], TB[LBK_SMALL_HMAX];
    __shared__ int last_flag[8];
    const int h = a.h;
    const double rho_top = a.rho[h - 1], gamma = a.gamma;
    int pass = persist_twoloop<NT, true>(a, geo, lds, gv, TA, TB, last_flag);
    const int rp = pass - 1;
    DirArgs da = {a.r, a.S[h - 1], a.g, 0.0, nullptr, nullptr, rho_top, nullptr, geo.g_lo, geo.g_hi,
                  a.ll + (size_t)(rp & 1) * LBK_LL_COMPS * LBK_LL_SEGS * 2, geo.L, a.seq_base + (unsigned)rp + 1u, a.err,
                  a.timeout};
    {
        const double beta = rho_top * TB[h - 1];
        const double alph = rho_top * TA[h - 1];
        da.coef = alph - beta;
    }
    double t8[8];
    persist_pass<8, true>(OpCommit<OBJ, LBK_D_TWOLOOP, NT, true, true>{a.x, da, a.a0, a.xn, a.gn, a.so, a.yo, geo.n,
                                                                       geo.n_loc, a.cand},
                          geo, a, pass++, SL(a.slot_c), HS(a.slot_c), nullptr, t8, lds, gv, last_flag);
    coop_publish(a, 1, rho_top, gamma);
}
#endif  // LBK_PERSIST_ITER

// The persistent two-loop alone (LBFGS_PERSIST=2; the north star's "persistent-block fused
// two-loop"): one resident grid runs all 2h (or 2h - 1) two-loop passes of an iteration, the
// m-deep s/y ring streamed by the same workgroups pass after pass, with the in-launch stage 2 of
// persist_pass; the commit follows as its own launch and reads the passes' slots as after the
// launch sequence. Without the commit's registers (162 VGPRs, 3 waves per SIMD) the grid keeps the
// two-loop passes' occupancy. Every workgroup reads only the rows it wrote itself in an earlier
// pass (same segments, same waves), so no vector data crosses workgroups inside the launch.
#ifndef LBK_PERSIST2_WAVES
#define LBK_PERSIST2_WAVES 4  // waves per SIMD the register allocation must allow
#endif
template <bool NT>
__global__ __launch_bounds__(LB_BLOCK) __attribute__((amdgpu_waves_per_eu(LBK_PERSIST2_WAVES)))
void k_persist_twoloop(SmallArgs a, Geo geo) {
    __shared__ double lds[4][8];
    __shared__ double gv[8][8];
    __shared__ double TA[LBK_SMALL_HMAX], TB[LBK_SMALL_HMAX];
    __shared__ int last_flag[8];
    (void)persist_twoloop<NT, false>(a, geo, lds, gv, TA, TB, last_flag);
}
#undef SL

// z = x + alpha d over the whole local range incl. ghosts (host-callback objectives)
__global__ void k_point(double* __restrict__ z, const double* __restrict__ x, const double* __restrict__ d,
                        double alpha, int64_t lo, int64_t hi) {
    const int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < hi) z[i] = x[i] + alpha * d[i];
}

// elementwise primitives of vector_utils.cpp:43-73 over the local range
//   op 0: out = alpha * a      (scalarProduct, :43-51)
//   op 1: out = a + b          (add, :53-63)
//   op 2: out = -a             (negative, :65-73)
//   op 3: out = a + alpha * b  (x + (alpha d), the trial point of every line search)
// out may alias a or b (the CUDA-compat loop's in-place axpys, lbfgs_driver.c iterate_cuda): each
// element is read before it is written, and no __restrict__ promises otherwise
__global__ void k_elementwise(int op, double* out, const double* a, const double* b, double alpha, int64_t n_loc) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_loc; i += (int64_t)gridDim.x * blockDim.x) {
        double v;
        switch (op) {
            case 0: v = alpha * a[i]; break;
            case 1: v = a[i] + b[i]; break;
            case 2: v = -a[i]; break;
            default: v = a[i] + alpha * b[i]; break;
        }
        out[i] = v;
    }
}

// Unfused mode (LBFGS_FLAG_UNFUSED): one elementwise kernel per BLAS-1 update, the shape of
// the reference's parallel-implementation/L-BFGS.cu:208-280 (cublasDdot / cublasDaxpy /
// cublasDscal each a launch), with every dot a separate k_dot pass. Coefficients come from the
// reduction slots on the device with the same formulas and operand order as the fused passes,
// so both modes give bit-identical iterates.
//   LBK_U_AXPY_Q  out = a - (rho T(pa)) b                       q -= alpha_i y_i  (lbfgs.cpp:133-137)
//   LBK_U_AXPY_R  out = a + b ((rho T(pa)) - (rho T(pb)))       r += s_i (alpha_i - beta) (:159-164)
//   LBK_U_SCALE   out = a * scal                                r = gamma q      (:150-154)
//   LBK_U_NEG     out = -a                                      d = -r           (:171)
//   LBK_U_SUB     out = a - b                                   s, y             (:177-178)
//   LBK_U_POINT   out = a + scal * b                            x + alpha d      (:159)
template <int OP>
__device__ __forceinline__ double upd(double a, double b, double coef) {
    if (OP == LBK_U_AXPY_Q) return a - coef * b;
    if (OP == LBK_U_AXPY_R) return a + b * coef;
    if (OP == LBK_U_SCALE) return a * coef;
    if (OP == LBK_U_NEG) return -a;
    if (OP == LBK_U_SUB) return a - b;
    return a + coef * b;
}

template <int OP, bool NT>
__global__ __launch_bounds__(256) void k_update(double* out, const double* a,  // in place: out == a
                                                const double* __restrict__ b, double rho,
                                                const double* __restrict__ pa, const double* __restrict__ pb,
                                                double scal, int64_t n_loc) {
    double coef = scal;
    if (OP == LBK_U_AXPY_Q) coef = rho * slot_total(pa);
    if (OP == LBK_U_AXPY_R) {
        const double beta = rho * slot_total(pb);
        const double alpha = rho * slot_total(pa);
        coef = alpha - beta;
    }
    const bool has_b = OP == LBK_U_AXPY_Q || OP == LBK_U_AXPY_R || OP == LBK_U_SUB || OP == LBK_U_POINT;
    const int64_t npair = n_loc >> 1;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npair; p += stride) {
        const double2 av = ldv<NT>(a + 2 * p);
        double2 bv = av;
        if (has_b) bv = ldv<NT>(b + 2 * p);
        double2 o;
        o.x = upd<OP>(av.x, bv.x, coef);
        o.y = upd<OP>(av.y, bv.y, coef);
        stv<NT>(out + 2 * p, o);
    }
    if ((n_loc & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        const int64_t i = n_loc - 1;
        out[i] = upd<OP>(a[i], has_b ? b[i] : 0.0, coef);
    }
}

// integer checksums of the bit patterns (exact in any order)
__global__ void k_checksum(const double* __restrict__ x, int64_t n_loc, int64_t elem_lo,
                           unsigned long long* out) {
    unsigned long long a = 0, b = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_loc;
         i += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long u = dbits(x[i]);
        a += u;
        b += (unsigned long long)(elem_lo + i + 1) * u;
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        a += __shfl_xor(a, m, 64);
        b += __shfl_xor(b, m, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(out, a);
        atomicAdd(out + 1, b);
    }
}

// Box probe (lbk_stream_probe; bench.py's box_copy_tbps): the two-loop passes' 3 R + 1 W stream
// in their own geometry, unroll and cache policy - k_axpy_dot's loads and store with alpha = 0, so
// q is written back unchanged and the probe can run on the solver's own buffers - and no stage 2.
// It measures what this box's HBM gives the passes' access pattern, so a bench line can be read
// against the box it ran on. The dot is kept live (a store nobody reads, almost never taken) so
// the s loads are not dropped.
template <bool NT>
__global__ __launch_bounds__(LB_BLOCK) void k_probe_stream(double* q, const double* __restrict__ y,
                                                           const double* __restrict__ sv, double alpha, Geo geo,
                                                           double* sink) {
    const Seg s = seg_setup(geo);
    double acc[1] = {0.0};
    stream(OpAxpyDot<NT>{q, q, y, sv, alpha}, s, geo, acc);
    if (acc[0] == 1.0) sink[blockIdx.x] = acc[0];
}
// The commit's 4 R + 4 W mix (lbfgs_stream_probe_variant 6): x, g, r, s read and x_new, g_new, s, y
// written with k_commit's loads, stores and cache policies (the TWOLOOP direction d = -(r + s c)),
// in the two-loop passes' row geometry, elementwise arithmetic only and no stencil, f or stage 2:
// what this box gives the commit's access pattern.
template <bool NT>
struct OpProbeCommit {
    const double* __restrict__ x;
    const double* __restrict__ g;
    const double* __restrict__ r;
    const double* __restrict__ s;
    double* __restrict__ xn;
    double* __restrict__ gn;
    double* __restrict__ so;
    double* __restrict__ yo;
    double alpha, coef;
    struct Row {
        double2 x, g, r, s;
    };
    __device__ void load(Row& w, int64_t i) const {
        w.x = ldx<NT>(x + i);
        w.g = ldx<NT>(g + i);
        w.r = ldd<NT>(r + i);
        w.s = ldv<NT>(s + i);
    }
    template <bool MASK>
    __device__ void apply(Row& w, int64_t i, int64_t, bool v0, bool v1, double (&acc)[1]) const {
        double2 d, z, sv, yv;
        d.x = -(w.r.x + w.s.x * coef);
        d.y = -(w.r.y + w.s.y * coef);
        z.x = w.x.x + alpha * d.x;
        z.y = w.x.y + alpha * d.y;
        sv.x = z.x - w.x.x;
        sv.y = z.y - w.x.y;
        yv.x = z.x - w.g.x;
        yv.y = z.y - w.g.y;
        st2x<MASK, NT>(xn + i, z, v0, v1);
        st2x<MASK, NT>(gn + i, d, v0, v1);
        st2h<MASK, NT>(so + i, sv, v0, v1);
        st2h<MASK, NT>(yo + i, yv, v0, v1);
        acc[0] = fma2<MASK>(w.g, d, acc[0], v0, v1);
    }
};
template <bool NT>
__global__ __launch_bounds__(LB_BLOCK) void k_probe_commit(OpProbeCommit<NT> op, Geo geo, double* sink) {
    const Seg s = seg_setup(geo);
    double acc[1] = {0.0};
    stream(op, s, geo, acc);
    if (acc[0] == 1.0) sink[blockIdx.x] = acc[0];
}

// Gap analysis (lbfgs_stream_probe_variant): the probe's stream with the pass's own segment
// reduction after it - reduce_publish with the given Red (a plain partial store, or the collect
// stage 2) - but no source slot read: k_axpy_dot without src_total.
template <bool NT>
__global__ __launch_bounds__(LB_BLOCK) void k_probe_stream2(double* q, const double* __restrict__ y,
                                                            const double* __restrict__ sv, double alpha, Geo geo,
                                                            Red red) {
    run_pass<OpAxpyDot<NT>, 1>(OpAxpyDot<NT>{q, q, y, sv, alpha}, geo, red);
}

}  // namespace

// =========================================================================================
// Host side of the device layer
// =========================================================================================
// Host exchange group: ranks of one process (threads, one stream each, possibly on one GPU)
// exchange the result-slot group partials through host memory instead of RCCL. Used to test
// the sharded path on a single GPU; same data layout as the RCCL all-gather.
struct lbk_group {
    int world;
    pthread_barrier_t bar;
    double table[LBK_WSLOT];
    unsigned long long ck[LBK_GROUPS][2];
};

// vector allocation modes (lbk_vec_alloc, LBFGS_VEC_ALLOC)
enum { LBK_VEC_POOL = 0, LBK_VEC_PLAIN = 1, LBK_VEC_CONTIGUOUS = 2 };
constexpr size_t kPoolMinBytes = size_t(64) << 20;

struct lbk_ctx {
    lbk_geo geo;
    int device;
    hipStream_t stream;
    double* partials;   // LBK_KMAX * LBK_SEGS
    unsigned* cnt;      // LBK_GROUPS
    double* slots;      // LBK_NSLOTS * LBK_SLOT
    double* h_slots;    // pinned mirror
    double* dh_slots;   // the mirror as the device addresses it
    double* wslots;     // LBK_NWSLOTS * LBK_WSLOT (wide slots)
    double* h_wslots;   // pinned mirror
    double* dh_wslots;
    // one rank: stage 2 writes every result slot into its pinned host mirror too, so a fetch is a
    // stream synchronisation and no copy (LBFGS_DIRECT=0: hipMemcpyAsync of the slot instead)
    int direct;
    unsigned char slot_mirror[LBK_NSLOTS + LBK_NWSLOTS];  // last write of the slot went to the mirror
    unsigned long long* d_ck;
    unsigned long long* h_ck;
    double *h_xchg, *dh_xchg;  // mapped pinned scratch (LBK_WSLOT doubles) for kernel-side small copies
    int64_t vec_doubles;  // allocation per vector
    ncclComm_t comm;
    // RCCL waits are bounded: the communicator's init (on a helper thread), every enqueue and a
    // host wait on an RCCL collective end after rccl_timeout_s (LBFGS_RCCL_TIMEOUT, 60 s) with the
    // communicator abandoned or aborted, never in a hang; rccl_hung: an aborted collective may
    // still sit on the stream, which destroy then does not wait for
    double rccl_timeout_s;
    double rccl_stall_ms;  // test hook: LBFGS_DEBUG_RCCL_STALL (rccl_debug_stall)
    double rccl_wait_s;    // ... and its bound on the host's waits on collectives (0: rccl_timeout_s)
    unsigned *stall_release_h, *stall_release_d;  // ... and its release word (pinned), set at the abort
    int rccl_hung;
    char err[256];
    // profiling
    int prof_on;
    std::vector<hipEvent_t> ev_free;
    struct Pending {
        int kind;
        hipEvent_t a, b;
        double bytes;
    };
    std::vector<Pending> pending;
    double prof_ms[LBK_K_COUNT];
    int64_t prof_n[LBK_K_COUNT];
    double prof_bytes[LBK_K_COUNT];
    double bytes_total;
    int nt;          // non-temporal streaming loads/stores
    int ghost_slot;  // sharded: slot holding the all-gathered edge d values (-1: none)
    int ticket;      // reduction mode (see reduce_publish)
    lbk_group* grp;  // emulated ranks: host exchange group (tests; NULL with RCCL)
    lbk_xgmi* xg;    // sharded, one process per GPU: peer mailboxes over xGMI (lbfgs_xgmi.hip)
    int nt_vf;       // the vector-free passes' NT policy (c->nt while they launch)
    int ticket_env;  // LBFGS_TICKET override (-1: none)
    int xg_on;       // 1: exchanges go through xg instead of RCCL
    uint64_t* d_ckslot;  // [LBK_GROUPS][2] checksum words for the peer exchange
    // LBFGS_REV=1: every other pass walks its segments last to first, so a pass starts on the
    // tail of the vector its predecessor wrote last (still in the Infinity Cache / L2)
    int rev_on, rev_par;
    // deferred stage 2 (src_total): single-component two-loop reductions with
    // coop_max < nseg <= defer_max leave their partials for the consuming pass
    int defer_max;
    // collect-mode stage 2 (kred): on, the launch being set up uses it, flagged partials, tags
    int collect_on, collect_now;
    double collect_timeout_s;  // a collector's wait before it gives up (LBFGS_COLLECT_TIMEOUT, 10 s)
    unsigned long long* coll_ll;
    unsigned coll_seq;
    int defer_now;        // the launch in progress defers its stage 2
    int defer_region;     // partials region (component) the next deferred producer writes
    int pend_slot;        // slot whose stage 2 is still pending (-1: none)
    const double* pend_part;
    int pend_taken;       // the launch in progress consumes it
    // cooperative small-n iteration (k_coop_iter): nseg <= coop_max (0: off)
    int coop_max;
    // persistent iteration for large n (LBFGS_PERSIST=1, opt-in A/B): resident workgroups, their
    // segments per pass, stage-2 counters and flagged group values
    int persist_on, persist_gmax, persist2_gmax, persist_stride, persist_alt, persist_lds;
    unsigned long long *persist_cnt, *persist_gflag;
    unsigned long long coop_ll_bytes;
    unsigned long long* coop_ll;   // flagged partials (SmallArgs::ll)
    unsigned long long coop_base;  // passes tagged so far (the next launch's sequence base)
    // device-resident line searches (k_coop_search, LBFGS_DEV_SEARCH): flagged partials and sequence
    // numbers of their own (never rolled back), the state in mapped host memory
    int dev_wolfe;
    int wolfe_max;         // their grid cap: k_coop_search's own occupancy x CUs (and coop_max)
    int coop_fallbacks;    // device searches redone on the host loop after a barrier time-out
    double search_timeout_s; // the device search's wait per grid barrier (LBFGS_SEARCH_TIMEOUT, 2 s)
    unsigned long long* wolfe_ll;
    unsigned long long wolfe_seq;
    lbk_search *wolfe_out_h, *wolfe_out_d;
    unsigned* coop_err_h;          // pinned: barrier timeout
    unsigned* coop_err_d;
    double wall_khz;
    // cooperative launches' completion records (pinned; sp_h[0] = done word, sp_h[4 + 4 e..] the
    // record of epoch e mod 4) and speculative verdicts (device, 4 words)
    unsigned long long* sp_h;
    unsigned long long* sp_dh;
    unsigned long long* sp_vd;
    unsigned long long sp_epoch;     // last epoch issued
    unsigned long long sp_base[4];   // coop_base at each epoch's launch (release on a no-go)
    double sp_bytes[4];
    int sp_spec[4];                  // the epoch's launch was speculative
    hipEvent_t xfer_ev[4];  // lbk_*_local_async completion (host-callback transfers)
    hipEvent_t mark_ev;     // lbk_mark / lbk_fetch_marked
    // ticket launches' completion words (Red::done = sp_h + 1): the epoch last issued, and per
    // slot the epoch of the launch that last wrote its mirror (0: none, fetch synchronises)
    unsigned long long s2_epoch;
    unsigned long long slot_s2[LBK_NSLOTS + LBK_NWSLOTS];
    // a slot fetch without one: k_slot_publish's epoch (sp_h[2]), the last issued
    unsigned long long pub_epoch;
    // the device line search's completion word (sp_h[3], written by k_coop_search's block 0)
    unsigned long long search_epoch;
    // host waits on the completion words (small_wait): spin-then-sleep, the last four waits' durations
    // per word, and the time slept / waits completed (lbfgs_wait_stats)
    int vec_plain_fallbacks;  // vectors the driver could not give contiguous (lbk_vec_alloc)
    int vec_mode;             // LBK_VEC_POOL (default) / _PLAIN / _CONTIGUOUS (LBFGS_VEC_ALLOC; lbk_vec_alloc)
    int vec_pooled;           // this context's vectors taken from / added to the contiguous pool
    size_t vec_pool_cap;      // bytes the process-wide pool may own (LBFGS_VEC_POOL_GB, 32 GiB)
    size_t vec_pool_min;      // smallest pooled vector (LBFGS_VEC_POOL_MIN_MB, 64 MiB)
    int wait_adaptive;
    double wait_hist[4][4];
    unsigned wait_pos[4];
    double wait_slept_s;
    unsigned long long waits;
    double *dq_A, *dq_b, *dq_t;  // dense quadratic objective (lbk_dense_set): A (n x n), b, terms
    // folded exchanges (sharded over the mailboxes; LBFGS_XGMI_FOLD=0: off): the two-loop's
    // single-component reductions travel from the producing pass straight into the consuming pass
    int fold_env;          // LBFGS_XGMI_FOLD (default 1)
    int xf_on;             // peers connected and enabled, fold on
    lbk_xgmi_fold xf;
    int xf_slot;           // slot of the last folded exchange not yet consumed (-1: none)
    unsigned xf_epoch;
    int xf_edges;          // ... whose producer also pushed its rank edges
    int xf_taken;          // the launch in progress consumes it (src_total polls the mailbox)
    int xf_gate_err;       // a shared-GPU gate launch (take_fold) failed: the next launch reports it
    unsigned long long* fold_wait;  // profiling: ticks the consumers' workgroup 0 waited (device)
    void* xfer_pool;       // staged whole-vector transfers (LBFGS_XFER=staged), lazily
    int fold_now;          // the launch in progress pushes its reduction (epoch fold_epoch)
    unsigned fold_epoch;
    int fold_edges;
    // LBFGS_CU_PARTITION (sharded, tests and one-card rehearsals): the solver stream runs on this
    // rank's own cu_count CUs, disjoint from every other rank's, as if each rank had a GPU
    int cu_part, cu_count;
};

namespace {

#define HIPCHK(c, expr)                                                                      \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) {                                                              \
            snprintf((c)->err, sizeof((c)->err), "%s:%d %s: %s", __FILE__, __LINE__, #expr, \
                     hipGetErrorString(e_));                                                 \
            return -2;                                                                       \
        }                                                                                    \
    } while (0)

Geo kgeo(const lbk_ctx* c) {
    Geo g;
    g.n = c->geo.n;
    g.L = c->geo.L;
    g.nseg = c->geo.nseg;
    g.seg_lo = c->geo.seg_lo;
    g.elem_lo = c->geo.elem_lo;
    g.n_loc = c->geo.n_loc;
    g.g_lo = c->geo.g_lo;
    g.g_hi = c->geo.g_hi;
    g.spg = LBK_SEG_PER_GROUP;
    g.rev = c->rev_on ? c->rev_par : 0;
    g.ppart = nullptr;
    g.edge_slot = nullptr;
    return g;
}

// Geometry of the vector-free commit (ORC_CANON_VF): segments of F canonical segments
// (F = lbk_geo.vf_f, a function of n only), 1024 / F of them per group, so a rank owns the same
// elements in both geometries. Short canonical segments (n <= ~1e7) leave each wave of the
// vector-free commit only 1-3 rows, and its fixed costs per segment (the two wave-run edges,
// a 4h+7-component reduction) dominate; F up to 8 restores runs of ~10 rows.
// The base length is the canonical L except for LBK_MIDL_LO <= n < LBK_VFL_LO, where the
// canonical segments are 2048 long but the vector-free commit keeps the 512-minimum length
// (measured there: 2048-element segments cost the vector-free mode 25 %, profiles/r01/lmin_ab.txt).
// Invariant: for every n that shards (world > 1) the base length equals the canonical L, so a
// rank's vector-free segments cover exactly its canonical elements (vgeo inherits elem_lo /
// n_loc from kgeo). Today n < LBK_VFL_LO never shards (lbk_geometry_plan); lbk_create checks it.
int64_t vf_base_len(int64_t n, int64_t canon_L) {
    if (n < LBK_MIDL_LO || n >= LBK_VFL_LO) return canon_L;
    const int64_t per = (n + LBK_SEGS - 1) / LBK_SEGS;
    int64_t L = ((per + 127) / 128) * 128;
    return L < 512 ? 512 : L;
}

Geo vgeo(const lbk_ctx* c) {
    Geo g = kgeo(c);
    const int F = c->geo.vf_f;
    const int64_t base = vf_base_len(c->geo.n, c->geo.L);
    if (F <= 1 && base == c->geo.L) return g;
    g.L = base * F;
    g.nseg = (c->geo.n + g.L - 1) / g.L;
    g.spg = LBK_SEG_PER_GROUP / F;
    g.seg_lo = std::min<int64_t>((int64_t)c->geo.g_lo * g.spg, g.nseg);
    return g;
}

int geo_blocks(const lbk_ctx* c, const Geo& g) {
    return (int)(std::min<int64_t>((int64_t)c->geo.g_hi * g.spg, g.nseg) - g.seg_lo);
}

// regular slots 0..LBK_NSLOTS-1 (LBK_KMAX components), wide slots LBK_WSLOT0 + w (LBK_KW)
double* slot_base(const lbk_ctx* c, int slot) {
    return slot < LBK_NSLOTS ? c->slots + (int64_t)slot * LBK_SLOT
                             : c->wslots + (int64_t)(slot - LBK_WSLOT0) * LBK_WSLOT;
}
double* slot_host(const lbk_ctx* c, int slot) {
    return slot < LBK_NSLOTS ? c->h_slots + (int64_t)slot * LBK_SLOT
                             : c->h_wslots + (int64_t)(slot - LBK_WSLOT0) * LBK_WSLOT;
}
int slot_stride(int slot) { return slot < LBK_NSLOTS ? LBK_KMAX : LBK_KW; }
// The host mirror as kernels address it, or nullptr. Mirrored: the slots the host reads back
// (multi-component reductions: commit, trials, objective; wide slots). A single-component
// two-loop reduction only feeds the next pass on the device; writing it over PCIe as well would
// hold every pass's completion behind a host-memory write (measured -6..-11 % at n = 1e6).
bool mirrored(const lbk_ctx* c, int slot, int K) { return c->direct && (K >= 2 || slot >= LBK_NSLOTS); }
double* slot_dhost(const lbk_ctx* c, int slot) {
    if (!c->direct) return nullptr;
    return slot < LBK_NSLOTS ? c->dh_slots + (int64_t)slot * LBK_SLOT
                             : c->dh_wslots + (int64_t)(slot - LBK_WSLOT0) * LBK_WSLOT;
}

Red kred(lbk_ctx* c, int slot, int K = 1) {
    Red r;
    r.partials = c->partials;
    r.cnt = c->cnt;
    r.slot = slot_base(c, slot);
    r.hslot = mirrored(c, slot, K) ? slot_dhost(c, slot) : nullptr;
    c->slot_mirror[slot < LBK_NSLOTS ? slot : LBK_NSLOTS + slot - LBK_WSLOT0] = r.hslot != nullptr;
    r.kstride = slot_stride(slot);
    r.ticket = c->ticket;
    r.done = nullptr;
    r.epoch = 0;
    r.fp = FoldPush{nullptr, 0, 0, 0, 0u};
    r.ll = nullptr;
    r.seq = 0;
    r.err = nullptr;
    r.timeout = 0;
    c->collect_now = 0;
    // collect mode (one rank, reduce-kernel stage 2 otherwise): stage 2 inside the launch, no
    // reduce kernel after it (LBFGS_COLLECT)
    // (regular slots only: a wide slot's tree would poll its up to 96 components batch by batch)
    if (c->collect_on && !r.ticket && c->geo.world == 1 && !c->comm && !c->grp && c->geo.nseg > c->coop_max &&
        K <= LBK_KMAX && slot < LBK_NSLOTS) {
        r.ll = c->coll_ll;
        r.seq = ++c->coll_seq;
        r.err = c->coop_err_d;
        r.timeout = (unsigned long long)(c->collect_timeout_s * c->wall_khz * 1e3);
        c->collect_now = 1;
    }
    const int si = slot < LBK_NSLOTS ? slot : LBK_NSLOTS + slot - LBK_WSLOT0;
    c->slot_s2[si] = 0;
    // each group's last arriver stores the word, so it stands for the whole slot only when every
    // segment is in one group (with several, the first group done would release the host early)
    if (r.ticket && r.hslot && c->geo.world == 1 && !c->comm && !c->grp && c->sp_dh &&
        c->geo.nseg <= LBK_SEG_PER_GROUP) {
        r.done = c->sp_dh + 1;
        r.epoch = ++c->s2_epoch;
        c->slot_s2[si] = r.epoch;
    }
    return r;
}

const double* sref(const lbk_ctx* c, int ref) {
    return c->slots + (int64_t)(ref / LBK_KMAX) * LBK_SLOT + (ref % LBK_KMAX);
}

int nblocks(const lbk_ctx* c) { return (int)(c->geo.seg_hi - c->geo.seg_lo); }

const double* ghost_ptr(const lbk_ctx* c) {
    if (c->geo.world <= 1 || c->ghost_slot < 0) return nullptr;
    return c->slots + (int64_t)c->ghost_slot * LBK_SLOT;
}

hipEvent_t ev_get(lbk_ctx* c) {
    if (!c->ev_free.empty()) {
        hipEvent_t e = c->ev_free.back();
        c->ev_free.pop_back();
        return e;
    }
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

int prof_flush(lbk_ctx* c) {
    for (auto& p : c->pending) {
        float ms = 0.f;
        HIPCHK(c, hipEventSynchronize(p.b));
        HIPCHK(c, hipEventElapsedTime(&ms, p.a, p.b));
        c->prof_ms[p.kind] += ms;
        c->prof_n[p.kind] += 1;
        c->prof_bytes[p.kind] += p.bytes;
        c->ev_free.push_back(p.a);
        c->ev_free.push_back(p.b);
    }
    c->pending.clear();
    return 0;
}

double mono_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

// Ends an RCCL call on the non-blocking communicator: ncclInProgress is polled through
// ncclCommGetAsyncError for at most rccl_timeout_s; a timeout or an error aborts the communicator
// (ncclCommAbort also stops its kernels) and leaves the context without one (-3, LBFGS_ERR_RCCL).
int rccl_settle(lbk_ctx* c, ncclResult_t r, const char* what) {
    const double t_end = mono_s() + c->rccl_timeout_s;
    while (r == ncclInProgress) {
        if (mono_s() > t_end) break;
        usleep(100);
        if (ncclCommGetAsyncError(c->comm, &r) != ncclSuccess) r = ncclInternalError;
    }
    if (r == ncclSuccess) return 0;
    if (r == ncclInProgress)
        snprintf(c->err, sizeof c->err, "%s: no progress in %.0f s (RCCL communicator aborted)", what, c->rccl_timeout_s);
    else
        snprintf(c->err, sizeof c->err, "%s: %s (RCCL communicator aborted)", what, ncclGetErrorString(r));
    (void)ncclCommAbort(c->comm);
    c->comm = nullptr;
    c->rccl_hung = 1;
    return -3;
}

// A host wait on the solver stream while RCCL work is queued on it: bounded like rccl_settle
int rccl_stream_wait(lbk_ctx* c, const char* what) {
    const double bound = c->rccl_wait_s > 0.0 ? c->rccl_wait_s : c->rccl_timeout_s;
    const double t_end = mono_s() + bound;
    for (;;) {
        const hipError_t e = hipStreamQuery(c->stream);
        if (e == hipSuccess) return 0;
        if (e != hipErrorNotReady) {
            snprintf(c->err, sizeof c->err, "%s: %s", what, hipGetErrorString(e));
            return -2;
        }
        if (mono_s() > t_end) break;
        usleep(50);
    }
    snprintf(c->err, sizeof c->err, "%s: the RCCL collective did not complete in %.1f s (communicator aborted)", what,
             bound);
    if (c->stall_release_h) __atomic_store_n(c->stall_release_h, 1u, __ATOMIC_RELEASE);  // test hook's stand-in
    if (c->comm) (void)ncclCommAbort(c->comm);
    c->comm = nullptr;
    c->rccl_hung = 1;
    return -3;
}

// Small copies between device memory and the context's mapped pinned scratch (h_xchg) done by a
// kernel's loads and stores, not a copy engine (the result-slot fetches likewise: k_slot_publish);
// the caller waits on the stream before the host reads the scratch.
__global__ __launch_bounds__(256) void k_copy_words(const double* __restrict__ src, double* __restrict__ dst, int n) {
    for (int i = (int)threadIdx.x; i < n; i += 256) dst[i] = src[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}
int kcopy(lbk_ctx* c, double* dst, const double* src, int n) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_copy_words, dim3(1), dim3(256), 0, c->stream, src, dst, n);
    HIPCHK(c, hipGetLastError());
    return 0;
}

// A host wait on the solver stream. With an RCCL communicator, collectives may sit on the stream,
// and a peer that dies mid-solve would leave a plain hipStreamSynchronize waiting forever: the wait
// is then bounded (rccl_stream_wait, LBFGS_RCCL_TIMEOUT) and ends in LBFGS_ERR_RCCL. Without one
// every wait on the stream is on this process's own kernels, whose in-kernel waits are bounded.
int stream_wait(lbk_ctx* c, const char* what) {
    // (after an abort, rccl_hung: the aborted collective may still sit on the stream)
    if (c->comm || c->rccl_hung) return rccl_stream_wait(c, what);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

// Test hook (LBFGS_DEBUG_RCCL_STALL="stall_ms,wait_s"): a one-thread kernel queued ahead of every
// RCCL collective that sleeps stall_ms on the device, standing in for a peer that stops answering,
// and wait_s as the bound of the host's waits on collectives; the kernel ends on its own, so the GPU
// is never held. tests/test_gpu_rccl.py sets a stall longer than the bound.
// The stand-in ends early when the host aborts the communicator (*release, pinned), as an aborted
// RCCL collective stops: the abort then finds the stream moving again, as it would on a real hang.
__global__ void k_stall(unsigned long long ticks, const unsigned* release) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks &&
           __hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u)
        __builtin_amdgcn_s_sleep(127);
}
void rccl_debug_stall(lbk_ctx* c) {
    if (c->rccl_stall_ms <= 0.0 || !c->stall_release_d) return;
    hipLaunchKernelGGL(k_stall, dim3(1), dim3(1), 0, c->stream, (unsigned long long)(c->rccl_stall_ms * c->wall_khz),
                       (const unsigned*)c->stall_release_d);
}

// Sharded runs: each rank owns groups [g_lo, g_hi) of every result slot; gather them so
// every rank holds all 8 (one RCCL all-gather of (8/world) x KMAX doubles per reduction, in
// place, on the solver stream), or through the host group for emulated ranks.
int flush_fold(lbk_ctx* c);
int exchange_buf(lbk_ctx* c, double* base, int ks, double* host_mirror = nullptr) {
    const int per = (c->geo.g_hi - c->geo.g_lo) * ks;
    if (c->xg_on) {  // a folded exchange's epoch is collected before the next one is issued
        const int rc = flush_fold(c);
        if (rc) return rc;
    }
    if (c->grp) {
        // through the rank's mapped pinned scratch, copied by kernels on the solver stream (kcopy):
        // this rank's groups out, the whole table back in, each waited for before the barrier
        lbk_group* G = c->grp;
        if (kcopy(c, c->dh_xchg, base + c->geo.g_lo * ks, per)) return -2;
        HIPCHK(c, hipStreamSynchronize(c->stream));
        memcpy(G->table + c->geo.g_lo * ks, (const void*)c->h_xchg, sizeof(double) * per);
        pthread_barrier_wait(&G->bar);
        memcpy(c->h_xchg, G->table, sizeof(double) * LBK_GROUPS * ks);
        if (kcopy(c, base, c->dh_xchg, LBK_GROUPS * ks)) return -2;
        HIPCHK(c, hipStreamSynchronize(c->stream));
        pthread_barrier_wait(&G->bar);
        return 0;
    }
    if (c->xg_on) {
        if (lbk_xgmi_exchange(c->xg, c->stream, base, ks, c->geo.g_lo, c->geo.g_hi, host_mirror) != 0) {
            snprintf(c->err, sizeof c->err, "xgmi exchange launch failed");
            return -3;
        }
        return 0;
    }
    if (!c->comm) {
        snprintf(c->err, sizeof c->err, "sharded context has no exchange backend (no RCCL id, peers not enabled)");
        return -3;
    }
    rccl_debug_stall(c);
    return rccl_settle(c, ncclAllGather(base + c->geo.g_lo * ks, base, (size_t)per, ncclDouble, c->comm, c->stream),
                       "ncclAllGather");
}

// Over the peer mailboxes the exchange kernel also completes the host mirror of the slots the
// host reads back (as the stage 2 does on one rank, see mirrored()): no device-to-host copy
// before those reads
int exchange_slot(lbk_ctx* c, int slot, int K = 1, bool host_read = true) {
    double* hm = nullptr;  // (a host-mirroring exchange measured neutral, profiles/r01/xgmi_mirror_ab.txt)
    (void)K;
    (void)host_read;
    const int rc = exchange_buf(c, slot_base(c, slot), slot_stride(slot), hm);
    c->slot_mirror[slot < LBK_NSLOTS ? slot : LBK_NSLOTS + slot - LBK_WSLOT0] = rc == 0 && hm != nullptr;
    return rc;
}

// exchange_slot bracketed by events when profiling (LBK_K_EXCHANGE: bench.py's exchange_share)
int exchange_timed(lbk_ctx* c, int slot, int K = 1, bool host_read = true) {
    hipEvent_t a = nullptr, b = nullptr;
    if (c->prof_on) {
        if (c->pending.size() > 4096 && prof_flush(c) != 0) return -2;
        a = ev_get(c);
        b = ev_get(c);
        if (a) HIPCHK(c, hipEventRecord(a, c->stream));
    }
    const int rc = exchange_slot(c, slot, K, host_read);
    if (a && b) {
        HIPCHK(c, hipEventRecord(b, c->stream));
        c->pending.push_back({LBK_K_EXCHANGE, a, b, 0.0});
    }
    return rc;
}

// Deferred partials live in the two highest components of the partials array: a consuming launch
// reads them while its own workgroups store their partials (components 0..K-1, K <= 87), and a
// deferred producer and its consumer alternate between the two.
double* defer_part(const lbk_ctx* c, int region) { return c->partials + (int64_t)(LBK_KW - 2 + region) * LBK_SEGS; }

// A folded exchange that no pass consumed (the next launch is not its consumer, or the host reads
// the slot): wait for the peers' pushes with the collect kernel (timed as an exchange). Every new
// exchange epoch is issued behind this in stream order, so a rank never pushes epoch e + 1 before
// it holds every peer's e (the mailbox parity rule).
int flush_fold(lbk_ctx* c) {
    if (c->xf_slot < 0 || c->xf_taken) return 0;
    hipEvent_t a = nullptr, b = nullptr;
    if (c->prof_on) {
        a = ev_get(c);
        b = ev_get(c);
        if (a) HIPCHK(c, hipEventRecord(a, c->stream));
    }
    const int rc = lbk_xgmi_collect(c->xg, c->stream, slot_base(c, c->xf_slot), slot_stride(c->xf_slot), c->geo.g_lo,
                                    c->geo.g_hi, c->xf_epoch, c->xf_edges);
    c->xf_slot = -1;
    if (rc) {
        snprintf(c->err, sizeof c->err, "xgmi collect launch failed");
        return -3;
    }
    if (a && b) {
        HIPCHK(c, hipEventRecord(b, c->stream));
        c->pending.push_back({LBK_K_EXCHANGE, a, b, 0.0});
    }
    return 0;
}

// a pending (deferred) stage 2 that no consumer took: run it as the reduce kernel now; the same
// for a folded exchange
int flush_pending(lbk_ctx* c) {
    {
        const int rc = flush_fold(c);
        if (rc) return rc;
    }
    if (c->pend_slot < 0) return 0;
    const Geo g = kgeo(c);
    hipLaunchKernelGGL(k_group_reduce<1>, dim3(c->geo.g_hi - c->geo.g_lo), dim3(LB_BLOCK), 0, c->stream, c->pend_part,
                       g, slot_base(c, c->pend_slot), (double*)nullptr, LBK_KMAX, FoldPush{nullptr, 0, 0, 0, 0u});
    HIPCHK(c, hipGetLastError());
    c->pend_slot = -1;
    return 0;
}

// Folded exchange, producer: this launch's single-component reduction into `slot` (and, for an r
// pass, the rank-edge values) is pushed to the peers from inside the pass; set up its Red.
void fold_producer(lbk_ctx* c, Red& r, bool edges) {
    if (!c->xf_on) return;
    r.fp = FoldPush{c->xf.peers, c->xf.positions, c->xf.world, c->xf.rank, lbk_xgmi_next_epoch(c->xg)};
    c->fold_now = 1;
    c->fold_epoch = r.fp.epoch;
    c->fold_edges = edges ? 1 : 0;
}

// Folded exchange, consumer: a launch whose first source (src_total) is the pending folded slot
// polls the mailbox for it in its prologue
FoldSrc take_fold(lbk_ctx* c, int ref) {
    FoldSrc f{nullptr, 0u, nullptr, nullptr, 0ull, nullptr};
    if (c->xf_slot < 0 || ref % LBK_KMAX != 0 || c->xf_slot != ref / LBK_KMAX) return f;
    if (c->xf.shared_device && !c->cu_part) {
        // ranks sharing one GPU (forced fold: tests, rehearsals): a consuming pass's workgroups
        // polling in its prologue can hold every CU a peer's producing pass waits for. A
        // one-wavefront gate (the collect kernel) waits first, so the pass launches with the
        // values already in the mailbox and its prologue's poll is the same code, satisfied at once.
        // With the CUs partitioned between the ranks (cu_part) no rank can hold another's CUs, so
        // there is no gate: the consumer waits in its prologue exactly as across distinct GPUs.
        hipEvent_t a = nullptr, b = nullptr;
        if (c->prof_on && (a = ev_get(c)) && (b = ev_get(c))) (void)hipEventRecord(a, c->stream);
        if (lbk_xgmi_collect(c->xg, c->stream, slot_base(c, c->xf_slot), slot_stride(c->xf_slot), c->geo.g_lo,
                             c->geo.g_hi, c->xf_epoch, 0) != 0)
            c->xf_gate_err = 1;
        if (a && b) {
            (void)hipEventRecord(b, c->stream);
            c->pending.push_back({LBK_K_EXCHANGE, a, b, 0.0});
        }
    }
    f.mbx = c->xf.own + (size_t)(c->xf_epoch & 1u) * (size_t)c->xf.positions * 2;
    f.mepoch = c->xf_epoch;
    f.merr = c->xf.err;
    f.merrd = c->xf.errd;
    f.mtmo = c->xf.timeout;
    f.wait = c->prof_on ? c->fold_wait : nullptr;
    c->xf_taken = 1;
    return f;
}

// A single-component reduction into `slot` may leave its stage 2 to the next pass (returns the
// Red to launch with; sets defer_now). Only on one rank, with the reduce-kernel stage 2, and for
// segment counts where every consumer workgroup reading all partials is cheaper than a launch.
Red kred_deferrable(lbk_ctx* c, int slot) {
    Red r = kred(c, slot);
    if (c->geo.world == 1 && !c->comm && !c->ticket && c->geo.nseg > c->coop_max && c->geo.nseg <= c->defer_max) {
        r.partials = defer_part(c, c->defer_region);
        c->defer_now = 1;
        r.ll = nullptr;  // the consumer forms the trees instead
        c->collect_now = 0;
    }
    return r;
}

// the consumer side: the partials of `ref`'s slot if its stage 2 is pending (and take it)
const double* take_pending(lbk_ctx* c, int ref) {
    if (c->pend_slot < 0 || c->pend_slot != ref / LBK_KMAX) return nullptr;
    c->pend_taken = 1;
    return c->pend_part;
}

// launch wrapper: byte accounting, optional event timing, all-gather of group partials
template <class F>
int launch(lbk_ctx* c, int kind, double vec_passes, int slot, F&& fn, int K = 1, bool exchange = true,
           const Geo* gv = nullptr) {
    if (c->xf_gate_err) {
        snprintf(c->err, sizeof c->err, "xgmi gate launch failed");
        return -3;
    }
    if (c->xf_slot >= 0 && !c->xf_taken) {
        const int rc = flush_fold(c);
        if (rc) return rc;
    }
    if (c->pend_slot >= 0 && !c->pend_taken) {
        const int rc = flush_pending(c);
        if (rc) return rc;
    }
    const double bytes = vec_passes * 8.0 * (double)c->geo.n_loc;
    c->bytes_total += bytes;
    hipEvent_t a = nullptr, b = nullptr;
    if (c->prof_on) {
        if (c->pending.size() > 4096 && prof_flush(c) != 0) return -2;
        a = ev_get(c);
        b = ev_get(c);
        if (a) HIPCHK(c, hipEventRecord(a, c->stream));
    }
    if (nblocks(c) > 0) {
        fn();
        HIPCHK(c, hipGetLastError());
        c->rev_par ^= 1;
    }
    // the pass kernel's own interval ends here; a separate stage 2 is timed as its own kind
    if (c->prof_on && a && b) {
        HIPCHK(c, hipEventRecord(b, c->stream));
        c->pending.push_back({kind, a, b, bytes});
        a = b = nullptr;
        if (slot >= 0 && !c->ticket && !c->defer_now && !c->collect_now) {
            a = ev_get(c);
            b = ev_get(c);
            if (a) HIPCHK(c, hipEventRecord(a, c->stream));
            kind = LBK_K_GROUP_REDUCE;
        }
    }
    if (c->pend_taken) {  // the consumer's workgroup 0 stored the pending slot's group values
        c->pend_slot = -1;
        c->pend_taken = 0;
    }
    if (c->xf_taken) {  // ... and the folded slot's other groups, from the mailbox
        c->xf_slot = -1;
        c->xf_taken = 0;
    }
    FoldPush fp{nullptr, 0, 0, 0, 0u};
    if (c->fold_now && !c->ticket)  // the reduce kernel's workgroups push the group values
        fp = FoldPush{c->xf.peers, c->xf.positions, c->xf.world, c->xf.rank, c->fold_epoch};
    if (c->defer_now) {
        c->pend_slot = slot;
        c->pend_part = defer_part(c, c->defer_region);
        c->defer_region ^= 1;
        c->defer_now = 0;
    } else if (slot >= 0 && !c->ticket && !c->collect_now) {
        const Geo g = gv ? *gv : kgeo(c);
        double* sl = slot_base(c, slot);
        double* hs = mirrored(c, slot, K) ? slot_dhost(c, slot) : nullptr;
        const int ks = slot_stride(slot);
        const dim3 grid(c->geo.g_hi - c->geo.g_lo), blk(LB_BLOCK);
        switch (K) {
            case 1: hipLaunchKernelGGL(k_group_reduce<1>, grid, blk, 0, c->stream, c->partials, g, sl, hs, ks, fp); break;
            case 2: hipLaunchKernelGGL(k_group_reduce<2>, grid, blk, 0, c->stream, c->partials, g, sl, hs, ks, fp); break;
            case 7: hipLaunchKernelGGL(k_group_reduce<7>, grid, blk, 0, c->stream, c->partials, g, sl, hs, ks, fp); break;
            case 8: hipLaunchKernelGGL(k_group_reduce<8>, grid, blk, 0, c->stream, c->partials, g, sl, hs, ks, fp); break;
            default:
                hipLaunchKernelGGL(k_group_reduce_wide, dim3(c->geo.g_hi - c->geo.g_lo, (K + 7) / 8), blk, 0, c->stream,
                                   c->partials, g, sl, hs, K, ks);
                break;
        }
        HIPCHK(c, hipGetLastError());
    }
    if (c->prof_on && a && b) {
        HIPCHK(c, hipEventRecord(b, c->stream));
        c->pending.push_back({kind, a, b, 0.0});
    }
    c->collect_now = 0;
    if (c->fold_now) {  // pushed by the pass (or its reduce kernel): no exchange launch
        c->xf_slot = slot;
        c->xf_epoch = c->fold_epoch;
        c->xf_edges = c->fold_edges;
        c->xf_taken = 0;
        c->fold_now = 0;
        return 0;
    }
    if (exchange && (c->geo.world > 1 || c->comm) && slot >= 0) return exchange_timed(c, slot, K);
    return 0;
}

// sharded vector-free: edges of (x, g, s, y) into the slot, all-gather, neighbours' edges into
// the ghost cells
int vf_exchange_ghosts(lbk_ctx* c, int wslot, double* x, double* g, double* s, double* y) {
    double* sl = slot_base(c, wslot);
    const lbk_geo& G = c->geo;
    hipLaunchKernelGGL(k_vf_edges, dim3(1), dim3(64), 0, c->stream, sl, x, g, s, y, G.n_loc, G.g_lo, G.g_hi);
    HIPCHK(c, hipGetLastError());
    const int rc = exchange_slot(c, wslot, 1, false);  // edges: read by k_vf_ghosts only
    if (rc) return rc;
    hipLaunchKernelGGL(k_vf_ghosts, dim3(1), dim3(64), 0, c->stream, sl, x, g, s, y, G.n_loc, G.g_lo, G.g_hi,
                       G.elem_lo > 0 ? 1 : 0, G.elem_lo + G.n_loc < G.n ? 1 : 0);
    HIPCHK(c, hipGetLastError());
    return 0;
}

}  // namespace

#define NT_DISPATCH(c, ...)                            \
    do {                                               \
        if ((c)->nt) {                                 \
            constexpr bool NT_ = true;                 \
            __VA_ARGS__;                               \
        } else {                                       \
            constexpr bool NT_ = false;                \
            __VA_ARGS__;                               \
        }                                              \
    } while (0)

#define OBJ_DISPATCH1(obj, ...)                                      \
    switch (obj) {                                                            \
        case LBK_OBJ_ROSENBROCK: { constexpr int O_ = LBK_OBJ_ROSENBROCK; __VA_ARGS__; } break;         \
        case LBK_OBJ_QUAD_TRIDIAG: { constexpr int O_ = LBK_OBJ_QUAD_TRIDIAG; __VA_ARGS__; } break;     \
        case LBK_OBJ_QUAD_SEPARABLE: { constexpr int O_ = LBK_OBJ_QUAD_SEPARABLE; __VA_ARGS__; } break; \
        default: return -1;                                                   \
    }

#define OBJ_DISPATCH(obj, ...)                             \
    if (c->nt) {                                           \
        constexpr bool NT_ = true;                         \
        OBJ_DISPATCH1(obj, __VA_ARGS__);                   \
    } else {                                               \
        constexpr bool NT_ = false;                        \
        OBJ_DISPATCH1(obj, __VA_ARGS__);                   \
    }

