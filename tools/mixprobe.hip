// tools/mixprobe.hip — the HBM ceiling of each read/write mix the solver's passes stream, measured
// in the passes' OWN access pattern (is k_commit's 4R + 4W, k_vf_commit's
// 22R + 4W or k_mid's 2R + 1W at the chip's ceiling for that mix, or is there headroom?).
//
// Geometry exactly as the product's pass kernels (lbfgs_kernels_impl.h stream()): one 256-thread
// workgroup per canonical segment of L elements, wave w visits rows 4u + w of 128 elements, lane l
// the two elements 2l, 2l + 1 (one 16-B load per vector), U rows of every vector loaded before the
// first use, no masks (n a multiple of 128 here). Per element: the NR loaded values are summed, one
// product goes into a dot accumulator (so no load is dead), and NW distinct values are stored.
// Policies per operand class: non-temporal (nt) or default, for loads and stores separately; the
// store order (all stores of a row together, or interleaved with the next row's loads) is a variant.
//
// Reports algorithmic GB/s = (NR + NW) * 8 * n / kernel time (HIP events, median of 15 reps, one
// warm-up), n = 1e8 (configs[2]: 800 MB per vector, far beyond the 256 MiB Infinity Cache).
// "_alt" cases walk the segments in the opposite direction on every other rep, as the product's
// consecutive passes do (LBFGS_REV): a rep then starts on the tail the previous rep touched last.
// Above n = 4e8 only the cases with at most 4 inputs run (8 vectors of 8n bytes are allocated).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mixprobe tools/mixprobe.hip
// Run:   tools/mixprobe [n]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

#define MAXV 24
struct Vecs {
    const double* in[MAXV];
    double* out[MAXV];
    const double* pair;  // IL > 0: inputs 1 and 2 share this buffer, alternating blocks of IL rows
};

typedef double dvec2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ dvec2 ld(const double* p) {
    if (NT) return __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(p));
    return *reinterpret_cast<const dvec2*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(double* p, dvec2 v) {
    if (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(p));
    else
        *reinterpret_cast<dvec2*>(p) = v;
}

// LNT / SNT: nt loads / stores; the first TWL inputs and the first TWS outputs (the "work"
// vectors q / r / d of the product) keep the default policy; INPL: output 0 is input 0 (in place,
// as the two-loop's q); IL > 0: inputs 1 and 2 (the two-loop's s_i and y_{i+1}) are one stream,
// blocks of IL rows of 128 elements alternating between them
// RUN: wave w takes the contiguous rows [w R, (w + 1) R), R = ceil(rows / 4) (the vector-free
// commit's ORC_CANON_VF walk) instead of rows 4u + w
// TAIL: the end of a product pass's workgroup (reduce_publish): 1 - wave butterflies, the four wave
// sums through LDS, a barrier and one plain store of the segment's partial; 2 - the same with the
// partial stored write-through at agent scope (the ticket / collect forms' stores)
template <int NR, int NW, int U, bool LNT, bool SNT, int TWL, int TWS, bool INPL, int IL = 0, bool RUN = false,
          int TAIL = 0>
__global__ __launch_bounds__(256) void k_mix(Vecs v, int64_t n, int64_t L, int rev, double* sink) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t seg = rev ? (int64_t)gridDim.x - 1 - blockIdx.x : blockIdx.x;
    const int64_t sbeg0 = seg * L;
    const int64_t len = min(L, n - sbeg0);
    const int nrows = (int)(len / 128);
    const int R = (nrows + 3) / 4;
    const int myrows = RUN ? max(0, min(R, nrows - w * R)) : (nrows > w ? (nrows - w + 3) / 4 : 0);
    const int64_t sbeg = sbeg0;
    double acc = 0.0;
    for (int u0 = 0; u0 < myrows; u0 += U) {
        dvec2 a[U][NR];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            if (u0 + j >= myrows) break;
            const int64_t off = sbeg + (RUN ? (int64_t)(w * R + u0 + j) : (int64_t)(4 * (u0 + j) + w)) * 128 + 2 * lane;
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                if (IL > 0 && (k == 1 || k == 2)) {
                    const int64_t grow = off / 128;
                    const int64_t ioff = ((grow / IL) * 2 * IL + (k - 1) * IL + grow % IL) * 128 + 2 * lane;
                    a[j][k] = ld<LNT>(v.pair + ioff);
                } else {
                    a[j][k] = (k < TWL) ? ld<false>(v.in[k] + off) : ld<LNT>(v.in[k] + off);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            if (u0 + j >= myrows) break;
            const int64_t off = sbeg + (RUN ? (int64_t)(w * R + u0 + j) : (int64_t)(4 * (u0 + j) + w)) * 128 + 2 * lane;
            dvec2 s = a[j][0];
#pragma unroll
            for (int k = 1; k < NR; ++k) s = s + a[j][k];
            acc = fma(s.x, a[j][0].x, fma(s.y, a[j][0].y, acc));
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                const dvec2 o = s + (double)(k + 1);
                double* dst = (INPL && k == 0) ? const_cast<double*>(v.in[0]) : v.out[k];
                if (k < TWS)
                    st<false>(dst + off, o);
                else
                    st<SNT>(dst + off, o);
            }
        }
    }
    if constexpr (TAIL > 0) {
        __shared__ double wl[4];
        double a = acc;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) a += __shfl_xor(a, m, 64);
        if (lane == 0) wl[w] = a;
        __syncthreads();
        if (threadIdx.x == 0) {
            const double p = (wl[0] + wl[1]) + (wl[2] + wl[3]);
            if (TAIL == 1)
                sink[seg] = p;
            else
                __hip_atomic_store(reinterpret_cast<unsigned long long*>(sink + seg), __double_as_longlong(p),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else {
        if (acc == 1234.5678) sink[0] = acc;
    }
}

struct Case {
    const char* name;
    int nr, nw;
    void (*launch)(Vecs, int64_t, int64_t, int, int, double*);
    bool alt;
};

// LDSK > 0: LDSK KiB of dynamic LDS per workgroup (caps the workgroups per CU: 60 KiB -> 2, the
// vector-free commit's occupancy of 2 waves per SIMD)
template <int NR, int NW, int U, bool LNT, bool SNT, int TWL, int TWS, bool INPL, int IL = 0, bool RUN = false,
          int LDSK = 0, int TAIL = 0>
void launch(Vecs v, int64_t n, int64_t L, int nseg, int rev, double* sink) {
    hipLaunchKernelGGL((k_mix<NR, NW, U, LNT, SNT, TWL, TWS, INPL, IL, RUN, TAIL>), dim3(nseg), dim3(256), LDSK * 1024, 0, v,
                       n, L, rev, sink);
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? (int64_t)atof(argv[1]) : 100000000;
    // the canonical segment length at this n: roundup(ceil(n / 8192), 128)
    const int64_t L = std::max<int64_t>(512, ((n + 8191) / 8192 + 127) / 128 * 128);
    const int nseg = (int)((n + L - 1) / L);
    const int64_t npad = (int64_t)nseg * L;
    const int maxnr = n > 400000000 ? 4 : MAXV;
    std::vector<double*> bufs(MAXV + 4, nullptr);
    for (int k = 0; k < MAXV + 4; ++k) {
        if (k >= maxnr && k < MAXV) continue;
        CK(hipMalloc(&bufs[k], sizeof(double) * npad));
        CK(hipMemset(bufs[k], 0, sizeof(double) * npad));
    }
    double* sink;
    CK(hipMalloc(&sink, std::max<size_t>(64, sizeof(double) * (size_t)nseg)));  // TAIL: one partial per segment
    double* pair;
    CK(hipMalloc(&pair, sizeof(double) * 2 * npad));
    CK(hipMemset(pair, 0, sizeof(double) * 2 * npad));
    Vecs v;
    v.pair = pair;
    for (int k = 0; k < MAXV; ++k) v.in[k] = bufs[k];
    for (int k = 0; k < MAXV; ++k) v.out[k] = bufs[MAXV + 3 - (k % 4)];  // outputs disjoint from the inputs (NW <= 4)
    // names: <R>r<W>w_u<U>_<load policy><store policy>  (nt / df = default); "work" operands as the
    // product's kernels: k_mid q (df) + y -> r (df); k_axpy_dot q (df) + y + s -> q (df, in place);
    // k_commit r (df) + x + s + g -> x' + g' + s + y; k_vf_commit 22 nt -> 4 nt
    Case cases[] = {
        {"1r0w_u4_nt", 1, 0, launch<1, 0, 4, true, true, 0, 0, false>, false},
        {"1r1w_u4_ntnt", 1, 1, launch<1, 1, 4, true, true, 0, 0, false>, false},
        {"mid_2r1w_u4", 2, 1, launch<2, 1, 4, true, true, 1, 1, false>, false},
        {"mid_2r1w_u8", 2, 1, launch<2, 1, 8, true, true, 1, 1, false>, false},
        {"axpy_3r1w_u4", 3, 1, launch<3, 1, 4, true, true, 1, 1, true>, false},
        {"3r1w_u4_allnt", 3, 1, launch<3, 1, 4, true, true, 0, 0, false>, false},
        {"commit_4r4w_u4", 4, 4, launch<4, 4, 4, true, true, 1, 0, false>, false},
        {"commit_4r4w_u2", 4, 4, launch<4, 4, 2, true, true, 1, 0, false>, false},
        {"commit_4r4w_u8", 4, 4, launch<4, 4, 8, true, true, 1, 0, false>, false},
        {"4r4w_u4_ntld_dfst", 4, 4, launch<4, 4, 4, true, false, 1, 0, false>, false},
        {"4r4w_u4_alldf", 4, 4, launch<4, 4, 4, false, false, 0, 0, false>, false},
        {"4r2w_u4", 4, 2, launch<4, 2, 4, true, true, 1, 0, false>, false},
        {"4r0w_u4", 4, 0, launch<4, 0, 4, true, true, 1, 0, false>, false},
        {"vf_22r4w_u1", 22, 4, launch<22, 4, 1, true, true, 0, 0, false>, false},
        {"vf_22r4w_u2", 22, 4, launch<22, 4, 2, true, true, 0, 0, false>, false},
        {"22r4w_u1_ntld_dfst", 22, 4, launch<22, 4, 1, true, false, 0, 0, false>, false},
        {"22r0w_u1", 22, 0, launch<22, 0, 1, true, true, 0, 0, false>, false},
        {"axpy_3r1w_u4_inpl_allnt", 3, 1, launch<3, 1, 4, true, true, 0, 0, true>, false},
        {"3r1w_u4_outpl_qdf", 3, 1, launch<3, 1, 4, true, true, 1, 1, false>, false},
        {"axpy_3r1w_u4_inpl_allnt_alt", 3, 1, launch<3, 1, 4, true, true, 0, 0, true>, true},
        {"mid_2r1w_u8_allnt", 2, 1, launch<2, 1, 8, true, true, 0, 0, false>, false},
        {"commit_4r4w_u4_allnt", 4, 4, launch<4, 4, 4, true, true, 0, 0, false>, false},
        {"mid_2r1w_u8_alt", 2, 1, launch<2, 1, 8, true, true, 1, 1, false>, true},
        {"axpy_3r1w_u4_alt", 3, 1, launch<3, 1, 4, true, true, 1, 1, true>, true},
        // the workgroup's reduction tail of the product pass (TAIL 1: plain store, 2: write-through)
        {"axpy_3r1w_u4_tail1", 3, 1, launch<3, 1, 4, true, true, 1, 1, true, 0, false, 0, 1>, false},
        {"axpy_3r1w_u4_tail2", 3, 1, launch<3, 1, 4, true, true, 1, 1, true, 0, false, 0, 2>, false},
        {"axpy_3r1w_u4_tail1_alt", 3, 1, launch<3, 1, 4, true, true, 1, 1, true, 0, false, 0, 1>, true},
        {"axpy_3r1w_u4_tail2_alt", 3, 1, launch<3, 1, 4, true, true, 1, 1, true, 0, false, 0, 2>, true},
        {"commit_4r4w_u4_alt", 4, 4, launch<4, 4, 4, true, true, 1, 0, false>, true},
        // s_i / y_{i+1} interleaved in one buffer (blocks of 1, 4, 16, 96 rows), q in place
        {"axpy_3r1w_u4_il1", 3, 1, launch<3, 1, 4, true, true, 1, 1, true, 1>, false},
        {"axpy_3r1w_u4_il4", 3, 1, launch<3, 1, 4, true, true, 1, 1, true, 4>, false},
        {"axpy_3r1w_u4_il16", 3, 1, launch<3, 1, 4, true, true, 1, 1, true, 16>, false},
        {"axpy_3r1w_u4_il96", 3, 1, launch<3, 1, 4, true, true, 1, 1, true, 96>, false},
        {"axpy_3r1w_u4_il1_alt", 3, 1, launch<3, 1, 4, true, true, 1, 1, true, 1>, true},
        {"axpy_3r1w_u4_il4_alt", 3, 1, launch<3, 1, 4, true, true, 1, 1, true, 4>, true},
        {"axpy_3r1w_u4_il1_allnt", 3, 1, launch<3, 1, 4, true, true, 0, 0, true, 1>, false},
        {"axpy_3r1w_u4_il4_allnt", 3, 1, launch<3, 1, 4, true, true, 0, 0, true, 4>, false},
        // the vector-free commit's walk (contiguous run per wave) and occupancy (2 waves / SIMD)
        {"vf_22r4w_u1_occ2", 22, 4, launch<22, 4, 1, true, true, 0, 0, false, 0, false, 60>, false},
        {"vf_22r4w_u1_run", 22, 4, launch<22, 4, 1, true, true, 0, 0, false, 0, true>, false},
        {"vf_22r4w_u1_run_occ2", 22, 4, launch<22, 4, 1, true, true, 0, 0, false, 0, true, 60>, false},
        {"vf_22r4w_u2_occ2", 22, 4, launch<22, 4, 2, true, true, 0, 0, false, 0, false, 60>, false},
        {"vf_22r4w_u2_run_occ2", 22, 4, launch<22, 4, 2, true, true, 0, 0, false, 0, true, 60>, false},
        {"vf_22r4w_u1_occ1", 22, 4, launch<22, 4, 1, true, true, 0, 0, false, 0, false, 100>, false},
        // round 4: two-loop passes in pairs (the first of a pair keeps q in registers and stores
        // nothing, the second recomputes it from the pair's source and stores q two steps on):
        // 3R + 0W then 4R + 1W move the same 8 vectors as two 3R + 1W passes with one write fewer
        {"pairA_3r0w_u4_alt", 3, 0, launch<3, 0, 4, true, true, 1, 0, false>, true},
        {"pairB_4r1w_u4_inpl_alt", 4, 1, launch<4, 1, 4, true, true, 1, 1, true>, true},
        {"pairB_4r1w_u4_outpl_alt", 4, 1, launch<4, 1, 4, true, true, 1, 1, false>, true},
        {"pairM_3r1w_u8_alt", 3, 1, launch<3, 1, 8, true, true, 1, 1, false>, true},
        {"commit5_5r4w_u4_alt", 5, 4, launch<5, 4, 4, true, true, 1, 0, false>, true},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("n=%lld L=%lld segments=%d (one 256-thread workgroup each)\n", (long long)n, (long long)L, nseg);
    for (const Case& c : cases) {
        if (c.nr > maxnr) continue;
        std::vector<float> ms;
        for (int r = 0; r < 16; ++r) {
            CK(hipEventRecord(e0, 0));
            c.launch(v, n, L, nseg, c.alt ? (r & 1) : 0, sink);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        const double gbs = (double)(c.nr + c.nw) * 8.0 * (double)n / (med * 1e-3) / 1e9;
        printf("%-28s %2dR %2dW  %9.1f us  %7.1f GB/s  (min %.1f us)\n", c.name, c.nr, c.nw, med * 1e3, gbs,
               ms.front() * 1e3);
    }
    for (auto b : bufs)
        if (b) CK(hipFree(b));
    CK(hipFree(pair));
    return 0;
}
