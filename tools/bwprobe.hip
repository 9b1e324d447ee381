// tools/bwprobe.hip — HBM bandwidth calibration on MI355X for the solver's access mixes.
// Streams fp64 vectors of n elements with 16-B loads (double2) and reports GB/s (algorithmic
// bytes / kernel time, HIP events, median of reps) for:
//   read1   : sum(a)                          1R
//   copy    : b = a                           1R 1W
//   r3w1    : q = q - c*y; acc += s.q         3R 1W   (the two-loop pass mix)
//   r3w1_nt : same with non-temporal loads/stores
//   r4w4    : the commit mix (x,d,g read, halo; 4 writes) approximated as 3R 4W
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bwprobe tools/bwprobe.hip
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

template <bool NT>
__device__ __forceinline__ double2 ld(const double* p) {
    if (NT) {
        double2 v;
        v.x = __builtin_nontemporal_load(p);
        v.y = __builtin_nontemporal_load(p + 1);
        return v;
    }
    return *reinterpret_cast<const double2*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(double* p, double2 v) {
    if (NT) {
        __builtin_nontemporal_store(v.x, p);
        __builtin_nontemporal_store(v.y, p + 1);
    } else {
        *reinterpret_cast<double2*>(p) = v;
    }
}

__global__ void k_read1(const double* __restrict__ a, int64_t n2, double* out) {
    double acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
        double2 v = ld<false>(a + 2 * i);
        acc += v.x + v.y;
    }
    if (acc == 12345.678) out[0] = acc;
}

__global__ void k_copy(const double* __restrict__ a, double* __restrict__ b, int64_t n2) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x)
        st<false>(b + 2 * i, ld<false>(a + 2 * i));
}

template <bool NT, int U>
__global__ void k_r3w1(double* q, const double* __restrict__ y, const double* __restrict__ s, double c, int64_t n2,
                       double* out) {
    double acc = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n2; i += U * stride) {
        double2 qv[U], yv[U], sv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            qv[j] = ld<NT>(q + 2 * (i + j * stride));
            yv[j] = ld<NT>(y + 2 * (i + j * stride));
            sv[j] = ld<NT>(s + 2 * (i + j * stride));
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            double2 r;
            r.x = qv[j].x - c * yv[j].x;
            r.y = qv[j].y - c * yv[j].y;
            st<NT>(q + 2 * (i + j * stride), r);
            acc = fma(sv[j].x, r.x, acc);
            acc = fma(sv[j].y, r.y, acc);
        }
    }
    for (; i < n2; i += stride) {
        double2 qv = ld<NT>(q + 2 * i), yv = ld<NT>(y + 2 * i), sv = ld<NT>(s + 2 * i);
        double2 r;
        r.x = qv.x - c * yv.x;
        r.y = qv.y - c * yv.y;
        st<NT>(q + 2 * i, r);
        acc = fma(sv.x, r.x, fma(sv.y, r.y, acc));
    }
    if (acc == 12345.678) out[0] = acc;
}

__global__ void k_r3w4(const double* __restrict__ x, const double* __restrict__ d, const double* __restrict__ g,
                       double* __restrict__ xn, double* __restrict__ gn, double* __restrict__ so,
                       double* __restrict__ yo, int64_t n2) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
        double2 xv = ld<false>(x + 2 * i), dv = ld<false>(d + 2 * i), gv = ld<false>(g + 2 * i);
        double2 z, gg, s, y;
        z.x = xv.x + dv.x; z.y = xv.y + dv.y;
        gg.x = z.x * z.x; gg.y = z.y * z.y;
        s.x = z.x - xv.x; s.y = z.y - xv.y;
        y.x = gg.x - gv.x; y.y = gg.y - gv.y;
        st<false>(xn + 2 * i, z);
        st<false>(gn + 2 * i, gg);
        st<false>(so + 2 * i, s);
        st<false>(yo + 2 * i, y);
    }
}

// segment-style (the solver's layout): block b owns [b*L, (b+1)*L), rows of 128 elements
// interleaved over its 4 waves, U rows in flight per wave
template <bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void k_seg_r3w1(double* q, const double* __restrict__ y, const double* __restrict__ s,
                                                  double c, int64_t n, int64_t L, double* out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * L;
    const int nrows = (int)(L / 512);
    double acc = 0;
    for (int u0 = 0; u0 < nrows; u0 += U) {
        double2 qv[U], yv[U], sv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = base + (int64_t)(4 * (u0 + j) + w) * 128 + 2 * lane;
            if (u0 + j < nrows && i < n) { qv[j] = ld<NTL>(q + i); yv[j] = ld<NTL>(y + i); sv[j] = ld<NTL>(s + i); }
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = base + (int64_t)(4 * (u0 + j) + w) * 128 + 2 * lane;
            if (u0 + j < nrows && i < n) {
                double2 r;
                r.x = qv[j].x - c * yv[j].x;
                r.y = qv[j].y - c * yv[j].y;
                st<NTS>(q + i, r);
                acc = fma(sv[j].x, r.x, acc);
                acc = fma(sv[j].y, r.y, acc);
            }
        }
    }
    if (acc == 12345.678) out[0] = acc;
}

// the solver's pass shape with S segments of length L per workgroup, rows interleaved over 4
// waves, NT loads/stores, optional ticket tail (wave sums -> LDS -> atomic add), to price
// the per-workgroup reduction tail and the workgroup granularity
template <bool TICKET>
__global__ __launch_bounds__(256) void k_segS(double* q, const double* __restrict__ y, const double* __restrict__ s,
                                              double c, int64_t n, int64_t L, int S, double* part, unsigned* cnt) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __shared__ double lds[4][8];
    __shared__ int last;
    for (int k = 0; k < S; ++k) {
        const int64_t base = ((int64_t)blockIdx.x * S + k) * L;
        const int nrows_tot = (int)(L / 128);
        double acc = 0;
        int u0 = 0;
        for (; 4 * (u0 + 3) + w < nrows_tot; u0 += 4) {
            double2 qv[4], yv[4], sv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t i = base + (int64_t)(4 * (u0 + j) + w) * 128 + 2 * lane;
                if (i < n) { qv[j] = ld<true>(q + i); yv[j] = ld<true>(y + i); sv[j] = ld<true>(s + i); }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t i = base + (int64_t)(4 * (u0 + j) + w) * 128 + 2 * lane;
                if (i < n) {
                    double2 r;
                    r.x = qv[j].x - c * yv[j].x;
                    r.y = qv[j].y - c * yv[j].y;
                    st<true>(q + i, r);
                    acc = fma(sv[j].x, r.x, fma(sv[j].y, r.y, acc));
                }
            }
        }
        for (; 4 * u0 + w < nrows_tot; ++u0) {
            const int64_t i = base + (int64_t)(4 * u0 + w) * 128 + 2 * lane;
            if (i < n) {
                double2 qv = ld<true>(q + i), yv = ld<true>(y + i), sv = ld<true>(s + i);
                double2 r;
                r.x = qv.x - c * yv.x;
                r.y = qv.y - c * yv.y;
                st<true>(q + i, r);
                acc = fma(sv.x, r.x, fma(sv.y, r.y, acc));
            }
        }
        if (TICKET) {
            for (int m = 1; m < 64; m <<= 1) acc += __shfl_xor(acc, m, 64);
            if (lane == 0) lds[w][k & 7] = acc;
        }
    }
    if (TICKET) {
        __syncthreads();
        if (threadIdx.x < S) {
            const int k = threadIdx.x;
            const double p = (lds[0][k] + lds[1][k]) + (lds[2][k] + lds[3][k]);
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(part + (int64_t)blockIdx.x * S + k),
                               (unsigned long long)__double_as_longlong(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (threadIdx.x == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            unsigned old = __hip_atomic_fetch_add(cnt + (blockIdx.x & 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = (old == 0xffffffffu);
        }
        __syncthreads();
        if (last) part[0] = 1.0;
    }
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000LL;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int64_t n2 = n / 2;
    std::vector<double*> v(8);
    for (auto& p : v) {
        CK(hipMalloc(&p, n * sizeof(double)));
        CK(hipMemset(p, 0, n * sizeof(double)));
    }
    double* out;
    CK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int ncu = 256;
    auto run = [&](const char* name, double vecs, int grid, auto launch) {
        std::vector<float> t;
        for (int r = 0; r < reps + 2; ++r) {
            CK(hipEventRecord(a));
            launch(grid);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        double ms = t[t.size() / 2];
        printf("%-22s grid %6d  %8.3f ms  %7.1f GB/s\n", name, grid, ms, vecs * 8.0 * n / (ms * 1e-3) / 1e9);
    };
    for (int grid : {ncu * 4, ncu * 8}) {
        run("read1", 1, grid, [&](int gr) { hipLaunchKernelGGL(k_read1, dim3(gr), dim3(256), 0, 0, v[0], n2, out); });
        run("copy", 2, grid, [&](int gr) { hipLaunchKernelGGL(k_copy, dim3(gr), dim3(256), 0, 0, v[0], v[1], n2); });
        run("r3w1_u1", 4, grid, [&](int gr) { hipLaunchKernelGGL((k_r3w1<false, 1>), dim3(gr), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, n2, out); });
        run("r3w1_u4", 4, grid, [&](int gr) { hipLaunchKernelGGL((k_r3w1<false, 4>), dim3(gr), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, n2, out); });
        run("r3w1_nt4", 4, grid, [&](int gr) { hipLaunchKernelGGL((k_r3w1<true, 4>), dim3(gr), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, n2, out); });
        run("r3w4", 7, grid, [&](int gr) { hipLaunchKernelGGL(k_r3w4, dim3(gr), dim3(256), 0, 0, v[0], v[1], v[2], v[3], v[4], v[5], v[6], n2); });
    }
    // segment-style with L = 12288 (the solver's n=1e8 geometry) and array offsets
    const int64_t L = 12288;
    const int nb = (int)((n + L - 1) / L);
    for (int64_t pad : {(int64_t)0, (int64_t)4096 + 256, (int64_t)65536 + 1024, (int64_t)(1 << 21) + 4096}) {
        double* slab;
        const int64_t stride = ((n * 8 + 255) / 256) * 256 + pad;  // bytes between arrays
        CK(hipMalloc(&slab, 3 * stride + 4096));
        CK(hipMemset(slab, 0, 3 * stride + 4096));
        double* q = slab;
        double* y = (double*)((char*)slab + stride);
        double* sv = (double*)((char*)slab + 2 * stride);
        char nm[64];
        snprintf(nm, sizeof nm, "seg_u4 p%lld", (long long)pad);
        run(nm, 4, nb, [&](int gr) { hipLaunchKernelGGL((k_seg_r3w1<false, false, 4>), dim3(gr), dim3(256), 0, 0, q, y, sv, 0.5, n, L, out); });
        snprintf(nm, sizeof nm, "seg_u2 p%lld", (long long)pad);
        run(nm, 4, nb, [&](int gr) { hipLaunchKernelGGL((k_seg_r3w1<false, false, 2>), dim3(gr), dim3(256), 0, 0, q, y, sv, 0.5, n, L, out); });
        snprintf(nm, sizeof nm, "seg_ntl p%lld", (long long)pad);
        run(nm, 4, nb, [&](int gr) { hipLaunchKernelGGL((k_seg_r3w1<true, false, 4>), dim3(gr), dim3(256), 0, 0, q, y, sv, 0.5, n, L, out); });
        snprintf(nm, sizeof nm, "seg_nts p%lld", (long long)pad);
        run(nm, 4, nb, [&](int gr) { hipLaunchKernelGGL((k_seg_r3w1<false, true, 4>), dim3(gr), dim3(256), 0, 0, q, y, sv, 0.5, n, L, out); });
        snprintf(nm, sizeof nm, "seg_nt2 p%lld", (long long)pad);
        run(nm, 4, nb, [&](int gr) { hipLaunchKernelGGL((k_seg_r3w1<true, true, 4>), dim3(gr), dim3(256), 0, 0, q, y, sv, 0.5, n, L, out); });
        CK(hipFree(slab));
    }
    // workgroup granularity and ticket tail at the solver's geometry for this n
    {
        double* part;
        unsigned* cnt;
        CK(hipMalloc(&part, 8192 * 8 * sizeof(double)));
        CK(hipMalloc(&cnt, 64));
        CK(hipMemset(cnt, 0, 64));
        int64_t per = (n + 8191) / 8192;
        int64_t Lc = std::max<int64_t>(512, ((per + 127) / 128) * 128);
        int64_t nseg = (n + Lc - 1) / Lc;
        for (int S : {1, 2, 4, 8}) {
            int nbS = (int)((nseg + S - 1) / S);
            char nm[64];
            snprintf(nm, sizeof nm, "segS%d_L%lld_nt", S, (long long)Lc);
            run(nm, 4, nbS, [&](int gr) { hipLaunchKernelGGL((k_segS<false>), dim3(gr), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, n, Lc, S, part, cnt); });
            snprintf(nm, sizeof nm, "segS%d_L%lld_ticket", S, (long long)Lc);
            run(nm, 4, nbS, [&](int gr) { hipLaunchKernelGGL((k_segS<true>), dim3(gr), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, n, Lc, S, part, cnt); });
        }
    }
    // larger segments (fewer, longer-lived blocks)
    for (int64_t L2 : {(int64_t)49152, (int64_t)196608}) {
        const int nb2 = (int)((n + L2 - 1) / L2);
        char nm[64];
        snprintf(nm, sizeof nm, "seg_L%lld", (long long)L2);
        run(nm, 4, nb2, [&](int gr) { hipLaunchKernelGGL((k_seg_r3w1<false, false, 4>), dim3(gr), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, n, L2, out); });
    }
    return 0;
}
