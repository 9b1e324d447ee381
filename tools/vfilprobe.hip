// tools/vfilprobe.hip — does the vector-free commit's 22R + 4W stream run faster when its basis
// vectors are stored interleaved row by row (k_vf_commit at 5.2-5.5 TB/s
// against 5.97-6.03 for its mix with two rows in flight)?
//
// The product's k_vf_commit loads, per 128-element row and wave, one 1-KiB row of each of 2h + 2
// = 22 vectors (x, g, s_0..s_9, y_0..y_9) and stores one row of 4 (x', g', s', y'): 26 DRAM pages
// touched per row. Stored interleaved - s_l and y_l of a pair in one buffer, alternating 128-
// element rows - the same row of a pair is one 2-KiB run. This probe streams 22R + 4W in the
// vector-free commit's geometry (one 256-thread workgroup per segment of the canonical L, each
// wave a contiguous run of rows, lane l elements 2l and 2l + 1, every load of a row issued before
// the first use, 2 waves per SIMD as the product's 252 VGPRs allow: 60 KiB of LDS per workgroup)
// with the basis in P pair buffers of RPR rows per run:
//   sep      22 separate vectors, 4 separate outputs (the product today)
//   pair2    x, g separate; 10 buffers of (s_l, y_l) alternating rows; outputs x', g' separate and
//            (s', y') alternating rows
//   quad4    x, g separate; 5 buffers of (s_l, y_l, s_l+1, y_l+1) alternating rows; outputs as pair2
// Reports algorithmic GB/s = 26 * 8 * n / time (median of 15 reps after one warm-up), n = 1e8.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/vfilprobe tools/vfilprobe.hip
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

typedef double dvec2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ dvec2 ldn(const double* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(p));
}
__device__ __forceinline__ void stn(double* p, dvec2 v) { __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(p)); }

struct Bufs {
    const double* in[22];  // RPR == 1: 22 vectors; else in[0], in[1] = x, g and in[2 + b] the b-th group buffer
    double* out[4];        // WPR == 1: 4 vectors; else out[0], out[1] plain, out[2] the (s', y') pair buffer
};

// RPR: basis vectors per group buffer (1 = separate); WPR: 1 = 4 separate outputs, 2 = s'/y' paired
template <int RPR, int WPR>
__global__ __launch_bounds__(256) void k_vfil(Bufs B, int64_t n, int64_t L, double* sink) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t sbeg = (int64_t)blockIdx.x * L;
    const int64_t len = min(L, n - sbeg);
    const int nrows = (int)(len / 128);
    const int R = (nrows + 3) / 4;
    const int r0 = w * R, r1 = min(r0 + R, nrows);
    double acc = 0.0;
    for (int row = r0; row < r1; ++row) {
        const int64_t grow = sbeg / 128 + row;  // global row
        const int64_t off = grow * 128 + 2 * lane;
        dvec2 a[22];
        a[0] = ldn(B.in[0] + off);
        a[1] = ldn(B.in[1] + off);
#pragma unroll
        for (int k = 0; k < 20; ++k) {
            if (RPR == 1) {
                a[2 + k] = ldn(B.in[2 + k] + off);
            } else {
                const int b = k / RPR, j = k % RPR;
                a[2 + k] = ldn(B.in[2 + b] + (grow * RPR + j) * 128 + 2 * lane);
            }
        }
        dvec2 s = a[0];
#pragma unroll
        for (int k = 1; k < 22; ++k) s = s + a[k];
        acc = fma(s.x, a[1].x, fma(s.y, a[1].y, acc));
        stn(B.out[0] + off, s);
        stn(B.out[1] + off, s + 1.0);
        if (WPR == 1) {
            stn(B.out[2] + off, s + 2.0);
            stn(B.out[3] + off, s + 3.0);
        } else {
            stn(B.out[2] + (grow * 2) * 128 + 2 * lane, s + 2.0);
            stn(B.out[2] + (grow * 2 + 1) * 128 + 2 * lane, s + 3.0);
        }
    }
    if (acc == 1234.5678) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? (int64_t)atof(argv[1]) : 100000000;
    const int64_t L = std::max<int64_t>(512, ((n + 8191) / 8192 + 127) / 128 * 128);
    const int nseg = (int)((n + L - 1) / L);
    const int64_t npad = (int64_t)nseg * L;
    // 22 + 4 vectors of npad doubles; grouped layouts carve their buffers out of the same memory
    std::vector<double*> v(26);
    for (auto& p : v) {
        CK(hipMalloc(&p, sizeof(double) * npad));
        CK(hipMemset(p, 0, sizeof(double) * npad));
    }
    double* sink;
    CK(hipMalloc(&sink, 64));
    // group buffers: RPR consecutive vectors' memory as one buffer of RPR * npad (contiguous allocs)
    std::vector<double*> g2(10), g4(5), w2(1);
    for (auto& p : g2) CK(hipMalloc(&p, sizeof(double) * 2 * npad));
    for (auto& p : g4) CK(hipMalloc(&p, sizeof(double) * 4 * npad));
    CK(hipMalloc(&w2[0], sizeof(double) * 2 * npad));
    for (auto p : g2) CK(hipMemset(p, 0, sizeof(double) * 2 * npad));
    for (auto p : g4) CK(hipMemset(p, 0, sizeof(double) * 4 * npad));
    CK(hipMemset(w2[0], 0, sizeof(double) * 2 * npad));
    Bufs sep, pair2, quad4, sep_off, pair2_off;
    for (int k = 0; k < 22; ++k) sep.in[k] = v[k];
    for (int k = 0; k < 4; ++k) sep.out[k] = v[22 + k];
    // the product's vectors start 32 doubles (256 B) into their allocation (the ghost-cell pad):
    // the same streams at that offset (npad > n + 32, so the last rows stay inside)
    sep_off = sep;
    for (int k = 0; k < 22; ++k) sep_off.in[k] = v[k] + 32;
    for (int k = 0; k < 4; ++k) sep_off.out[k] = v[22 + k] + 32;
    pair2 = sep;
    quad4 = sep;
    for (int b = 0; b < 10; ++b) pair2.in[2 + b] = g2[b];
    for (int b = 0; b < 5; ++b) quad4.in[2 + b] = g4[b];
    pair2.out[2] = quad4.out[2] = w2[0];
    pair2_off = pair2;
    for (int k = 0; k < 2; ++k) pair2_off.in[k] = v[k] + 32;
    for (int b = 0; b < 10; ++b) pair2_off.in[2 + b] = g2[b] + 32;
    for (int k = 0; k < 2; ++k) pair2_off.out[k] = v[22 + k] + 32;
    pair2_off.out[2] = w2[0] + 32;
    struct Case {
        const char* name;
        void (*k)(Bufs, int64_t, int64_t, double*);
        Bufs* b;
    } cases[] = {{"sep_22r4w", k_vfil<1, 1>, &sep},
                 {"pair2_22r4w", k_vfil<2, 2>, &pair2},
                 {"quad4_22r4w", k_vfil<4, 2>, &quad4},
                 {"sep_22r4w(again)", k_vfil<1, 1>, &sep},
                 {"pair2_22r4w(again)", k_vfil<2, 2>, &pair2},
                 {"sep_22r4w_off256B", k_vfil<1, 1>, &sep_off},
                 {"pair2_22r4w_off256B", k_vfil<2, 2>, &pair2_off},
                 {"sep_22r4w_off256B(again)", k_vfil<1, 1>, &sep_off}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("n=%lld L=%lld segments=%d, 60 KiB LDS per workgroup (2 waves / SIMD)\n", (long long)n, (long long)L, nseg);
    for (const Case& c : cases) {
        std::vector<float> ms;
        for (int r = 0; r < 16; ++r) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(c.k, dim3(nseg), dim3(256), 60 * 1024, 0, *c.b, n, L, sink);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        printf("%-26s %9.1f us  %7.1f GB/s  (min %.1f us)\n", c.name, med * 1e3, 26.0 * 8.0 * (double)n / (med * 1e-3) / 1e9,
               ms.front() * 1e3);
    }
    return 0;
}
