// tools/vfprobe.hip — HBM bandwidth of many-stream mixes on MI355X (the vector-free commit
// reads 2h + 2 vectors and writes 4). Each kernel streams R read arrays and W write arrays of
// n doubles with 16-B accesses, with R dot accumulators per lane (the register footprint of
// the real kernel), and reports algorithmic GB/s (HIP events, median of reps).
//   grid<R,W,U> : grid-stride over element pairs, U pairs in flight per lane
//   seg<R,W,U>  : the solver's layout — a workgroup per L-element segment, rows of 128
//                 interleaved over its 4 waves, U rows per step
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/vfprobe tools/vfprobe.hip
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

template <int R, int W>
struct Arrays {
    const double* r[R];
    double* w[W];
};

template <int R, int W, int U, bool NT>
__global__ __launch_bounds__(256) void k_grid(Arrays<R, W> A, int64_t n2, double* out) {
    double acc[R];
#pragma unroll
    for (int k = 0; k < R; ++k) acc[k] = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += U * stride) {
        dvec2 v[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < R; ++k)
                if (i + u * stride < n2) v[u][k] = ld<NT>(A.r[k] + 2 * (i + u * stride));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + u * stride >= n2) break;
            dvec2 s = v[u][0];
#pragma unroll
            for (int k = 1; k < R; ++k) s = s + 0.5 * v[u][k];
#pragma unroll
            for (int k = 0; k < W; ++k) st<NT>(A.w[k] + 2 * (i + u * stride), s + (double)k);
#pragma unroll
            for (int k = 0; k < R; ++k) acc[k] = fma(s.x, v[u][k].x, fma(s.y, v[u][k].y, acc[k]));
        }
    }
    double t = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) t += acc[k];
    if (t == 12345.678) out[0] = t;
}

template <int R, int W, int U, bool NT>
__global__ __launch_bounds__(256) void k_seg(Arrays<R, W> A, int64_t n, int64_t L, double* out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * L;
    const int nrows = (int)(L / 512);
    double acc[R];
#pragma unroll
    for (int k = 0; k < R; ++k) acc[k] = 0.0;
    for (int u0 = 0; u0 < nrows; u0 += U) {
        dvec2 v[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + (int64_t)(4 * (u0 + u) + w) * 128 + 2 * lane;
#pragma unroll
            for (int k = 0; k < R; ++k)
                if (u0 + u < nrows && i < n) v[u][k] = ld<NT>(A.r[k] + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + (int64_t)(4 * (u0 + u) + w) * 128 + 2 * lane;
            if (u0 + u >= nrows || i >= n) break;
            dvec2 s = v[u][0];
#pragma unroll
            for (int k = 1; k < R; ++k) s = s + 0.5 * v[u][k];
#pragma unroll
            for (int k = 0; k < W; ++k) st<NT>(A.w[k] + i, s + (double)k);
#pragma unroll
            for (int k = 0; k < R; ++k) acc[k] = fma(s.x, v[u][k].x, fma(s.y, v[u][k].y, acc[k]));
        }
    }
    double t = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) t += acc[k];
    if (t == 12345.678) out[0] = t;
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000LL;
    const int reps = argc > 2 ? atoi(argv[2]) : 7;
    const int64_t n2 = n / 2;
    const int NV = 26;
    std::vector<double*> v(NV);
    for (auto& p : v) {
        CK(hipMalloc(&p, n * sizeof(double) + 4096));
        CK(hipMemset(p, 0, n * sizeof(double)));
    }
    double* out;
    CK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char* name, double vecs, int grid, auto launch) {
        std::vector<float> t;
        for (int r = 0; r < reps + 2; ++r) {
            CK(hipEventRecord(a));
            launch(grid);
            CK(hipGetLastError());
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const double ms = t[t.size() / 2];
        printf("%-26s grid %6d  %8.3f ms  %7.1f GB/s\n", name, grid, ms, vecs * 8.0 * n / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    const int64_t per = (n + 8191) / 8192;
    const int64_t L = std::max<int64_t>(512, ((per + 127) / 128) * 128);
    const int nseg = (int)((n + L - 1) / L);
#define CASE(R, W, U, NT)                                                                                    \
    {                                                                                                      \
        Arrays<R, W> A;                                                                                    \
        for (int k = 0; k < R; ++k) A.r[k] = v[k];                                                         \
        for (int k = 0; k < W; ++k) A.w[k] = v[R + k];                                                     \
        char nm[64];                                                                                       \
        snprintf(nm, sizeof nm, "grid R%d W%d U%d %s", R, W, U, NT ? "nt" : "");                           \
        for (int g : {1024, 2048})                                                                         \
            run(nm, R + W, g, [&](int gr) { hipLaunchKernelGGL((k_grid<R, W, U, NT>), dim3(gr), dim3(256), 0, 0, A, n2, out); }); \
        snprintf(nm, sizeof nm, "seg R%d W%d U%d %s", R, W, U, NT ? "nt" : "");                            \
        run(nm, R + W, nseg, [&](int gr) { hipLaunchKernelGGL((k_seg<R, W, U, NT>), dim3(gr), dim3(256), 0, 0, A, n, L, out); }); \
    }
    CASE(3, 1, 1, true)
    CASE(2, 4, 1, true)
    CASE(6, 4, 1, true)
    CASE(12, 4, 1, true)
    CASE(22, 4, 1, true)
    CASE(22, 4, 1, false)
    CASE(22, 4, 2, true)
    CASE(22, 1, 1, true)
    CASE(22, 0, 1, true)
    return 0;
}
