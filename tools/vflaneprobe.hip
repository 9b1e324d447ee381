// tools/vflaneprobe.hip — the vector-free commit's stream shape with one element per lane against
// two, before changing ORC_CANON_VF's order for it. k_vf_commit at h = 10
// reads 2h + 2 = 22 vectors, writes 4 and keeps 6 + 4h + 1 = 47 accumulators per lane (the new
// Gram rows y'·b_l and g'·b_l over the 2h basis vectors, whatever the row shape). Each kernel here
// streams the same 22 R + 4 W in the solver's segment layout (a workgroup per L-element segment,
// wave w on rows 4u + w) with 47 live fma chains per lane:
//   E2 U1 : 128-element rows, two elements per lane (16-B accesses), one row in flight (today)
//   E1 U1 : 64-element rows, one element per lane (8-B accesses), one row in flight
//   E1 U2 : the same with two rows in flight
//   E1 U4 : four rows in flight
// and reports algorithmic TB/s (HIP events, median of reps) and each kernel's VGPR count (from
// the code object: build with --save-temps, or read the .s). WPE = amdgpu_waves_per_eu floor.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/vflaneprobe tools/vflaneprobe.hip
// usage: tools/vflaneprobe [n] [reps]
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

constexpr int R = 22, W = 4, NB = 20, K = 6 + 2 * NB + 1;  // K = 47 at h = 10

struct Arrays {
    const double* r[R];
    double* w[W];
};

typedef double dvec2 __attribute__((ext_vector_type(2)));

// one element (E = 1) or two (E = 2) per lane; rows of 64 E elements, wave w on rows 4u + w
template <int E, int U, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_vf_shape(Arrays A, int64_t n,
                                                                                              int64_t L, double* out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * L;
    constexpr int ROW = 64 * E;
    const int nrows = (int)(L / (4 * ROW));
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    for (int u0 = 0; u0 < nrows; u0 += U) {
        double v[U][R][E];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + (int64_t)(4 * (u0 + u) + w) * ROW + E * lane;
#pragma unroll
            for (int k = 0; k < R; ++k) {
                if (u0 + u < nrows && i < n) {
                    if (E == 2) {
                        const dvec2 x = __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(A.r[k] + i));
                        v[u][k][0] = x.x;
                        v[u][k][E - 1] = x.y;
                    } else {
                        v[u][k][0] = __builtin_nontemporal_load(A.r[k] + i);
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + (int64_t)(4 * (u0 + u) + w) * ROW + E * lane;
            if (u0 + u >= nrows || i >= n) break;
            double o[E][W];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                // d = combination of the basis rows, the trial point and the new gradient-like row
                double d = v[u][0][e];
#pragma unroll
                for (int k = 1; k < R; ++k) d = d + 0.5 * v[u][k][e];
                const double y = d - v[u][1][e], g = d * 0.25 + v[u][2][e];
                o[e][0] = d;
                o[e][1] = y;
                o[e][2] = g;
                o[e][3] = d + y;
                // the new Gram rows: y'·b_l and g'·b_l over the basis, and 7 more reductions
#pragma unroll
                for (int l = 0; l < NB; ++l) {
                    acc[l] = fma(y, v[u][l + 2][e], acc[l]);
                    acc[NB + l] = fma(g, v[u][l + 2][e], acc[NB + l]);
                }
#pragma unroll
                for (int k = 2 * NB; k < K; ++k) acc[k] = fma(o[e][k & 3], v[u][k - 2 * NB][e], acc[k]);
            }
#pragma unroll
            for (int k = 0; k < W; ++k) {
                if (E == 2) {
                    dvec2 p;
                    p.x = o[0][k];
                    p.y = o[E - 1][k];
                    __builtin_nontemporal_store(p, reinterpret_cast<dvec2*>(A.w[k] + i));
                } else {
                    __builtin_nontemporal_store(o[0][k], A.w[k] + i);
                }
            }
        }
    }
    double t = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) t += acc[k];
    if (t == 12345.678) out[threadIdx.x & 7] = t;
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? (int64_t)atof(argv[1]) : 100000000LL;
    const int reps = argc > 2 ? atoi(argv[2]) : 9;
    std::vector<double*> v(R + W);
    for (size_t j = 0; j < v.size(); ++j) {
        CK(hipMalloc(&v[j], n * sizeof(double) + 4096));
        CK(hipMemset(v[j], 0, n * sizeof(double)));
    }
    double* out;
    CK(hipMalloc(&out, 64));
    Arrays A;
    for (int k = 0; k < R; ++k) A.r[k] = v[k];
    for (int k = 0; k < W; ++k) A.w[k] = v[R + k];
    // random-ish data (zeros stream faster): one fill kernel via hipMemset patterns is not enough,
    // so the basis rows get a byte pattern that is a finite, nonzero double
    for (int k = 0; k < R; ++k) CK(hipMemsetD32(reinterpret_cast<unsigned*>(v[k]), 0x3fd55555u + 7u * k, (size_t)n * 2));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // the vector-free segment: 512 elements x F (n = 1e8: 12288, the canonical L)
    const int64_t per = (n + 8191) / 8192;
    const int64_t L = std::max<int64_t>(512, ((per + 511) / 512) * 512);
    const int nseg = (int)((n + L - 1) / L);
    auto run = [&](const char* name, auto launch) {
        std::vector<float> t;
        for (int r = 0; r < reps + 2; ++r) {
            CK(hipEventRecord(a));
            launch();
            CK(hipGetLastError());
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const double ms = t[t.size() / 2];
        printf("%-18s L %6lld segs %6d  %8.3f ms  %6.3f TB/s\n", name, (long long)L, nseg, ms,
               (R + W) * 8.0 * n / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
#define CASE(E, U, WPE) \
    run("E" #E " U" #U " wpe" #WPE, [&] { hipLaunchKernelGGL((k_vf_shape<E, U, WPE>), dim3(nseg), dim3(256), 0, 0, A, n, L, out); });
    for (int round = 0; round < 2; ++round) {
        CASE(2, 1, 1)
        CASE(2, 1, 2)
        CASE(1, 1, 1)
        CASE(1, 1, 2)
        CASE(1, 1, 3)
        CASE(1, 2, 1)
        CASE(1, 2, 2)
        CASE(1, 4, 1)
    }
    return 0;
}
