// tools/gldsprobe.hip — does LDS-DMA (global_load_lds_dwordx4) beat register loads for the
// two-loop pass mix (3 reads + 1 write, q = q - c y; acc += s . q) on MI355X?
//   reg<U>  : the solver's shape — segment per workgroup, rows 4u+w, U rows of loads in flight
//   glds<U> : same, but the 3 read rows of a step land in a per-wave LDS ring by LDS-DMA
//             (1 KiB per wave-instruction), the next step's DMA issued before this step is
//             consumed; counted vmcnt waits, ds_read_b128 into registers
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/gldsprobe tools/gldsprobe.hip
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

__device__ __forceinline__ dvec2 ldnt(const double* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(p));
}
__device__ __forceinline__ void stnt(double* p, dvec2 v) { __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(p)); }

template <int U>
__global__ __launch_bounds__(256) void k_reg(double* q, const double* __restrict__ y, const double* __restrict__ s,
                                             double c, int64_t L, double* out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * L;
    const int nrows = (int)(L / 512);
    double acc = 0;
    for (int u0 = 0; u0 < nrows; u0 += U) {
        dvec2 qv[U], yv[U], sv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = base + (int64_t)(4 * (u0 + j) + w) * 128 + 2 * lane;
            qv[j] = ldnt(q + i);
            yv[j] = ldnt(y + i);
            sv[j] = ldnt(s + i);
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = base + (int64_t)(4 * (u0 + j) + w) * 128 + 2 * lane;
            const dvec2 r = qv[j] - c * yv[j];
            stnt(q + i, r);
            acc = fma(sv[j].x, r.x, fma(sv[j].y, r.y, acc));
        }
    }
    if (acc == 12345.678) out[0] = acc;
}

// LDS-DMA: 16 B per lane, 1 KiB per wave-instruction, destination M0 + lane * 16
__device__ __forceinline__ void glds16(const double* g, double* lds_wave) {
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g), (__attribute__((address_space(3))) void*)(lds_wave), 16, 0, 2 /* nt */);
}

template <int U>
__global__ __launch_bounds__(256) void k_glds(double* q, const double* __restrict__ y, const double* __restrict__ s,
                                              double c, int64_t L, double* out) {
    // [buffer][wave][stream][row in step][128 doubles]
    __shared__ __attribute__((aligned(1024))) double ring[2][4][3][U][128];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * L;
    const int nrows = (int)(L / 512);
    const int nsteps = nrows / U;
    double acc = 0;
    auto issue = [&](int step, int b) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = base + (int64_t)(4 * (step * U + j) + w) * 128 + 2 * lane;
            glds16(q + i, &ring[b][w][0][j][0]);
            glds16(y + i, &ring[b][w][1][j][0]);
            glds16(s + i, &ring[b][w][2][j][0]);
        }
    };
    issue(0, 0);
    for (int st = 0; st < nsteps; ++st) {
        const int b = st & 1;
        if (st + 1 < nsteps) {
            issue(st + 1, b ^ 1);
            // this step's 3U DMAs landed once at most the next step's 3U are outstanding
            if (U == 1) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            if (U == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            if (U == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = base + (int64_t)(4 * (st * U + j) + w) * 128 + 2 * lane;
            const dvec2 qv = *reinterpret_cast<const dvec2*>(&ring[b][w][0][j][2 * lane]);
            const dvec2 yv = *reinterpret_cast<const dvec2*>(&ring[b][w][1][j][2 * lane]);
            const dvec2 sv = *reinterpret_cast<const dvec2*>(&ring[b][w][2][j][2 * lane]);
            const dvec2 r = qv - c * yv;
            stnt(q + i, r);
            acc = fma(sv.x, r.x, fma(sv.y, r.y, acc));
        }
    }
    if (acc == 12345.678) out[0] = acc;
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000LL;
    const int reps = argc > 2 ? atoi(argv[2]) : 9;
    const int64_t L = 12288;  // the solver's segment at n = 1e8 (24 rows per wave)
    const int nb = (int)(n / L);
    const int64_t nn = (int64_t)nb * L;
    std::vector<double*> v(3);
    for (auto& p : v) {
        CK(hipMalloc(&p, nn * sizeof(double)));
        CK(hipMemset(p, 0, nn * sizeof(double)));
    }
    double* out;
    CK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
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
        printf("%-10s %8.3f ms  %7.1f GB/s\n", name, ms, 4.0 * 8.0 * nn / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("reg2", [&] { hipLaunchKernelGGL(k_reg<2>, dim3(nb), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, L, out); });
        run("reg4", [&] { hipLaunchKernelGGL(k_reg<4>, dim3(nb), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, L, out); });
        run("glds1", [&] { hipLaunchKernelGGL(k_glds<1>, dim3(nb), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, L, out); });
        run("glds2", [&] { hipLaunchKernelGGL(k_glds<2>, dim3(nb), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, L, out); });
        run("glds4", [&] { hipLaunchKernelGGL(k_glds<4>, dim3(nb), dim3(256), 0, 0, v[0], v[1], v[2], 0.5, L, out); });
    }
    return 0;
}
