// tools/cooplaunch_probe.hip — hipLaunchCooperativeKernel against a plain launch for the library's
// grid-barrier kernels (k_coop_iter / k_coop_search use plain launches with an
// in-kernel grid barrier, capped by their own occupancy instead of the cooperative API).
//
// The kernel has the cooperative iteration's shape: one 256-thread workgroup per segment (G
// workgroups), P passes, each pass a stream over the workgroup's segment (3 loads + 1 store per
// element) and a grid barrier (an agent-scope arrival counter, every workgroup spinning until the
// pass's count is complete) - the same residency requirement. Measured for each launch API:
//   queued : B launches back to back on one stream, one synchronisation at the end (the library
//            queues iteration k + 1 behind iteration k)
//   synced : one launch, then a stream synchronisation, B times (a launch the host waits for)
// Reports microseconds per launch (median of 5 reps). Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/cooplaunch_probe tools/cooplaunch_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
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

__global__ __launch_bounds__(256) void k_passes(double* q, const double* y, const double* s, int64_t L, int passes,
                                                unsigned* cnt, unsigned base, unsigned* err) {
    const int64_t o = (int64_t)blockIdx.x * L;
    double acc = 0.0;
    for (int p = 0; p < passes; ++p) {
        for (int64_t i = threadIdx.x; i < L; i += 256) {
            const double v = q[o + i] - 1e-300 * y[o + i];
            q[o + i] = v;
            acc = fma(s[o + i], v, acc);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned want = (base + (unsigned)p + 1u) * gridDim.x;
            long long spins = 0;
            while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1ll << 26)) {  // never hang: a grid that is not resident gives up
                    *err = 1;
                    break;
                }
            }
        }
        __syncthreads();
    }
    if (acc == 1234.5) q[o] = acc;
}

int main() {
    int dev = 0, cus = 0, coop = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_passes, 256, 0));
    printf("device %d: %d CUs, cooperative launch attribute %d, occupancy %d workgroups/CU\n", dev, cus, coop, occ);
    const int64_t L = 512;  // elements per workgroup (the small-n segment)
    const int passes = 12;  // a two-loop at h = 5 plus the commit
    const int B = 400;
    double *q, *y, *s;
    unsigned *cnt, *err;
    const int gmax = 256;
    CK(hipMalloc(&q, sizeof(double) * L * gmax));
    CK(hipMalloc(&y, sizeof(double) * L * gmax));
    CK(hipMalloc(&s, sizeof(double) * L * gmax));
    CK(hipMemset(q, 0, sizeof(double) * L * gmax));
    CK(hipMemset(y, 0, sizeof(double) * L * gmax));
    CK(hipMemset(s, 0, sizeof(double) * L * gmax));
    CK(hipMalloc(&cnt, sizeof(unsigned)));
    CK(hipHostMalloc(&err, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
    *err = 0;
    unsigned* derr = nullptr;
    CK(hipHostGetDevicePointer((void**)&derr, err, 0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    unsigned base = 0;
    for (int G : {20, 196, 256}) {
        for (int api = 0; api < 2; ++api) {
            for (int mode = 0; mode < 2; ++mode) {
                std::vector<double> reps;
                for (int r = 0; r < 5; ++r) {
                    CK(hipMemset(cnt, 0, sizeof(unsigned)));
                    CK(hipDeviceSynchronize());
                    base = 0;
                    const auto t0 = std::chrono::steady_clock::now();
                    for (int b = 0; b < B; ++b) {
                        int64_t Lx = L;
                        int px = passes;
                        unsigned bx = base;
                        void* args[] = {&q, &y, &s, &Lx, &px, &cnt, &bx, &derr};
                        if (api == 0)
                            CK(hipLaunchKernel((const void*)k_passes, dim3(G), dim3(256), args, 0, st));
                        else
                            CK(hipLaunchCooperativeKernel((const void*)k_passes, dim3(G), dim3(256), args, 0, st));
                        base += (unsigned)passes;
                        if (mode == 1) CK(hipStreamSynchronize(st));
                    }
                    CK(hipStreamSynchronize(st));
                    const double us =
                        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / B;
                    reps.push_back(us);
                }
                std::sort(reps.begin(), reps.end());
                printf("G=%3d %-22s %-7s %8.2f us per launch (min %.2f)%s\n", G,
                       api ? "hipLaunchCooperative" : "hipLaunchKernel", mode ? "synced" : "queued", reps[2], reps[0],
                       *err ? "  BARRIER GAVE UP" : "");
                *err = 0;
            }
        }
    }
    return 0;
}
