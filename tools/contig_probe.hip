// tools/contig_probe.hip — are host uploads into physically contiguous allocations
// (hipExtMallocWithFlags(..., hipDeviceMallocContiguous)) seen by the next kernel on the stream?
// T host threads, one stream and one device buffer each (contiguous or plain hipMalloc), repeat:
// hipMemsetAsync(0) -> sync -> hipMemcpyAsync H2D from pageable random data -> sync -> a kernel
// sums the buffer's bit patterns (integer, exact) -> compare with the host's sum. Reports the
// mismatches per mode. usage: contig_probe [threads] [iterations] [doubles]
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

__global__ void k_sum(const unsigned long long* __restrict__ x, long long n, unsigned long long* out) {
    unsigned long long a = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        a += x[i] * (unsigned long long)(i + 1);
    for (int m = 1; m < 64; m <<= 1) a += __shfl_xor(a, m, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, a);
}

static int run(int contig, int T, int iters, long long n) {
    std::atomic<int> bad{0}, errs{0};
    auto work = [&](int t) {
        hipStream_t s;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) { errs++; return; }
        unsigned long long* d = nullptr;
        unsigned long long* dout = nullptr;
        const size_t bytes = sizeof(unsigned long long) * (size_t)n;
        hipError_t e = contig ? hipExtMallocWithFlags((void**)&d, bytes, hipDeviceMallocContiguous)
                              : hipMalloc((void**)&d, bytes);
        if (e != hipSuccess || hipMalloc((void**)&dout, 8) != hipSuccess) { errs++; return; }
        std::vector<unsigned long long> h((size_t)n);
        unsigned long long seed = 0x9e3779b97f4a7c15ull * (t + 1) + (unsigned long long)contig;
        for (int it = 0; it < iters; ++it) {
            unsigned long long want = 0;
            for (long long i = 0; i < n; ++i) {
                seed ^= seed << 13; seed ^= seed >> 7; seed ^= seed << 17;
                h[(size_t)i] = seed;
                want += seed * (unsigned long long)(i + 1);
            }
            unsigned long long got = 0;
            if (hipMemsetAsync(d, 0, bytes, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess ||
                hipMemcpyAsync(d, h.data(), bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess || hipMemsetAsync(dout, 0, 8, s) != hipSuccess) { errs++; break; }
            hipLaunchKernelGGL(k_sum, dim3(512), dim3(256), 0, s, d, n, dout);
            if (hipMemcpyAsync(&got, dout, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess) { errs++; break; }
            if (got != want) bad++;
        }
        (void)hipFree(d);
        (void)hipFree(dout);
        (void)hipStreamDestroy(s);
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
    printf("%s: threads %d iterations %d doubles %lld: mismatches %d, errors %d\n", contig ? "contiguous" : "plain", T,
           iters, n, bad.load(), errs.load());
    fflush(stdout);
    return bad.load() + errs.load();
}

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 4;
    const int iters = argc > 2 ? atoi(argv[2]) : 50;
    const long long n = argc > 3 ? atoll(argv[3]) : 1000000;
    int r = 0;
    for (int round = 0; round < 2; ++round) {
        r += run(0, T, iters, n);
        r += run(1, T, iters, n);
    }
    return r ? 1 : 0;
}
