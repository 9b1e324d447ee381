// tools/contig_probe.hip — are host transfers into / out of physically contiguous allocations
// (hipExtMallocWithFlags(..., hipDeviceMallocContiguous)) coherent with the kernels around them?
// T host threads, one non-blocking stream and one device buffer each, repeating either
//   up:   hipMemsetAsync(0) -> sync -> hipMemcpyAsync H2D of random data -> sync -> a kernel sums the
//         buffer (integer, exact) -> compare with the host's sum;
//   down: a kernel fills the buffer with a pattern -> sync -> hipMemcpyAsync D2H -> sync -> compare,
// for plain / contiguous allocations and pageable / pinned host buffers. Reports mismatches per case.
// usage: contig_probe [threads] [iterations] [doubles] [sync: L2 write-back / invalidate around DMAs]
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

__global__ void k_fill(unsigned long long* __restrict__ x, long long n, unsigned long long key) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        x[i] = (unsigned long long)i * 0x9e3779b97f4a7c15ull ^ key;
}

// cache maintenance around a DMA (sync mode): every XCD's L2 written back before the copy (dirty
// lines from kernels must reach HBM before the copy engine reads it, and must not be evicted over
// what it writes), and invalidated after it (kernels must not hit stale lines of what it wrote);
// 256 workgroups land on every XCD (round-robin dispatch)
__global__ void k_l2_wb() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__global__ void k_l2_inv() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
static int g_sync = 0;
static void maint(hipStream_t s, int inv) {
    if (!g_sync) return;
    if (inv) hipLaunchKernelGGL(k_l2_inv, dim3(256), dim3(64), 0, s);
    else hipLaunchKernelGGL(k_l2_wb, dim3(256), dim3(64), 0, s);
}

static int run(int contig, int pinned, int down, int T, int iters, long long n) {
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
        std::vector<unsigned long long> hv;
        unsigned long long* h = nullptr;
        if (pinned) {
            if (hipHostMalloc((void**)&h, bytes, hipHostMallocDefault) != hipSuccess) { errs++; return; }
        } else {
            hv.resize((size_t)n);
            h = hv.data();
        }
        unsigned long long seed = 0x9e3779b97f4a7c15ull * (t + 1) + (unsigned long long)(contig + 2 * pinned);
        for (int it = 0; it < iters; ++it) {
            if (!down) {
                unsigned long long want = 0;
                for (long long i = 0; i < n; ++i) {
                    seed ^= seed << 13; seed ^= seed >> 7; seed ^= seed << 17;
                    h[i] = seed;
                    want += seed * (unsigned long long)(i + 1);
                }
                unsigned long long got = 0;
                if (hipMemsetAsync(d, 0, bytes, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) { errs++; break; }
                maint(s, 0);
                if (hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s) != hipSuccess) { errs++; break; }
                maint(s, 1);
                if (hipStreamSynchronize(s) != hipSuccess || hipMemsetAsync(dout, 0, 8, s) != hipSuccess) { errs++; break; }
                hipLaunchKernelGGL(k_sum, dim3(512), dim3(256), 0, s, d, n, dout);
                if (hipGetLastError() != hipSuccess) { errs++; break; }
                maint(s, 0);
                if (hipMemcpyAsync(&got, dout, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipStreamSynchronize(s) != hipSuccess) { errs++; break; }
                if (got != want) {
                    if (bad.fetch_add(1) < 3) printf("  up mismatch t%d it%d: got %llx want %llx\n", t, it, got, want);
                }
            } else {
                const unsigned long long key = seed + (unsigned long long)it * 7919ull;
                memset(h, 0, bytes);
                hipLaunchKernelGGL(k_fill, dim3(512), dim3(256), 0, s, d, n, key);
                if (hipGetLastError() != hipSuccess) { errs++; break; }
                maint(s, 0);
                if (hipStreamSynchronize(s) != hipSuccess ||
                    hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipStreamSynchronize(s) != hipSuccess) { errs++; break; }
                long long wrong = 0, first = -1;
                for (long long i = 0; i < n; ++i)
                    if (h[i] != ((unsigned long long)i * 0x9e3779b97f4a7c15ull ^ key)) {
                        if (first < 0) first = i;
                        ++wrong;
                    }
                if (wrong && bad.fetch_add(1) < 3)
                    printf("  down mismatch t%d it%d: %lld wrong from %lld: got %llx\n", t, it, wrong, first, h[first]);
            }
        }
        if (pinned) (void)hipHostFree(h);
        (void)hipFree(d);
        (void)hipFree(dout);
        (void)hipStreamDestroy(s);
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
    printf("%-5s %-10s %-8s %-4s: threads %d iterations %d doubles %lld: mismatched iterations %d, errors %d\n",
           g_sync ? "sync" : "raw", contig ? "contiguous" : "plain", pinned ? "pinned" : "pageable", down ? "down" : "up", T, iters, n,
           bad.load(), errs.load());
    fflush(stdout);
    return bad.load() + errs.load();
}

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 4;
    const int iters = argc > 2 ? atoi(argv[2]) : 50;
    const long long n = argc > 3 ? atoll(argv[3]) : 1000000;
    g_sync = argc > 4 ? atoi(argv[4]) : 0;
    int r = 0;
    for (int round = 0; round < 2; ++round)
        for (int down = 0; down < 2; ++down)
            for (int pinned = 0; pinned < 2; ++pinned)
                for (int contig = 0; contig < 2; ++contig) r += run(contig, pinned, down, T, iters, n);
    return r ? 1 : 0;
}
