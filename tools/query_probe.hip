// tools/query_probe.hip — does a host thread that polls hipStreamQuery while the stream is busy
// make another runtime thread spin (in the one-card N = 8 rehearsal every rank ran
// two threads at 100 %, the job's 16-CPU quota throttled, and configs[4] ran at half speed)?
//
// A kernel that runs for 10 ms (one workgroup, a wall-clock loop) is launched 200 times on one
// stream; the host waits for each with one of:
//   spin       : a pause loop on a host-mapped completion word the kernel stores
//   spin+query : the same, with hipStreamQuery every 65536 turns (lbfgs_kernels.hip small_wait)
//   sync       : hipStreamSynchronize
//   spin+event : the pause loop with hipEventQuery on an event recorded after the kernel
//   evsync     : hipEventRecord after the kernel, hipEventSynchronize on it
//   d2h+sync   : a 512-byte hipMemcpyAsync into pinned host memory after the kernel, then
//                hipStreamSynchronize (the library's fetch of a slot that is not mirrored)
//   ev+spin    : hipEventRecord after the kernel (never waited on), the pause loop
//   queued     : 24 short kernels queued behind the long one, the pause loop on the last
// For each, the CPU seconds of every thread of the process over the 2 s (/proc/self/task), so a
// runtime thread that spins shows up beside the waiting one.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/query_probe tools/query_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <map>
#include <string>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

__global__ void k_busy(unsigned long long* done, unsigned long long seq, long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    __threadfence_system();
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

std::map<int, long> thread_ticks() {
    std::map<int, long> out;
    DIR* d = opendir("/proc/self/task");
    if (!d) return out;
    while (dirent* e = readdir(d)) {
        if (e->d_name[0] == '.') continue;
        const std::string p = std::string("/proc/self/task/") + e->d_name + "/stat";
        FILE* f = fopen(p.c_str(), "r");
        if (!f) continue;
        char buf[1024];
        const size_t n = fread(buf, 1, sizeof buf - 1, f);
        fclose(f);
        buf[n] = 0;
        const char* r = strrchr(buf, ')');
        if (!r) continue;
        // fields after ')': state ppid pgrp session tty tpgid flags minflt cminflt majflt cmajflt utime stime
        unsigned long ut = 0, st = 0;
        char state;
        int ppid, pgrp, sess, tty, tpgid;
        unsigned flags;
        unsigned long mi, cmi, ma, cma;
        if (sscanf(r + 2, "%c %d %d %d %d %d %u %lu %lu %lu %lu %lu %lu", &state, &ppid, &pgrp, &sess, &tty, &tpgid,
                   &flags, &mi, &cmi, &ma, &cma, &ut, &st) == 13)
            out[atoi(e->d_name)] = (long)(ut + st);
    }
    closedir(d);
    return out;
}

int main() {
    int clk_khz = 0;
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
    const long long ticks = (long long)clk_khz * 10;  // 10 ms
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long* done_h;
    CK(hipHostMalloc((void**)&done_h, sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent));
    *done_h = 0;
    unsigned long long* done_d;
    CK(hipHostGetDevicePointer((void**)&done_d, done_h, 0));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    unsigned long long seq = 0;
    double* slot_d;
    double* slot_h;
    CK(hipMalloc((void**)&slot_d, 512));
    CK(hipMemset(slot_d, 0, 512));
    CK(hipHostMalloc((void**)&slot_h, 512, hipHostMallocDefault));
    const char* names[] = {"spin", "spin+query", "sync", "spin+event", "spin+query",
                           "evsync", "d2h+sync", "ev+spin", "queued", "evsync", "d2h+sync"};
    for (int mode = 0; mode < 11; ++mode) {
        const auto a = thread_ticks();
        const auto t0 = std::chrono::steady_clock::now();
        const int B = 200;
        for (int b = 0; b < B; ++b) {
            ++seq;
            if (mode == 8) {
                hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s, done_d, seq - 1, ticks);
                for (int q = 0; q < 23; ++q) hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s, done_d, seq - 1, 1000);
            }
            hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s, done_d, seq, mode == 8 ? 1000 : ticks);
            if (mode == 3 || mode == 5 || mode == 7 || mode == 9) CK(hipEventRecord(ev, s));
            if (mode == 2) {
                CK(hipStreamSynchronize(s));
                continue;
            }
            if (mode == 5 || mode == 9) {
                CK(hipEventSynchronize(ev));
                continue;
            }
            if (mode == 6 || mode == 10) {
                CK(hipMemcpyAsync(slot_h, slot_d, 512, hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
                continue;
            }
            for (unsigned long it = 1;; ++it) {
                if (__atomic_load_n(done_h, __ATOMIC_ACQUIRE) >= seq) break;
                if ((it & 0xffff) == 0) {
                    if (mode == 1 || mode == 4) (void)hipStreamQuery(s);
                    if (mode == 3) (void)hipEventQuery(ev);
                }
                __builtin_ia32_pause();
            }
        }
        CK(hipStreamSynchronize(s));
        const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const auto b2 = thread_ticks();
        std::vector<double> busy;
        for (auto& kv : b2) {
            auto it = a.find(kv.first);
            busy.push_back((kv.second - (it == a.end() ? 0 : it->second)) / 100.0 / wall);
        }
        std::sort(busy.rbegin(), busy.rend());
        printf("%-11s wall %.2f s, %zu threads, CPU share of the busiest:", names[mode], wall, b2.size());
        for (size_t i = 0; i < std::min<size_t>(4, busy.size()); ++i) printf(" %.2f", busy[i]);
        printf("\n");
        fflush(stdout);
    }
    return 0;
}
