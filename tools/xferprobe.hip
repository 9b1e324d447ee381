// tools/xferprobe.hip — host <-> device transfer of one n-vector from PAGEABLE caller memory (the
// C ABI's x0_host / x_out_host, lbfgs_minimize), the way configs[3]'s time to solution pays it
// (the reference pays the same copies, parallel-implementation/L-BFGS.cu:176,
// 360-365). Strategies, each timed end to end on the host (median of 5 after a warm-up):
//   pageable   hipMemcpy straight from / to the pageable buffer (the runtime stages it)
//   register   hipHostRegister the caller's buffer, one async copy, hipHostUnregister
//   staged T C pinned ring of 4 chunks of C MiB, the chunk copies into / out of it done by T host
//              threads while the DMA engine moves the previous chunk
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/xferprobe tools/xferprobe.hip -lpthread
// Run:   tools/xferprobe [n]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_copy(void* dst, const void* src, size_t bytes, int T) {
    if (T <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (bytes / T + 4095) & ~(size_t)4095;
    for (int t = 0; t < T; ++t) {
        const size_t lo = std::min(bytes, per * t), hi = std::min(bytes, per * (t + 1));
        if (hi > lo) th.emplace_back([=] { memcpy((char*)dst + lo, (const char*)src + lo, hi - lo); });
    }
    for (auto& x : th) x.join();
}

struct Ring {
    static const int NB = 4;
    char* buf[NB];
    hipEvent_t ev[NB];
    size_t chunk;
};

static void staged_h2d(Ring& R, hipStream_t s, double* dev, const double* host, size_t bytes, int T) {
    int i = 0;
    for (size_t off = 0; off < bytes; off += R.chunk, ++i) {
        const int b = i % Ring::NB;
        const size_t len = std::min(R.chunk, bytes - off);
        CK(hipEventSynchronize(R.ev[b]));  // the DMA that last read this buffer is done
        par_copy(R.buf[b], (const char*)host + off, len, T);
        CK(hipMemcpyAsync((char*)dev + off, R.buf[b], len, hipMemcpyHostToDevice, s));
        CK(hipEventRecord(R.ev[b], s));
    }
    CK(hipStreamSynchronize(s));
}

static void staged_d2h(Ring& R, hipStream_t s, double* host, const double* dev, size_t bytes, int T) {
    const size_t nchunk = (bytes + R.chunk - 1) / R.chunk;
    // keep NB - 1 chunk downloads in flight ahead of the host copies out of the ring
    size_t issued = 0;
    auto issue = [&](size_t i) {
        const int b = i % Ring::NB;
        const size_t off = i * R.chunk, len = std::min(R.chunk, bytes - off);
        CK(hipMemcpyAsync(R.buf[b], (const char*)dev + off, len, hipMemcpyDeviceToHost, s));
        CK(hipEventRecord(R.ev[b], s));
    };
    for (; issued < std::min<size_t>(nchunk, Ring::NB - 1); ++issued) issue(issued);
    for (size_t i = 0; i < nchunk; ++i) {
        const int b = i % Ring::NB;
        CK(hipEventSynchronize(R.ev[b]));
        if (issued < nchunk) issue(issued++);
        const size_t off = i * R.chunk, len = std::min(R.chunk, bytes - off);
        par_copy((char*)host + off, R.buf[b], len, T);
    }
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? (size_t)atof(argv[1]) : 100000000;
    const size_t bytes = n * sizeof(double);
    double* host = (double*)malloc(bytes);  // pageable, as a caller's std::vector / numpy array
    double* back = (double*)malloc(bytes);
    for (size_t i = 0; i < n; ++i) host[i] = (double)(i % 1000) * 0.25;
    memset(back, 0, bytes);
    double* dev;
    CK(hipMalloc(&dev, bytes));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    auto report = [&](const char* name, std::vector<double> up, std::vector<double> down) {
        const double u = med(up), d = med(down);
        printf("%-16s H2D %7.2f ms (%6.1f GB/s)   D2H %7.2f ms (%6.1f GB/s)\n", name, u * 1e3, bytes / u / 1e9,
               d * 1e3, bytes / d / 1e9);
        fflush(stdout);
    };
    {
        std::vector<double> up, down;
        for (int r = 0; r < 6; ++r) {
            double t0 = now();
            CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            double t1 = now();
            CK(hipMemcpyAsync(back, dev, bytes, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            double t2 = now();
            if (r) up.push_back(t1 - t0), down.push_back(t2 - t1);
        }
        report("pageable", up, down);
    }
    {
        std::vector<double> up, down;
        for (int r = 0; r < 6; ++r) {
            double t0 = now();
            CK(hipHostRegister(host, bytes, hipHostRegisterDefault));
            CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            CK(hipHostUnregister(host));
            double t1 = now();
            CK(hipHostRegister(back, bytes, hipHostRegisterDefault));
            CK(hipMemcpyAsync(back, dev, bytes, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            CK(hipHostUnregister(back));
            double t2 = now();
            if (r) up.push_back(t1 - t0), down.push_back(t2 - t1);
        }
        report("register", up, down);
    }
    for (size_t mib : {8, 32}) {
        Ring R;
        R.chunk = mib << 20;
        for (int b = 0; b < Ring::NB; ++b) {
            CK(hipHostMalloc((void**)&R.buf[b], R.chunk, hipHostMallocDefault));
            CK(hipEventCreateWithFlags(&R.ev[b], hipEventDisableTiming));
            CK(hipEventRecord(R.ev[b], s));
        }
        for (int T : {1, 4, 8, 16}) {
            std::vector<double> up, down;
            for (int r = 0; r < 6; ++r) {
                double t0 = now();
                staged_h2d(R, s, dev, host, bytes, T);
                double t1 = now();
                staged_d2h(R, s, back, dev, bytes, T);
                double t2 = now();
                if (r) up.push_back(t1 - t0), down.push_back(t2 - t1);
            }
            char name[64];
            snprintf(name, sizeof name, "staged T%d C%zu", T, mib);
            report(name, up, down);
            if (memcmp(host, back, bytes) != 0) printf("  MISMATCH\n");
        }
        for (int b = 0; b < Ring::NB; ++b) {
            CK(hipHostFree(R.buf[b]));
            CK(hipEventDestroy(R.ev[b]));
        }
    }
    printf("host threads available: %u\n", std::thread::hardware_concurrency());
    CK(hipFree(dev));
    free(host);
    free(back);
    return 0;
}
