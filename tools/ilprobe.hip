// tools/ilprobe.hip — does storing the two-loop's operand pairs (s_i, y_{i+1}) interleaved in one
// buffer stream faster than separate vectors, in the two-loop's own pass sequence?
//
// Every two-loop pass reads a work vector (q or r, in place, default cache policy), s_i and
// y_{i+1} (non-temporal) and writes the work vector back: 3 R + 1 W. mixprobe's repeated single
// pass showed interleaved pairs faster; this probe runs the real sequence instead: m - 1 first-loop
// passes (i descending, q) then m - 1 second-loop passes (i ascending, r), each pass over a
// different pair, consecutive passes walking their segments in opposite directions, as the
// product's LBFGS_REV default. Geometry as the product's passes (one 256-thread workgroup per
// canonical segment, rows of 128, 4 rows of loads in flight, lane = 2 elements).
//
// Layouts: "sep"   one allocation per s_j and per y_j (the product today)
//          "ilR"   block B_j holds s_j and y_{j+1}, alternating runs of R rows (R = 1, 4, 96)
//          "sep1"  one allocation for all s_j and y_j back to back (control: same allocation
//                  shape as "il", no interleave)
// Reports algorithmic TB/s over the whole sequence (4 vectors x 8 n bytes per pass), median of 9.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ilprobe tools/ilprobe.hip
// Run:   tools/ilprobe [n] [m]
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

// row index grow of a vector stored as runs of R rows alternating with its partner (R > 0), or
// plainly (R == 0)
__device__ __forceinline__ int64_t ioff(int64_t grow, int R, int half) {
    if (R == 0) return grow * 128;
    return ((grow / R) * 2 * R + half * R + grow % R) * 128;
}

__global__ __launch_bounds__(256) void k_pass(double* w, const double* a, int ra, int ha, const double* b,
                                               int rb, int hb, int64_t L, int rev, double alpha, double* sink) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t seg = rev ? (int64_t)gridDim.x - 1 - blockIdx.x : blockIdx.x;
    const int64_t row0 = seg * L / 128;
    const int nrows = (int)(L / 128);
    const int myrows = (nrows - wv + 3) / 4;
    double acc = 0.0;
    constexpr int U = 4;
    for (int u0 = 0; u0 < myrows; u0 += U) {
        dvec2 q[U], x[U], y[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            if (u0 + j >= myrows) break;
            const int64_t grow = row0 + 4 * (u0 + j) + wv;
            q[j] = *reinterpret_cast<const dvec2*>(w + grow * 128 + 2 * lane);
            x[j] = ldnt(a + ioff(grow, ra, ha) + 2 * lane);
            y[j] = ldnt(b + ioff(grow, rb, hb) + 2 * lane);
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            if (u0 + j >= myrows) break;
            const int64_t grow = row0 + 4 * (u0 + j) + wv;
            const dvec2 nq = q[j] - alpha * y[j];
            acc = fma(x[j].x, nq.x, fma(x[j].y, nq.y, acc));
            *reinterpret_cast<dvec2*>(w + grow * 128 + 2 * lane) = nq;
        }
    }
    if (acc == 1234.5678) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int64_t n0 = argc > 1 ? (int64_t)atof(argv[1]) : 100000000;
    const int m = argc > 2 ? atoi(argv[2]) : 10;
    const int64_t L = std::max<int64_t>(512, ((n0 + 8191) / 8192 + 127) / 128 * 128);
    const int nseg = (int)((n0 + L - 1) / L);
    const int64_t n = (int64_t)nseg * L;  // whole segments only (a probe: no masked tail)
    const size_t vb = sizeof(double) * n;
    double *q, *r, *sink;
    CK(hipMalloc(&q, vb));
    CK(hipMalloc(&r, vb));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(q, 0, vb));
    CK(hipMemset(r, 0, vb));
    // one pool big enough for every layout: m + 1 pairs
    double* pool;
    CK(hipMalloc(&pool, 2 * vb * (m + 1)));
    CK(hipMemset(pool, 0, 2 * vb * (m + 1)));
    std::vector<double*> sep(2 * (m + 1));
    for (auto& p : sep) {
        CK(hipMalloc(&p, vb));
        CK(hipMemset(p, 0, vb));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("n=%lld L=%lld segments=%d m=%d: %d passes of 3R+1W per sequence\n", (long long)n, (long long)L, nseg, m,
           2 * (m - 1));
    struct Layout {
        const char* name;
        int kind;  // 0 sep, 1 sep1, 2 il
        int R;
    } lays[] = {{"sep", 0, 0}, {"sep1", 1, 0}, {"il1", 2, 1}, {"il4", 2, 4}, {"il96", 2, 96}, {"sep", 0, 0}};
    for (const Layout& ly : lays) {
        // operand i of pair j: s_j (half 0) / y_j (half 1)
        auto sv = [&](int j, const double** p, int* R, int* h) {
            if (ly.kind == 0) { *p = sep[2 * j]; *R = 0; *h = 0; }
            else if (ly.kind == 1) { *p = pool + (size_t)(2 * j) * n; *R = 0; *h = 0; }
            else { *p = pool + (size_t)2 * j * n; *R = ly.R; *h = 0; }  // block B_j: s_j, y_{j+1}
        };
        auto yv = [&](int j, const double** p, int* R, int* h) {
            if (ly.kind == 0) { *p = sep[2 * j + 1]; *R = 0; *h = 0; }
            else if (ly.kind == 1) { *p = pool + (size_t)(2 * j + 1) * n; *R = 0; *h = 0; }
            else { *p = pool + (size_t)2 * (j - 1) * n; *R = ly.R; *h = 1; }  // y_j lives in B_{j-1}
        };
        std::vector<float> ms;
        int rev = 0;
        for (int rep = 0; rep < 10; ++rep) {
            CK(hipEventRecord(e0, 0));
            for (int i = m - 2; i >= 0; --i) {  // first loop: q, s_i, y_{i+1} (pairs 1..m; B_0 = pair index 1)
                const double *a, *b; int ra, ha, rb, hb;
                sv(i + 1, &a, &ra, &ha); yv(i + 2, &b, &rb, &hb);
                hipLaunchKernelGGL(k_pass, dim3(nseg), dim3(256), 0, 0, q, a, ra, ha, b, rb, hb, L, rev, 0.5, sink);
                rev ^= 1;
            }
            for (int i = 0; i <= m - 2; ++i) {  // second loop: r, s_i, y_{i+1}
                const double *a, *b; int ra, ha, rb, hb;
                sv(i + 1, &a, &ra, &ha); yv(i + 2, &b, &rb, &hb);
                hipLaunchKernelGGL(k_pass, dim3(nseg), dim3(256), 0, 0, r, a, ra, ha, b, rb, hb, L, rev, 0.5, sink);
                rev ^= 1;
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (rep) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        const double bytes = 2.0 * (m - 1) * 4 * 8.0 * (double)n;
        printf("%-6s  %8.1f us per sequence  %7.1f us per pass  %6.3f TB/s  (min %.1f us)\n", ly.name, med * 1e3,
               med * 1e3 / (2 * (m - 1)), bytes / (med * 1e-3) / 1e12, ms.front() * 1e3);
    }
    return 0;
}
