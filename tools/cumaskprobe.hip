// tools/cumaskprobe.hip — does LBFGS_CU_PARTITION's stream CU mask really give each rank its own
// CUs? (the one-card rehearsal of distinct GPUs rests on it.)
//
// For world = 2, 4, 8: one stream per rank with the library's mask (CUs [r, r + 1) * cus / world,
// lbfgs_kernels.hip lbk_create), a kernel of many workgroups on every stream at once; each
// workgroup records the hardware id of the CU it ran on (XCC_ID, and HW_ID's CU / SH / SE fields).
// Prints, per world, the distinct CUs each rank's workgroups used and whether any CU was used by
// two ranks. Build: hipcc --offload-arch=gfx950 -O2 tools/cumaskprobe.hip -o tools/cumaskprobe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

// hwreg(HW_REG_HW_ID) = id 4, hwreg(HW_REG_XCC_ID) = id 20, all 32 bits (llvm-mc -mcpu=gfx950)
__global__ void k_where(unsigned* out, int spin) {
    if (threadIdx.x == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        out[blockIdx.x] = ((xcc & 0xfu) << 8) | ((hw >> 8) & 0xffu);  // XCC, SE / SH / CU
    }
    // keep the workgroup resident a while, so the ranks' grids overlap in time
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(2);
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("device CUs: %d\n", cus);
    const int blocks = 8192;
    int bad = 0;
    for (int world : {2, 4, 8}) {
        const int per = cus / world;
        std::vector<hipStream_t> st(world);
        std::vector<unsigned*> d(world);
        for (int r = 0; r < world; ++r) {
            std::vector<uint32_t> mask((cus + 31) / 32, 0u);
            for (int i = r * per; i < (r + 1) * per; ++i) mask[i >> 5] |= 1u << (i & 31);
            CK(hipExtStreamCreateWithCUMask(&st[r], (uint32_t)mask.size(), mask.data()));
            CK(hipMalloc(&d[r], sizeof(unsigned) * blocks));
            CK(hipMemset(d[r], 0xff, sizeof(unsigned) * blocks));
        }
        CK(hipDeviceSynchronize());
        for (int r = 0; r < world; ++r) hipLaunchKernelGGL(k_where, dim3(blocks), dim3(64), 0, st[r], d[r], 2000);
        CK(hipDeviceSynchronize());
        std::vector<std::set<unsigned>> used(world);
        std::set<unsigned> all;
        int overlap = 0;
        for (int r = 0; r < world; ++r) {
            std::vector<unsigned> h(blocks);
            CK(hipMemcpy(h.data(), d[r], sizeof(unsigned) * blocks, hipMemcpyDeviceToHost));
            for (unsigned v : h) used[r].insert(v);
        }
        for (int r = 0; r < world; ++r)
            for (unsigned v : used[r]) {
                if (all.count(v)) ++overlap;
                all.insert(v);
            }
        printf("world %d (%d CUs per rank):", world, per);
        for (int r = 0; r < world; ++r) printf(" rank%d=%zu", r, used[r].size());
        printf("  distinct over ranks %zu, CUs shared by two ranks %d\n", all.size(), overlap);
        // which XCDs each rank's CUs sit on (CUs per XCC id): one XCD per rank, or spread over all 8
        for (int r = 0; r < world; ++r) {
            int per_xcc[16] = {0};
            for (unsigned v : used[r]) per_xcc[(v >> 8) & 0xf]++;
            printf("  rank%d CUs per XCC:", r);
            for (int x = 0; x < 8; ++x) printf(" %d", per_xcc[x]);
            printf("\n");
        }
        if (overlap) bad = 1;
        for (int r = 0; r < world; ++r) {
            CK(hipFree(d[r]));
            CK(hipStreamDestroy(st[r]));
        }
    }
    printf(bad ? "RESULT: ranks share CUs\n" : "RESULT: disjoint\n");
    return bad;
}
