// lbfgs_kernels_vf.hip — vector-free mode entry points (lbk_vf_*), a translation unit of its
// own so the build runs in parallel.
#include "lbfgs_kernels_impl.h"

namespace {
template <int HB>
VfBasis<HB> vf_basis(int h, const double* const* S, const double* const* Y, const double* cs, const double* cy,
                     double cg) {
    VfBasis<HB> B;
    memset(&B, 0, sizeof B);
    B.h = h;
    B.cg = cg;
    for (int l = 0; l < h; ++l) {
        B.b[l] = S[l];
        B.c[l] = cs[l];
        B.b[h + l] = Y[l];
        B.c[h + l] = cy[l];
    }
    return B;
}

// the vector-free passes run under their own NT threshold (c->nt_vf)
struct NtScope {
    lbk_ctx* c;
    int saved;
    NtScope(lbk_ctx* c_, int nt) : c(c_), saved(c_->nt) { c->nt = nt; }
    ~NtScope() { c->nt = saved; }
};

// ... and its stage-2 form by its own segment count (the canonical rule applied to the
// vector-free geometry: tickets for <= 64 workgroups or sharded segments >= 8192)
struct TicketScope {
    lbk_ctx* c;
    int saved;
    TicketScope(lbk_ctx* c_, const Geo& g) : c(c_), saved(c_->ticket) {
        if (c->ticket_env < 0) c->ticket = (geo_blocks(c, g) <= 64 || (c->geo.world > 1 && g.L >= 8192)) ? 1 : 0;
    }
    ~TicketScope() { c->ticket = saved; }
};

template <int HB>
int vf_commit_hb(lbk_ctx* c, int obj, int h, const double* x, const double* g, const double* const* S,
                 const double* const* Y, const double* cs, const double* cy, double cg, double alpha,
                 const double* cand, double* xn, double* gn, double* so, double* yo, int wslot) {
    const NtScope nts(c, c->nt_vf);
    Geo geo = vgeo(c);
    const TicketScope tks(c, geo);
    Red r = kred(c, wslot);
    const VfBasis<HB> B = vf_basis<HB>(h, S, Y, cs, cy, cg);
    constexpr int K = LBK_VF_YB + 4 * HB + LBK_VF_NA;
    const int rc = launch(c, LBK_K_VF_COMMIT, 2.0 * h + 6.0, wslot, [&] {
        OBJ_DISPATCH(obj, {
            OpVfCommit<O_, HB, NT_> op{x, g, B, alpha, {cand[0]}, xn, gn, so, yo, geo.n, geo.n_loc};
            hipLaunchKernelGGL((k_vf_commit<O_, HB, NT_>), dim3(geo_blocks(c, geo)), dim3(LB_BLOCK), 0, c->stream, op,
                               geo, r);
        });
        return 0;
    }, K, false, &geo);
    if (rc || (c->geo.world == 1 && !c->comm)) return rc;
    return vf_exchange_ghosts(c, wslot, xn, gn, so, yo);
}

template <int HB>
int vf_dir_hb(lbk_ctx* c, int h, double* d, const double* g, const double* const* S, const double* const* Y,
              const double* cs, const double* cy, double cg) {
    const NtScope nts(c, c->nt_vf);
    const VfBasis<HB> B = vf_basis<HB>(h, S, Y, cs, cy, cg);
    const int64_t npair = c->geo.n_loc / 2;
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((npair + 255) / 256, 16384));
    return launch(c, LBK_K_VF_DIR, 2.0 * h + 2.0, -1, [&] {
        if (c->geo.n_loc <= 0) return;
        NT_DISPATCH(c, hipLaunchKernelGGL((k_vf_dir<HB, NT_>), dim3(nb), dim3(256), 0, c->stream, d, g, B,
                                          c->geo.n_loc));
    });
}
}  // namespace
extern "C" {

#define VF_BUCKETS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(10) X(12) X(16) X(20)

int lbk_vf_ghost_init(lbk_ctx* c, double* x, double* g, int wslot) {
    if (c->geo.world == 1) return 0;
    return vf_exchange_ghosts(c, wslot, x, g, nullptr, nullptr);
}

int lbk_vf_bucket(int h) {
    static const int hb[] = {0, 1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20};
    for (int v : hb)
        if (h <= v) return v;
    return -1;
}

int lbk_vf_commit(lbk_ctx* c, int obj, int h, const double* x, const double* g, const double* const* S,
                  const double* const* Y, const double* cs, const double* cy, double cg, double alpha,
                  const double* cand, double* xn, double* gn, double* so, double* yo, int wslot, int* hb_out) {
    const int hb = lbk_vf_bucket(h);
    if (hb < 0 || wslot < LBK_WSLOT0 || wslot >= LBK_WSLOT0 + LBK_NWSLOTS) {
        snprintf(c->err, sizeof c->err, "lbk_vf_commit: h=%d (max %d), slot %d", h, LBK_VF_HMAX, wslot);
        return -1;
    }
    *hb_out = hb;
    switch (hb) {
#define VF_CASE(HB) \
    case HB: return vf_commit_hb<HB>(c, obj, h, x, g, S, Y, cs, cy, cg, alpha, cand, xn, gn, so, yo, wslot);
        VF_BUCKETS(VF_CASE)
#undef VF_CASE
    }
    return -1;
}

int lbk_vf_dir(lbk_ctx* c, int h, double* d, const double* g, const double* const* S, const double* const* Y,
               const double* cs, const double* cy, double cg) {
    const int hb = lbk_vf_bucket(h);
    if (hb < 0) return -1;
    switch (hb) {
#define VF_CASE(HB) \
    case HB: return vf_dir_hb<HB>(c, h, d, g, S, Y, cs, cy, cg);
        VF_BUCKETS(VF_CASE)
#undef VF_CASE
    }
    return -1;
}

}  // extern "C"
