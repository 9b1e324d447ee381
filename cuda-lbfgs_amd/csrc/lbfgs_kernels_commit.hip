// lbfgs_kernels_commit.hip — lbk_commit and lbk_trials (the many OpCommit / OpTrials
// instantiations), a translation unit of their own so the build runs in parallel.
#include "lbfgs_kernels_impl.h"

extern "C" {

int lbk_commit(lbk_ctx* c, int obj, int dmode, const double* x, const double* dsrc, const double* s_last,
               const double* gg, double rho, int ref_beta, int ref_alpha, double alpha, double* xn, double* gn,
               double* s_out, double* y_out, int slot, double cand) {
    Geo g = kgeo(c);
    // the candidate step rides the first (speculative) commit of the direction modes
    const bool with_cand = cand > 0.0 && obj != LBK_OBJ_NONE && dmode != LBK_D_BUF;
    const int K = with_cand ? 8 : 7;
    Red r = kred(c, slot, K);
    DirArgs da = {dsrc, s_last, gg, 0.0, nullptr, nullptr, rho,
                  (dmode == LBK_D_BUF || dmode == LBK_D_TWOLOOP) ? ghost_ptr(c) : nullptr, c->geo.g_lo, c->geo.g_hi};
    if (dmode == LBK_D_TWOLOOP) {
        da.pa = sref(c, ref_alpha);
        da.pb = sref(c, ref_beta);
        g.ppart = take_pending(c, ref_beta);
    }
    double passes = 4.0 + (dmode == LBK_D_BUF ? 3.0 : dmode == LBK_D_NEG_G ? 2.0 : 4.0);
    if (with_cand) {
        return launch(c, LBK_K_COMMIT, passes, slot, [&] {
            if (dmode == LBK_D_NEG_G) {
                OBJ_DISPATCH(obj, hipLaunchKernelGGL((k_commit<O_, LBK_D_NEG_G, NT_, true>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, x, da, alpha, xn, gn, s_out, y_out, g, r, cand));
            } else {
                OBJ_DISPATCH(obj, hipLaunchKernelGGL((k_commit<O_, LBK_D_TWOLOOP, NT_, true>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, x, da, alpha, xn, gn, s_out, y_out, g, r, cand));
            }
            return 0;
        }, 8);
    }
    return launch(c, LBK_K_COMMIT, passes, slot, [&] {
        if (obj == LBK_OBJ_NONE) {
            NT_DISPATCH(c, switch (dmode) {
                case LBK_D_BUF: hipLaunchKernelGGL((k_commit<LBK_OBJ_NONE, LBK_D_BUF, NT_>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, x, da, alpha, xn, gn, s_out, y_out, g, r); break;
                case LBK_D_NEG_G: hipLaunchKernelGGL((k_commit<LBK_OBJ_NONE, LBK_D_NEG_G, NT_>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, x, da, alpha, xn, gn, s_out, y_out, g, r); break;
                default: hipLaunchKernelGGL((k_commit<LBK_OBJ_NONE, LBK_D_TWOLOOP, NT_>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, x, da, alpha, xn, gn, s_out, y_out, g, r); break;
            });
            return 0;
        }
        switch (dmode) {
            case LBK_D_BUF:
                OBJ_DISPATCH(obj, hipLaunchKernelGGL((k_commit<O_, LBK_D_BUF, NT_>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, x, da, alpha, xn, gn, s_out, y_out, g, r));
                break;
            case LBK_D_NEG_G:
                OBJ_DISPATCH(obj, hipLaunchKernelGGL((k_commit<O_, LBK_D_NEG_G, NT_>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, x, da, alpha, xn, gn, s_out, y_out, g, r));
                break;
            default:
                OBJ_DISPATCH(obj, hipLaunchKernelGGL((k_commit<O_, LBK_D_TWOLOOP, NT_>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, x, da, alpha, xn, gn, s_out, y_out, g, r));
                break;
        }
        return 0;
    }, 7);
}

int lbk_trials(lbk_ctx* c, int obj, int dmode, const double* x, const double* dsrc, const double* s_last,
               const double* gg, double rho, int ref_beta, int ref_alpha, const double* alphas, int nc, int dphi,
               int slot) {
    if (!((nc == 1 && dphi) || (nc == LBK_TRIALS_NC && !dphi) || (nc == 1 && !dphi)) || obj == LBK_OBJ_NONE) {
        snprintf(c->err, sizeof c->err, "lbk_trials: nc=%d dphi=%d obj=%d", nc, dphi, obj);
        return -1;
    }
    Geo g = kgeo(c);
    const int K = nc + (dphi ? 1 : 0);
    Red r = kred(c, slot, K);
    DirArgs da = {dsrc, s_last, gg, 0.0, nullptr, nullptr, rho,
                  (dmode == LBK_D_BUF || dmode == LBK_D_TWOLOOP) ? ghost_ptr(c) : nullptr, c->geo.g_lo, c->geo.g_hi};
    if (dmode == LBK_D_TWOLOOP) {
        da.pa = sref(c, ref_alpha);
        da.pb = sref(c, ref_beta);
        g.ppart = take_pending(c, ref_beta);
    }
    const double passes = dmode == LBK_D_TWOLOOP ? 3.0 : 2.0;
    const int kind = dphi ? LBK_K_TRIAL_FG : LBK_K_TRIAL_F;
#define TRIALS_LAUNCH(DM, NCC, DP)                                                                             \
    OBJ_DISPATCH(obj, {                                                                                    \
        OpTrials<O_, DM, NCC, DP, NT_> op{x, da, {}, c->geo.n, c->geo.n_loc};                               \
        for (int j = 0; j < NCC; ++j) op.a[j] = alphas[j];                                                   \
        hipLaunchKernelGGL((k_trials<O_, DM, NCC, DP, NT_>), dim3(nblocks(c)), dim3(LB_BLOCK), 0, c->stream, g, r, \
                           op);                                                                            \
    })
#define TRIALS_DM(DM)                                                   \
    if (nc == 1 && dphi) {                                              \
        TRIALS_LAUNCH(DM, 1, true);                                     \
    } else if (nc == 1) {                                               \
        TRIALS_LAUNCH(DM, 1, false);                                    \
    } else {                                                            \
        TRIALS_LAUNCH(DM, LBK_TRIALS_NC, false);                        \
    }
    return launch(c, kind, passes, slot, [&] {
        switch (dmode) {
            case LBK_D_BUF: TRIALS_DM(LBK_D_BUF) break;
            case LBK_D_NEG_G: TRIALS_DM(LBK_D_NEG_G) break;
            default: TRIALS_DM(LBK_D_TWOLOOP) break;
        }
        return 0;
    }, K);
#undef TRIALS_DM
#undef TRIALS_LAUNCH
}

}  // extern "C"
