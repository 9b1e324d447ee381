/* constants.h — drop-in for parallel-implementation/constants.h:1-23 (the CUDA path's
 * profile: C2 = 0.7, plus the unused MAX/MIN_STEP_SIZE). Runtime equivalent:
 * lbfgs_constants_cuda() in lbfgs_hip.h. Like the reference, it cannot be included together
 * with config.h in one translation unit. */
#ifndef CONSTANTS_H
#define CONSTANTS_H

constexpr double C1 = 1e-4;
constexpr double C2 = 0.7;
constexpr double INITIAL_STEP_SIZE = 1.0;
constexpr double BACKTRACKING_ALPHA = 0.5;
constexpr double BACKTRACKING_TOL = 1e-8;
constexpr double WOLFE_INTERP_MIN = 1e-10;
constexpr double WOLFE_INTERP_MAX = 10.0;
constexpr double MAX_STEP_SIZE = 10.0;
constexpr double MIN_STEP_SIZE = 1e-6;

#endif  // CONSTANTS_H
