#!/usr/bin/env python3
"""Generate golden fixtures from the REFERENCE itself (test infrastructure).

Runs oracle/_ref/ref_lbfgs — the reference's own sequential sources
(/root/reference/sequential-implementation/{lbfgs,vector_utils,line_search,benchmark,main}.cpp,
compiled unmodified by oracle/Makefile) driven by oracle/ref_driver.cpp, which only observes the
f/grad calls the reference LBFGS() makes. Each case is written as
  tests/golden/<case>.npz   arrays (float64 / uint64 only; load with allow_pickle=False)
  tests/golden/<case>.json  arguments + the reference's stdout
Only runnable where /root/reference exists (this container); the fixtures travel instead.

usage: python tests/golden/make_golden.py [case ...]
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_lbfgs")

# name: (objective, n, m, method, maxit, tol, seed, lo, hi, full_upto)
CASES = {
    # config 1 (BASELINE.json configs[0]): Rosenbrock n=1e4, m=5, backtracking, x0~U(-2,2) seed 42
    "rosen_n1e4_m5_bt": ("rosenbrock", 10000, 5, "backtracking", 1000, 1e-5, 42, -2.0, 2.0, 3),
    "rosen_n100_m5_bt": ("rosenbrock", 100, 5, "backtracking", 200, 1e-5, 42, -2.0, 2.0, 51),
    "rosen_n1e3_m10_bt_conv": ("rosenbrock", 1000, 10, "backtracking", 20000, 1e-5, 42, -2.0, 2.0, 1),
    "rosen_n1e4_m5_interp": ("rosenbrock", 10000, 5, "interpolation", 300, 1e-5, 42, -2.0, 2.0, 1),
    "rosen_n1e4_m5_wolfe": ("rosenbrock", 10000, 5, "wolfe", 300, 1e-5, 42, -2.0, 2.0, 1),
    "rosen_n1e4_m5_btw": ("rosenbrock", 10000, 5, "backtracking_wolfe", 300, 1e-5, 42, -2.0, 2.0, 1),
    "rosen_n1e5_m10_bt": ("rosenbrock", 100000, 10, "backtracking", 60, 1e-5, 42, -2.0, 2.0, 0),
    # config 4 family (generate_quadratic_function / _gradient, benchmark.cpp:16-56), Wolfe
    "qtri_n1e4_m20_wolfe": ("quad_tridiag", 10000, 20, "wolfe", 1000, 1e-5, 42, -2.0, 2.0, 2),
    "qtri_n1e5_m20_wolfe": ("quad_tridiag", 100000, 20, "wolfe", 1000, 1e-5, 42, -2.0, 2.0, 0),
    "qtri_n1e4_m10_bt": ("quad_tridiag", 10000, 10, "backtracking", 400, 1e-5, 42, -2.0, 2.0, 1),
    # main.cpp:24-58 exactly: separable quadratic, dim 1e4, U(-1000,1000) seed 42, 15000 it, m 10
    "qsep_main": ("quad_sep", 10000, 10, "backtracking", 15000, 1e-8, 42, -1000.0, 1000.0, 2),
    # edge cases
    "rosen_n1_bt": ("rosenbrock", 1, 5, "backtracking", 10, 1e-5, 42, -2.0, 2.0, 2),
    "rosen_n2_m3_bt": ("rosenbrock", 2, 3, "backtracking", 500, 1e-5, 42, -2.0, 2.0, 20),
    "rosen_n3_m1_wolfe": ("rosenbrock", 3, 1, "wolfe", 300, 1e-5, 42, -2.0, 2.0, 20),
    "rosen_n4097_m7_interp": ("rosenbrock", 4097, 7, "interpolation", 150, 1e-5, 7, -2.0, 2.0, 2),
}

# Guard paths of lbfgs.cpp driven by our own stress objectives (oracle/ref_driver.cpp), run by
# the reference itself: invalid rho + non-descent + skipped updates (tiny scale, tol 0), invalid
# gamma (y.y overflow), line-search failure (Wolfe on a double well).
STRESS = {
    "stress_tiny_sq_bt": ("stress_tiny_sq", 10, 3, "backtracking", 30, 0.0, 42, -1e-155, 1e-155, 0),
    "stress_tiny_sq_interp": ("stress_tiny_sq", 10, 3, "interpolation", 30, 0.0, 42, -1e-155, 1e-155, 0),
    "stress_tiny_sq_wolfe": ("stress_tiny_sq", 10, 3, "wolfe", 30, 0.0, 42, -1e-155, 1e-155, 0),
    "stress_tiny_sq_btw": ("stress_tiny_sq", 10, 3, "backtracking_wolfe", 30, 0.0, 42, -1e-155, 1e-155, 0),
    "stress_scaled_sq_bt": ("stress_scaled_sq", 10, 3, "backtracking", 4, 1e-5, 42, -1e-10, 1e-10, 0),
    "stress_quartic_well_wolfe": ("stress_quartic_well", 8, 3, "wolfe", 50, 1e-8, 42, -1.3, -1.2, 1),
    "stress_quartic_well_n1_wolfe": ("stress_quartic_well", 1, 3, "wolfe", 50, 1e-8, 42, -1.5, -1.0, 1),
    # the same guards through a benchmark objective (the device's fused path): the tridiagonal
    # quadratic at the 1e-155 scale (invalid rho; Wolfe: line-search failure)
    "stress_qtri_tiny_bt": ("quad_tridiag", 10, 3, "backtracking", 30, 0.0, 42, -1e-155, 1e-155, 0),
    "stress_qtri_tiny_wolfe": ("quad_tridiag", 10, 3, "wolfe", 30, 0.0, 42, -1e-155, 1e-155, 0),
    "stress_qtri_tiny_btw": ("quad_tridiag", 10, 3, "backtracking_wolfe", 30, 0.0, 42, -1e-155, 1e-155, 0),
    # edges of the loop itself: no iteration at all (maxit = 0), x0 at the minimiser (g = 0 exactly:
    # converged before the first step), a tolerance every |g| meets, a one-pair history, a
    # history longer than the run, n = 1 of the tridiagonal quadratic (both stencil edges at once),
    # tolerance 0 (runs to the cap or a failed search)
    "stress_edge_maxit0_bt": ("rosenbrock", 100, 5, "backtracking", 0, 1e-5, 42, -2.0, 2.0, 0),
    "stress_edge_optimum_wolfe": ("rosenbrock", 50, 5, "wolfe", 10, 1e-5, 42, 1.0, 1.0, 0),
    "stress_edge_qsep_optimum_interp": ("quad_sep", 10, 3, "interpolation", 10, 1e-5, 42, 1.0, 1.0, 0),
    "stress_edge_hugetol_btw": ("rosenbrock", 200, 3, "backtracking_wolfe", 10, 1e9, 42, -2.0, 2.0, 0),
    "stress_edge_m1_bt": ("rosenbrock", 1000, 1, "backtracking", 60, 1e-5, 42, -2.0, 2.0, 0),
    "stress_edge_m1_interp": ("rosenbrock", 1000, 1, "interpolation", 60, 1e-5, 42, -2.0, 2.0, 0),
    "stress_edge_qtri_n1_wolfe": ("quad_tridiag", 1, 3, "wolfe", 30, 1e-8, 42, -2.0, 2.0, 0),
    "stress_edge_m20_n3_bt": ("rosenbrock", 3, 20, "backtracking", 500, 1e-10, 42, -2.0, 2.0, 0),
    "stress_edge_tol0_n2_bt": ("rosenbrock", 2, 2, "backtracking", 300, 0.0, 5, -2.0, 2.0, 0),
}
CASES.update(STRESS)

KATS = {"kat_n1000": (1000, 7), "kat_n5": (5, 3)}


def run_case(name, spec, tmp):
    obj, n, m, method, maxit, tol, seed, lo, hi, full = spec
    prefix = os.path.join(tmp, name)
    cmd = [REF_BIN, obj, str(n), str(m), method, str(maxit), repr(tol), str(seed), repr(lo),
           repr(hi), prefix, str(full)]
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=600)
    f_calls = np.fromfile(prefix + ".f.bin", dtype=np.float64)
    graw = np.fromfile(prefix + ".g.bin", dtype=np.uint64).reshape(-1, 5)
    grad_c = graw[:, 0:2].copy()
    grad_norm = graw[:, 2].copy().view(np.float64)
    grad_nf = graw[:, 4].copy()
    xf = np.fromfile(prefix + ".x.bin", dtype=np.float64)
    x_full = xf.reshape(-1, n) if xf.size else np.zeros((0, n))
    ret = np.fromfile(prefix + ".ret.bin", dtype=np.uint64)
    ret_c = ret[:2].copy()
    arrays = dict(f_calls=f_calls, grad_c=grad_c, grad_norm=grad_norm, grad_nf=grad_nf,
                  x_full=x_full, ret_c=ret_c)
    if n <= 10000:
        arrays["ret_x"] = ret[2:].copy().view(np.float64)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    meta = dict(case=name, objective=obj, n=n, m=m, method=method, maxit=maxit, tol=tol,
                seed=seed, lo=lo, hi=hi, full_upto=full, stdout=out.stdout,
                generator="oracle/_ref/ref_lbfgs (reference sequential-implementation sources)")
    with open(os.path.join(HERE, name + ".json"), "w") as fp:
        json.dump(meta, fp, indent=1)
    print(f"{name}: {len(f_calls)} f-calls, {len(grad_c)} grad-calls, stdout={out.stdout.strip()[-60:]!r}")


def run_kat(name, n, seed, tmp):
    prefix = os.path.join(tmp, name)
    subprocess.run([REF_BIN, "kat", str(n), str(seed), prefix], check=True, timeout=60)
    raw = np.fromfile(prefix + ".kat.bin", dtype=np.float64)
    o = 0

    def take(k):
        nonlocal o
        v = raw[o:o + k]
        o += k
        return v.copy()

    x = take(n)
    arrays = dict(x=x, f_rosen=take(1), g_rosen=take(n), f_qtri=take(1), g_qtri=take(n),
                  f_qsep=take(1), g_qsep=take(n))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    with open(os.path.join(HERE, name + ".json"), "w") as fp:
        json.dump(dict(case=name, n=n, seed=seed, lo=-2.0, hi=2.0,
                       generator="oracle/_ref/ref_lbfgs kat"), fp, indent=1)
    print(f"{name}: ok")


def main(argv):
    if not os.path.exists(REF_BIN):
        sys.exit("build the reference first: make -C oracle ref")
    names = argv or list(CASES) + list(KATS)
    with tempfile.TemporaryDirectory() as tmp:
        for nm in names:
            if nm in CASES:
                run_case(nm, CASES[nm], tmp)
            elif nm in KATS:
                run_kat(nm, *KATS[nm], tmp)
            else:
                sys.exit(f"unknown case {nm}")


if __name__ == "__main__":
    main(sys.argv[1:])
