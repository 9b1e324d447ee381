"""LBFGS_FLAG_CUDA_COMPAT: the product reproduces the reference's CUDA path (LBFGS_CUDA,
parallel-implementation/L-BFGS.cu:105-380) - its loop on the device, the host line searches of
parallel-implementation/line_search.cpp (cached bisection backtracking-Wolfe, 0.5 floors,
safeguarded cubic), the stale iteration-0 gradient those searches get (L-BFGS.cu:293), the skipped
pairs with stale alpha/rho (:222-223), gamma = 1 when no pair is accepted (:237-262), the ring
slot k % m written unconditionally (:332-333) and the convergence test after the step (:353).

Checked bit for bit against the oracle's restatement (orc_lbfgs_cuda, ORC_CANON): trace f / |g| /
step / x checksums, the final x, the messages, status and iteration count. The restatement's line
searches are pinned to the reference's line_search.cpp (tests/test_oracle_cuda_path.py); its loop
is not (cuBLAS does not run here): parity unpinned for the loop, as DESIGN.md §6 says.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402
import oracle_lib as O  # noqa: E402

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


# (objective, n, m, search, maxit, tol, x0 lo, hi, seed): several hit the s.y <= 1e-10 skip many
# times (counted by the oracle: tests/test_oracle_cuda_path.py::test_cuda_path_skips_pairs)
CASES = [
    ("rosenbrock", 1, 3, "backtracking", 50, 1e-5, -2.0, 2.0, 42),
    ("rosenbrock", 64, 5, "backtracking", 12, 1e-5, -2.0, 2.0, 42),
    ("rosenbrock", 64, 5, "interpolation", 12, 1e-5, -2.0, 2.0, 42),
    ("rosenbrock", 64, 5, "wolfe", 12, 1e-5, -2.0, 2.0, 42),
    ("rosenbrock", 64, 5, "backtracking_wolfe", 12, 1e-5, -2.0, 2.0, 42),
    ("rosenbrock", 20, 3, "interpolation", 2000, 1e-13, -2.0, 2.0, 42),
    ("rosenbrock", 100, 5, "backtracking", 3000, 1e-12, -2.0, 2.0, 42),
    ("rosenbrock", 1000, 10, "wolfe", 200, 1e-12, -2.0, 2.0, 42),
    ("rosenbrock", 4097, 7, "backtracking_wolfe", 100, 1e-8, -2.0, 2.0, 9),
    ("quad_tridiag", 4000, 7, "backtracking_wolfe", 300, 1e-10, -2.0, 2.0, 42),
    ("quad_tridiag", 4000, 10, "wolfe", 60, 1e-8, -2.0, 2.0, 42),
    ("quad_tridiag", 100_003, 5, "backtracking", 40, 1e-8, -2.0, 2.0, 3),
    ("quad_sep", 1000, 5, "backtracking", 30, 1e-5, 1 - 1e-7, 1 + 1e-7, 42),
    ("quad_sep", 1000, 5, "interpolation", 30, 1e-5, -2.0, 2.0, 5),
    # edges: no iteration, x0 at the minimiser (g = 0: the step is taken, then |g| <= tol), n = 1
    ("rosenbrock", 100, 5, "backtracking", 0, 1e-5, -2.0, 2.0, 42),
    ("rosenbrock", 50, 5, "wolfe", 10, 1e-5, 1.0, 1.0, 42),
    ("quad_tridiag", 1, 3, "backtracking_wolfe", 30, 1e-8, -2.0, 2.0, 42),
]
_ids = [f"{c[0]}-n{c[1]}-m{c[2]}-{c[3]}-it{c[4]}" for c in CASES]


@pytest.mark.parametrize("case", CASES, ids=_ids)
def test_cuda_compat_bit_exact_vs_oracle(case):
    obj, n, m, ls, maxit, tol, lo, hi, seed = case
    x0 = O.x0_uniform(n, seed, lo, hi)
    o = O.lbfgs(obj, x0, ls, m, maxit, tol, mode=O.CANON, cuda=True, consts=O.CONSTANTS_H)
    with L.Context(n, m) as c:
        r = c.minimize(obj, x0, ls, maxit, tolerance=tol, trace=True,
                       cuda_compat=True, consts=L.constants("cuda"))
    assert r["status"] == o["status"]
    assert r["iterations"] == o["iters"]
    assert len(r["tr_f"]) == len(o["f"])
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
    assert np.array_equal(bits(r["tr_alpha"]), bits(o["alpha"]))
    assert np.array_equal(r["tr_c1"], o["c1"]) and np.array_equal(r["tr_c2"], o["c2"])
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
    assert r["messages"] == o["messages"]


# LBFGS_FLAG_CUDA_VARIANT: the four variant files' loops with their inline searches (current
# gradient, f(x_host) of the last transferred trial point, initial_f in f_prev / f_lo). The n = 5
# backtracking case prints L-BFGS-Backtracking.cu's "very small step size" warning.
VARIANT_CASES = [
    ("rosenbrock", 64, 5, "backtracking", 40, 1e-5, 42),
    ("rosenbrock", 5, 2, "backtracking", 3000, 1e-14, 2),
    ("rosenbrock", 1000, 10, "interpolation", 300, 1e-8, 42),
    ("rosenbrock", 20, 3, "interpolation", 2000, 1e-13, 42),
    ("rosenbrock", 1000, 10, "wolfe", 300, 1e-8, 42),
    ("rosenbrock", 20, 3, "wolfe", 2000, 1e-13, 42),
    ("rosenbrock", 1000, 10, "backtracking_wolfe", 300, 1e-8, 42),
    ("rosenbrock", 2, 2, "backtracking_wolfe", 3000, 1e-14, 1),
    ("quad_tridiag", 4000, 7, "wolfe", 100, 1e-8, 42),
    ("quad_tridiag", 100_003, 5, "backtracking_wolfe", 40, 1e-8, 3),
    ("quad_sep", 1000, 5, "interpolation", 30, 1e-5, 5),
    ("rosenbrock", 100, 5, "interpolation", 0, 1e-5, 42),
    ("quad_tridiag", 1, 3, "wolfe", 30, 1e-8, 42),
]


@pytest.mark.parametrize("case", VARIANT_CASES, ids=[f"{c[0]}-n{c[1]}-m{c[2]}-{c[3]}" for c in VARIANT_CASES])
def test_cuda_variant_bit_exact_vs_oracle(case):
    obj, n, m, ls, maxit, tol, seed = case
    x0 = O.x0_uniform(n, seed, -2.0, 2.0)
    o = O.lbfgs(obj, x0, ls, m, maxit, tol, mode=O.CANON, cuda=2, consts=O.CONSTANTS_H)
    with L.Context(n, m) as c:
        r = c.minimize(obj, x0, ls, maxit, tolerance=tol, trace=True, cuda_compat=True, cuda_variant=True,
                       consts=L.constants("cuda"))
    assert r["status"] == o["status"] and r["iterations"] == o["iters"]
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
    assert np.array_equal(bits(r["tr_alpha"]), bits(o["alpha"]))
    assert np.array_equal(r["tr_c1"], o["c1"]) and np.array_equal(r["tr_c2"], o["c2"])
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
    assert r["messages"] == o["messages"]


def test_cuda_compat_refuses_what_the_cuda_path_lacks():
    """the CUDA path has no vector-free form, no host objective here and no sharding"""
    n = 257
    x0 = O.x0_uniform(n, 1, -2.0, 2.0)
    with L.Context(n, 5) as c:
        with pytest.raises(L.LbfgsError):
            c.minimize("rosenbrock", x0, "backtracking", 5, cuda_compat=True, vector_free=True)
        with pytest.raises(L.LbfgsError):
            c.minimize("host", x0, "backtracking", 5, cuda_compat=True,
                       f=lambda x: float(np.sum(x * x)), grad=lambda x: 2 * x)
        with pytest.raises(L.LbfgsError):  # the variant flag alone
            c.minimize("rosenbrock", x0, "backtracking", 5, cuda_variant=True)
        # the context is still usable after a refusal
        r = c.minimize("rosenbrock", x0, "backtracking", 5, cuda_compat=True,
                       consts=L.constants("cuda"))
        assert r["iterations"] >= 1
