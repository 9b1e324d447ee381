"""Dense quadratic objective on the device (LBFGS_OBJ_DENSE_QUAD): the
known-answer problems of the reference's sequential-implementation/matrices.h, f = x'Ax + b'x with
2 A x* + b = 0 (A, b, x* extracted as data into tests/golden/matrices.npz).

* f and grad at a point bit-exact against the oracle's restatement (rows of A x in the device's
  lane-strided order, f terms in the canonical order);
* whole solves bit-exact against the oracle for every size and line search, reaching the header's
  minimizer;
* the C++ drop-in recognises lbfgs_amd::dense_quadratic_function / _gradient and runs them on the
  device (tests/cxx).
"""
import os
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402
import oracle_lib as O  # noqa: E402

pytestmark = pytest.mark.gpu

SIZES = [2, 3, 4, 5, 10, 50, 100, 500]
LINE_SEARCHES = ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"]
_data = np.load(os.path.join(ROOT, "tests", "golden", "matrices.npz"), allow_pickle=False)


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def problem(n):
    return _data[f"mat{n}"], _data[f"linear{n}"], _data[f"minimum{n}"]


@pytest.mark.parametrize("n", SIZES + [1000, 4097])
def test_dense_objective_bit_exact(n):
    if n in SIZES:
        A, b, _ = problem(n)
    else:  # larger SPD matrices of the same form (several row waves, partial last wave)
        rs = np.random.RandomState(n)
        M = rs.uniform(-1, 1, (n, n))
        A = (M + M.T) / (2 * n) + np.eye(n)
        b = rs.uniform(-1, 1, n)
    x = O.x0_uniform(n, 5, -2.0, 2.0)
    O.dense_set(A, b)
    with L.Context(n, 2) as c:
        c.set_dense_quadratic(A, b)
        f, g = c.objective("dense", x)
    assert bits([f])[0] == bits([O.f("dense", x, O.CANON)])[0]
    assert np.array_equal(bits(g), bits(O.grad("dense", x)))
    assert np.allclose(g, 2.0 * A @ x + b, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("ls", LINE_SEARCHES)
@pytest.mark.parametrize("n", SIZES)
def test_dense_solve_bit_exact_and_known_minimum(n, ls):
    A, b, xs = problem(n)
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    O.dense_set(A, b)
    o = O.lbfgs("dense", x0, ls, 5, 1000, 1e-5, mode=O.CANON)
    with L.Context(n, 5) as c:
        c.set_dense_quadratic(A, b)
        r = c.minimize("dense", x0, ls, 1000, trace=True)
    assert r["status"] == o["status"] == "converged" and r["iterations"] == o["iters"]
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
    assert np.array_equal(r["tr_c1"], o["c1"]) and np.array_equal(r["tr_c2"], o["c2"])
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
    assert r["messages"] == o["messages"]
    assert np.abs(r["x"] - xs).max() < 1e-4


def test_dense_needs_its_data():
    with L.Context(10, 3) as c:
        with pytest.raises(L.LbfgsError):
            c.minimize("dense", np.zeros(10), "backtracking", 10)


def test_dense_device_vs_host_callbacks_timing():
    """n = 500 (mat500): the same solve with the objective on the device and as numpy host
    callbacks; both converge to the header's minimizer. Reported, not asserted as a speed-up."""
    A, b, xs = problem(500)
    x0 = O.x0_uniform(500, 42, -2.0, 2.0)
    with L.Context(500, 5) as c:
        c.set_dense_quadratic(A, b)
        c.minimize("dense", x0, "wolfe", 1000)  # warm-up
        t0 = time.perf_counter()
        rd = c.minimize("dense", x0, "wolfe", 1000)
        td = time.perf_counter() - t0
        t0 = time.perf_counter()
        rh = c.minimize("host", x0, "wolfe", 1000, f=lambda x: float(x @ (A @ x) + b @ x),
                        grad=lambda x: 2.0 * (A @ x) + b)
        th = time.perf_counter() - t0
    print(f"\nmat500 wolfe: device {rd['iterations']} it in {td * 1e3:.2f} ms, host callbacks "
          f"{rh['iterations']} it in {th * 1e3:.2f} ms")
    assert np.abs(rd["x"] - xs).max() < 1e-4 and np.abs(rh["x"] - xs).max() < 1e-4
