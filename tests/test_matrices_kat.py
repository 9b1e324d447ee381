"""Known-answer tests from the reference's dense quadratics (sequential-implementation/matrices.h,
extracted as data into tests/golden/matrices.npz by tests/golden/make_matrices.py):
f(x) = x^T A x + b^T x, A symmetric positive definite (n = 2 ... 500), with the header's
minimizers x* (2 A x* + b = 0, printed to 5 decimals, float-rounded).

The objective comes through the general-objective path (the reference's LBFGS takes any
std::function, lbfgs.h:9-10): the oracle's ORC_OBJ_HOST on CPU, LBFGS_OBJ_HOST through the
C ABI on the GPU (host f/grad callbacks, device two-loop, line search and commit).

  * CPU: the oracle converges to x* within 1e-4 (max abs) for every n and line search
    (|x - x*| <= |g| / (2 lambda_min) <= 1e-5 / 0.2, plus the 5e-6 printing error of x*);
  * GPU: the device solver's trajectory is bit-exact against the oracle's canonical mode with
    the same callbacks, and ends at the same x.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import oracle_lib as O  # noqa: E402

SIZES = [2, 3, 4, 5, 10, 50, 100, 500]
LINE_SEARCHES = ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"]
_data = np.load(os.path.join(ROOT, "tests", "golden", "matrices.npz"), allow_pickle=False)


def problem(n):
    A, b, xs = _data[f"mat{n}"], _data[f"linear{n}"], _data[f"minimum{n}"]

    def f(x):
        return float(x @ (A @ x) + b @ x)

    def grad(x):
        return 2.0 * (A @ x) + b

    return A, b, xs, f, grad


def x0(n):
    return O.x0_uniform(n, 42, -2.0, 2.0)


@pytest.mark.parametrize("n", SIZES)
def test_fixture_consistent(n):
    A, b, xs, _, _ = problem(n)
    assert np.array_equal(A, A.T)
    assert np.linalg.eigvalsh(A).min() > 0.1
    assert np.abs(2.0 * A @ xs + b).max() < 1e-4 * max(1.0, np.abs(b).max()) * n ** 0.5


@pytest.mark.parametrize("ls", LINE_SEARCHES)
@pytest.mark.parametrize("n", SIZES)
def test_oracle_reaches_known_minimum(n, ls):
    _, _, xs, f, grad = problem(n)
    r = O.lbfgs("host", x0(n), ls, 5, 1000, 1e-5, mode=O.SEQ, f=f, grad=grad)
    assert r["status"] == "converged", r["messages"][-300:]
    assert np.abs(r["x"] - xs).max() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("ls", LINE_SEARCHES)
@pytest.mark.parametrize("n", SIZES)
def test_gpu_host_objective_bit_exact_and_known_minimum(n, ls):
    import lbfgs_amd as L

    _, _, xs, f, grad = problem(n)
    o = O.lbfgs("host", x0(n), ls, 5, 1000, 1e-5, mode=O.CANON, f=f, grad=grad)
    with L.Context(n, 5) as c:
        r = c.minimize("host", x0(n), ls, 1000, f=f, grad=grad, trace=True)
    assert r["status"] == o["status"] == "converged"
    assert r["iterations"] == o["iters"]
    assert np.array_equal(r["tr_f"].view(np.uint64), o["f"].view(np.uint64))
    assert np.array_equal(r["x"].view(np.uint64), o["x"].view(np.uint64))
    assert np.abs(r["x"] - xs).max() < 1e-4


@pytest.mark.parametrize("ls", LINE_SEARCHES)
@pytest.mark.parametrize("n", SIZES)
def test_oracle_dense_objective_reaches_known_minimum(n, ls):
    """The device dense-quadratic objective's restatement (ORC_OBJ_DENSE: rows of A x in the
    device's lane-strided order) solves every matrices.h problem to the header's minimizer."""
    A, b, xs, _, _ = problem(n)
    O.dense_set(A, b)
    r = O.lbfgs("dense", x0(n), ls, 5, 1000, 1e-5, mode=O.CANON)
    assert r["status"] == "converged", r["messages"][-300:]
    assert np.abs(r["x"] - xs).max() < 1e-4
