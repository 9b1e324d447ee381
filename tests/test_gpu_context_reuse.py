"""Contexts created one after another in one process (bench.py's sequence: the headline, its
one-GPU check, the vector-free line, configs[4]) and side by side: every solve must give the same
trajectory as the same solve on a context created first, whichever contexts ran or were freed
before it, with two contexts alive at once (each on its own stream) and after a context closed
with work still queued on another."""
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


def solve(n, m, ls, iters, seed, vector_free=False):
    x0 = L.x0_uniform(n, seed, -2.0, 2.0)
    with L.Context(n, m) as c:
        c.init("rosenbrock", x0, ls, tolerance=1e-5, vector_free=vector_free)
        r = c.step(iters)
        return r["f"], r["gnorm"], r["iterations"], c.get_x()


def test_sequential_contexts():
    first = solve(100_003, 5, "backtracking", 40, 1)
    others = [solve(300_001, 8, "wolfe", 20, 2), solve(20_000, 3, "interpolation", 30, 3),
              solve(100_003, 5, "backtracking", 40, 1, vector_free=True)]
    again = solve(100_003, 5, "backtracking", 40, 1)
    assert first[:3] == again[:3] and np.array_equal(bits(first[3]), bits(again[3]))
    assert all(np.isfinite(o[0]) for o in others)


def test_live_contexts_and_a_context_closed_mid_solve():
    n, m = 50_000, 5
    x0 = L.x0_uniform(n, 9, -2.0, 2.0)
    ref = solve(n, m, "backtracking", 30, 9)
    a, b = L.Context(n, m), L.Context(n, m)
    try:
        a.init("rosenbrock", x0, "backtracking", tolerance=1e-5)
        b.init("rosenbrock", x0, "backtracking", tolerance=1e-5)
        for _ in range(30):  # interleaved: the two streams run side by side
            ra, rb = a.step(1), b.step(1)
        assert ra["f"] == rb["f"] == ref[0] and np.array_equal(bits(a.get_x()), bits(ref[3]))
        assert np.array_equal(bits(b.get_x()), bits(ref[3]))
    finally:
        a.close()
        b.step(5)  # queued work still in flight when the context goes away
        b.close()
    assert solve(n, m, "backtracking", 30, 9)[:3] == ref[:3]
    with np.errstate(all="ignore"):
        o = O.lbfgs("rosenbrock", x0, "backtracking", m, 30, 1e-5, mode=O.CANON)
    assert np.array_equal(bits(ref[3]), bits(o["x"]))
