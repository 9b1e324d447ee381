"""Batched line-search trials (default on, LBFGS_BATCH=0 restores one pass per
step with d materialised first).

* The first commit of a backtracking iteration also reduces f at the search's second step
  a0 * beta, so a rejected first step needs no trial pass.
* A trial pass on a halving chain (backtracking alpha * beta, interpolation alpha * 0.5 once
  the reference's alpha_prev quirk makes delta 0) evaluates LBK_TRIALS_NC steps in one read of
  x and d; a Wolfe / backtracking-Wolfe pass evaluates f and g.d together.
* d stays unmaterialised (formed from r, s_{h-1} as the commit does) for the first two trial
  passes and the commit.
Every result must be the one-pass-per-step result bit for bit, and the canonical oracle's.
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


def same(a, b):
    for key in ("tr_f", "tr_gnorm", "x"):
        assert np.array_equal(bits(a[key]), bits(b[key])), key
    ta, tb = a["tr_alpha"], b["tr_alpha"]
    assert np.array_equal(np.isnan(ta), np.isnan(tb))
    assert np.array_equal(ta[~np.isnan(ta)], tb[~np.isnan(tb)])
    assert np.array_equal(a["tr_c1"], b["tr_c1"]) and np.array_equal(a["tr_c2"], b["tr_c2"])
    assert a["messages"] == b["messages"] and a["status"] == b["status"]


CASES = [("rosenbrock", 20_000, 5, "backtracking", 80), ("rosenbrock", 20_000, 5, "interpolation", 80),
         ("rosenbrock", 20_000, 5, "wolfe", 60), ("rosenbrock", 20_000, 5, "backtracking_wolfe", 40),
         ("quad_tridiag", 300_000, 20, "wolfe", 12), ("quad_tridiag", 300_000, 10, "backtracking", 30),
         ("rosenbrock", 1_000_003, 10, "backtracking", 40), ("rosenbrock", 1_000_003, 10, "interpolation", 30),
         ("quad_sep", 50_001, 3, "interpolation", 15), ("rosenbrock", 3, 1, "wolfe", 80)]


@pytest.mark.parametrize("obj,n,m,ls,iters", CASES)
def test_batched_trials_bit_identical(monkeypatch, obj, n, m, ls, iters):
    x0 = L.x0_uniform(n, 7, -2.0, 2.0)
    out = {}
    for batch in ("0", "1"):
        monkeypatch.setenv("LBFGS_BATCH", batch)
        with L.Context(n, m) as c:
            out[batch] = c.minimize(obj, x0, ls, iters, trace=True)
    a, b = out["0"], out["1"]
    same(a, b)
    assert b["passes"] <= a["passes"]
    assert b["bytes"] <= a["bytes"]
    o = O.lbfgs(obj, x0, ls, m, iters, 1e-5, mode=O.CANON)
    assert np.array_equal(bits(b["tr_f"]), bits(o["f"]))
    assert np.array_equal(b["tr_c1"], o["c1"]) and np.array_equal(b["tr_c2"], o["c2"])


def test_backtracking_rejections_cost_fewer_passes(monkeypatch):
    """Rosenbrock from U(-2, 2) rejects the unit step now and then: the batched run needs no trial
    pass for the second step and no k_last, and moves fewer bytes."""
    n, m, iters = 1_000_003, 10, 100
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    out = {}
    for batch in ("0", "1"):
        monkeypatch.setenv("LBFGS_BATCH", batch)
        with L.Context(n, m) as c:
            c.prof_reset()
            c.prof_enable(True)
            r = c.minimize("rosenbrock", x0, "backtracking", iters, trace=True)
            r["last"] = c.prof_get("last")["launches"]
            r["trials"] = c.prof_get("trial_f")["launches"]
            out[batch] = r
    a, b = out["0"], out["1"]
    same(a, b)
    assert a["trials_f"] > 0, "no rejected first step in this run: pick another"
    assert b["trials"] < a["trials"] and b["last"] < a["last"]
    assert b["bytes"] < a["bytes"]


@pytest.mark.parametrize("ls", ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"])
def test_standalone_line_search_batched(monkeypatch, ls):
    """lbfgs_line_search (the drop-in for line_search.cpp's four searches): same alpha with and
    without batching, on a direction where the unit step is rejected."""
    import ctypes as C

    n = 5000
    rs = np.random.RandomState(3)
    x = rs.uniform(-2, 2, n)
    g = O.grad("rosenbrock", x)
    d = -g  # |d| large: the unit step overshoots
    lib = L.lib()
    res = {}
    for batch in ("0", "1"):
        monkeypatch.setenv("LBFGS_BATCH", batch)
        with L.Context(n, 2) as c:
            a = C.c_double()
            k = L.constants()
            ptr = [v.ctypes.data_as(C.c_void_p) for v in (x, d, g)]
            rc = lib.lbfgs_line_search(c.h, L.OBJECTIVES["rosenbrock"], None, L.LINE_SEARCHES[ls],
                                       C.byref(k), *ptr, C.byref(a))
            assert rc == 0
            res[batch] = a.value
    assert res["0"] == res["1"] and res["1"] != 1.0  # the unit step was rejected
