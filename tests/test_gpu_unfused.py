"""Unfused mode (LBFGS_FLAG_UNFUSED, BASELINE configs[1] "unfused per-vector kernels"): one
launch per BLAS-1 operation in the shape of parallel-implementation/L-BFGS.cu:208-280 — a dot
and an update launch per pair and loop, gamma scaling and d = -r separately, a materialised
trial point x + alpha d and f evaluated on it, the commit as point / eval / s / y / dots.

The fused and unfused paths must give the same iterates bit for bit (same canonical
reductions, same operand order of every elementwise update), and both equal the oracle's
canonical mode.
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

CASES = ["rosen_n1e4_m5_bt", "rosen_n1e4_m5_interp", "rosen_n1e4_m5_wolfe", "rosen_n1e4_m5_btw",
         "qtri_n1e4_m10_bt", "qtri_n1e5_m20_wolfe", "rosen_n4097_m7_interp", "rosen_n1_bt",
         "rosen_n3_m1_wolfe", "qsep_main", "rosen_n1e5_m10_bt"]


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def run(meta, unfused):
    x0 = L.x0_uniform(meta["n"], meta["seed"], meta["lo"], meta["hi"])
    with L.Context(meta["n"], meta["m"]) as c:
        return c.minimize(meta["objective"], x0, meta["method"], meta["maxit"], tolerance=meta["tol"],
                          trace=True, unfused=unfused)


def same_trajectory(a, b):
    assert a["status"] == b["status"] and a["iterations"] == b["iterations"]
    for k in ("tr_f", "tr_gnorm", "x"):
        assert np.array_equal(bits(a[k]), bits(b[k])), k
    assert np.array_equal(a["tr_c1"], b["tr_c1"]) and np.array_equal(a["tr_c2"], b["tr_c2"])
    a1, a2 = a["tr_alpha"], b["tr_alpha"]
    assert np.array_equal(np.isnan(a1), np.isnan(a2))
    assert np.array_equal(a1[~np.isnan(a1)], a2[~np.isnan(a2)])
    assert a["messages"] == b["messages"]


@pytest.mark.parametrize("name", CASES)
def test_unfused_bit_exact_vs_fused_and_oracle(name):
    meta, _ = O.load_golden(name)
    ru = run(meta, True)
    rf = run(meta, False)
    same_trajectory(ru, rf)
    x0 = O.x0_uniform(meta["n"], meta["seed"], meta["lo"], meta["hi"])
    o = O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"], mode=O.CANON)
    assert np.array_equal(bits(ru["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(ru["x"]), bits(o["x"]))
    # more launches, more bytes: every dot and update is its own pass
    assert ru["passes"] >= rf["passes"]
    if ru["iterations"] > 0:
        assert ru["passes"] > rf["passes"]


def test_unfused_nontemporal_path_bit_exact(monkeypatch):
    """the non-temporal load/store variant of k_update (vectors > 128 MiB by default; forced
    here) gives the same bits"""
    meta, _ = O.load_golden("rosen_n1e4_m5_bt")
    monkeypatch.setenv("LBFGS_NT", "1")
    ru = run(meta, True)
    monkeypatch.delenv("LBFGS_NT")
    same_trajectory(ru, run(meta, False))


def test_unfused_steps_match_fused_steps_at_scale():
    """n = 3e6 (odd, many segments), 12 iterations through solver_init/step"""
    n, m = 3_000_001, 10
    x0 = L.x0_uniform(n, 7, -2.0, 2.0)
    out = []
    for unfused in (False, True):
        with L.Context(n, m) as c:
            c.init("rosenbrock", x0, "backtracking", trace=True, unfused=unfused)
            c.step(12)
            out.append((c.trace(), c.get_x()))
    (t1, x1), (t2, x2) = out
    assert np.array_equal(bits(t1["tr_f"]), bits(t2["tr_f"]))
    assert np.array_equal(bits(x1), bits(x2))


def test_unfused_rejects_host_objective():
    with L.Context(10, 3) as c:
        with pytest.raises(L.LbfgsError):
            c.minimize("host", np.zeros(10), "backtracking", 5, f=lambda x: 0.0, grad=lambda x: x,
                       unfused=True)
