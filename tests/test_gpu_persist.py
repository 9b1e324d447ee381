"""The persistent large-n form: LBFGS_PERSIST=2 (k_persist_twoloop, the north
star's persistent two-loop) runs the two-loop passes in one launch with the commit after it. (The
whole iteration in one launch, LBFGS_PERSIST=1, lost its A/B at every size and is compiled only into
variant builds, -DLBK_PERSIST_ITER=1.) One resident grid walks every
canonical segment of every pass, with the stage 2 of each pass in the launch. Same per-segment
arithmetic, same group trees, same fixed-order totals: their trajectories must be the launch
sequence's bit for bit (and so the canonical oracle's)."""
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
    assert np.array_equal(np.isnan(ta), np.isnan(tb)) and np.array_equal(ta[~np.isnan(ta)], tb[~np.isnan(tb)])
    assert np.array_equal(a["tr_c1"], b["tr_c1"]) and np.array_equal(a["tr_c2"], b["tr_c2"])
    assert a["messages"] == b["messages"] and a["status"] == b["status"] and a["iterations"] == b["iterations"]


@pytest.mark.parametrize("mode", ["2"])
@pytest.mark.parametrize("n,m,obj,ls,iters", [
    (3_000_000, 10, "rosenbrock", "backtracking", 16),     # 5860 segments of 512: tail group, 8 per workgroup
    (10_000_003, 10, "rosenbrock", "backtracking", 14),    # L = 1280, a short last segment
    (2_500_000, 7, "quad_tridiag", "wolfe", 12),           # rejected first trials: trial passes + recommits
    (1_200_000, 5, "rosenbrock", "interpolation", 20),     # 2048-element segments (mid-n rule)
])
def test_persistent_iteration_bit_exact(monkeypatch, mode, n, m, obj, ls, iters):
    x0 = L.x0_uniform(n, 5, -2.0, 2.0)
    with L.Context(n, m) as c:
        ref = c.minimize(obj, x0, ls, iters, trace=True)
    monkeypatch.setenv("LBFGS_PERSIST", mode)
    with L.Context(n, m) as c:
        c.prof_reset()
        c.prof_enable(True)
        got = c.minimize(obj, x0, ls, iters, trace=True)
        c.prof_enable(False)
        launches = c.prof_get("small_iter")["launches"]
    same(got, ref)
    assert launches >= 1  # the persistent kernel ran (one launch per iteration with h >= 1)


@pytest.mark.parametrize("mode", ["2"])
def test_persistent_iteration_vs_oracle(mode):
    """n = 3e6 through the persistent kernel against the canonical oracle itself (10 iterations)."""
    n, m, iters = 3_000_000, 10, 10
    os.environ["LBFGS_PERSIST"] = mode
    try:
        x0 = L.x0_uniform(n, 42, -2.0, 2.0)
        with L.Context(n, m) as c:
            r = c.minimize("rosenbrock", x0, "backtracking", iters, trace=True)
    finally:
        del os.environ["LBFGS_PERSIST"]
    o = O.lbfgs("rosenbrock", O.x0_uniform(n, 42, -2.0, 2.0), "backtracking", m, iters, 1e-5, mode=O.CANON)
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"])) and np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
