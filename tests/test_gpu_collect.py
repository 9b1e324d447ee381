"""Collect-mode stage 2 (LBFGS_COLLECT=1): every workgroup stores its segment
partials as flagged words and each group's last-dispatched workgroup forms the group's canonical
tree inside the producing launch, instead of a k_group_reduce launch after it. Same partials, same
tree shapes, same bits: trajectories must equal the default's bit for bit, over one-component
passes, the 8-component commit and the trial passes (wide slots - the vector-free commit - keep the
reduce kernel). Default on for segments of >= 3072 elements (n >= 2.5e7 on one GPU)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def solve(monkeypatch, collect, n, m, obj, ls, iters, vf, rev="1"):
    monkeypatch.setenv("LBFGS_COLLECT", collect)
    monkeypatch.setenv("LBFGS_REV", rev)
    x0 = L.x0_uniform(n, 11, -2.0, 2.0)
    with L.Context(n, m) as c:
        c.prof_reset()
        c.prof_enable(True)
        r = c.minimize(obj, x0, ls, iters, trace=True, vector_free=vf)
        c.prof_enable(False)
        r["reduce_launches"] = c.prof_get("group_reduce")["launches"]
    return r


@pytest.mark.parametrize("n,m,obj,ls,iters,vf,rev", [
    (2_500_000, 10, "rosenbrock", "backtracking", 14, False, "1"),    # 4883 segments, tail group of 787
    (3_000_017, 5, "quad_tridiag", "wolfe", 12, False, "1"),          # trial passes, f + g.d
    (5_000_000, 7, "rosenbrock", "interpolation", 12, False, "0"),    # forward walk only
    (2_361_601, 5, "rosenbrock", "backtracking", 10, False, "1"),     # tail group of 7 segments (short tree), last of 1 element
    (3_000_017, 10, "rosenbrock", "backtracking", 12, True, "1"),     # vector-free: wide slots
    (10_000_003, 5, "quad_sep", "backtracking_wolfe", 8, True, "1"),
])
def test_collect_bit_identical(monkeypatch, n, m, obj, ls, iters, vf, rev):
    a = solve(monkeypatch, "0", n, m, obj, ls, iters, vf, rev)
    b = solve(monkeypatch, "1", n, m, obj, ls, iters, vf, rev)
    for key in ("tr_f", "tr_gnorm", "x"):
        assert np.array_equal(bits(a[key]), bits(b[key])), key
    ta, tb = a["tr_alpha"], b["tr_alpha"]
    assert np.array_equal(np.isnan(ta), np.isnan(tb)) and np.array_equal(ta[~np.isnan(ta)], tb[~np.isnan(tb)])
    assert a["messages"] == b["messages"] and a["status"] == b["status"] and a["iterations"] == b["iterations"]
    if vf:  # the wide slots keep their reduce launches
        assert b["reduce_launches"] <= a["reduce_launches"]
    else:  # every stage 2 ran inside the passes
        assert a["reduce_launches"] > 0 and b["reduce_launches"] == 0
