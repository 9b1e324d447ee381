"""The cooperative forms are safe by construction.

* Each grid-barrier kernel is capped by its OWN occupancy: the device-resident line searches
  (k_coop_search) have a cap of their own (search_max), never above the cooperative iteration's, and
  a context whose cap is below the grid (LBFGS_COOP forcing it) runs the host loop instead.
* A device search whose grid barrier times out (forced here with LBFGS_SEARCH_TIMEOUT=0: every
  barrier gives up at its first miss) stored nothing, so the host loop redoes the search from the
  same state: the solve continues, bit-identical to the host loop and to the canonical oracle,
  instead of failing with "grid barrier timed out". The launch may have reached its commit pass
  (the recommit at the step it found), so the host then also repeats the first commit when its
  search ends at the first trial's step."""
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
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def solve(monkeypatch, env, n, m, obj, ls, iters, seed=3):
    for k in ("LBFGS_SEARCH_TIMEOUT", "LBFGS_DEV_WOLFE", "LBFGS_DEV_SEARCH", "LBFGS_COOP"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    x0 = L.x0_uniform(n, seed, -2.0, 2.0)
    with L.Context(n, m) as c:
        info0 = c.coop_info()
        r = c.minimize(obj, x0, ls, iters, trace=True)
        r["coop"] = c.coop_info()
        r["coop0"] = info0
    return x0, r


def same(a, b):
    for key in ("tr_f", "tr_gnorm", "tr_alpha", "x"):
        assert np.array_equal(bits(a[key]), bits(b[key])), key
    assert np.array_equal(a["tr_c1"], b["tr_c1"]) and np.array_equal(a["tr_c2"], b["tr_c2"])
    assert a["messages"] == b["messages"] and a["iterations"] == b["iterations"] and a["status"] == b["status"]


def test_grid_caps_from_each_kernels_occupancy(monkeypatch):
    _, r = solve(monkeypatch, {}, 10_000, 5, "rosenbrock", "wolfe", 3)
    cm, sm = r["coop0"]["coop_max"], r["coop0"]["search_max"]
    assert 0 < sm <= cm <= 256
    assert r["coop"]["fallbacks"] == 0


@pytest.mark.parametrize("n,m,obj,ls", [(10_000, 5, "rosenbrock", "wolfe"), (100_000, 10, "rosenbrock", "wolfe"),
                                        (30_001, 7, "rosenbrock", "wolfe"),
                                        (10_000, 5, "rosenbrock", "interpolation"),
                                        (30_001, 7, "quad_tridiag", "backtracking_wolfe"),
                                        (20_001, 3, "rosenbrock", "backtracking")])
def test_search_barrier_timeout_falls_back_bit_identical(monkeypatch, n, m, obj, ls):
    iters = 150
    x0, host = solve(monkeypatch, {"LBFGS_DEV_SEARCH": "0"}, n, m, obj, ls, iters)
    _, dev = solve(monkeypatch, {}, n, m, obj, ls, iters)
    _, forced = solve(monkeypatch, {"LBFGS_SEARCH_TIMEOUT": "0"}, n, m, obj, ls, iters)
    assert host["coop0"]["search_max"] == 0 and dev["coop0"]["search_max"] > 0
    # the forced run took the device path, timed out once, and then stayed on the host loop
    assert forced["coop"]["fallbacks"] == 1 and forced["coop"]["search_max"] == 0, forced["coop"]
    assert dev["coop"]["fallbacks"] == 0
    same(forced, host)
    same(dev, host)
    # the counters: the timed-out launch counts no trial pass and the host loop redoes the search
    # from the same state, so the trial passes are the host loop's; the redo commits again even at
    # the first trial's step (recommit_a0), at most once per solve since the device form then stays off
    for k in ("trials_f", "trials_fg"):
        assert forced[k] == host[k], (k, forced[k], host[k])
    assert host["commits"] <= forced["commits"] <= host["commits"] + 1, (forced["commits"], host["commits"])
    o = O.lbfgs(obj, x0, ls, m, iters, 1e-5, mode=O.CANON)
    assert np.array_equal(bits(forced["tr_f"]), bits(o["f"])) and np.array_equal(bits(forced["x"]), bits(o["x"]))


def test_cap_below_the_grid_takes_the_host_loop(monkeypatch):
    """LBFGS_COOP=64 puts the cooperative caps below n = 1e5's 196 segments: neither grid-barrier
    form may launch, and the trajectory is the oracle's"""
    n, m = 100_000, 10
    x0, r = solve(monkeypatch, {"LBFGS_COOP": "64"}, n, m, "rosenbrock", "wolfe", 60)
    assert r["coop0"]["coop_max"] == 64 and r["coop0"]["search_max"] <= 64
    assert r["coop"]["fallbacks"] == 0
    o = O.lbfgs("rosenbrock", x0, "wolfe", m, 60, 1e-5, mode=O.CANON)
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"])) and np.array_equal(bits(r["x"]), bits(o["x"]))
