"""The device-resident line searches at small n: once a search
needs a trial pass beyond the commit's first one, the rest of it - backtracking, interpolation,
Wolfe or backtracking-Wolfe (sequential-implementation/line_search.cpp:19-30, 57-121, 125-189,
33-55) - and the commit at the step it finds run in ONE cooperative launch (k_coop_search).

Against the host loop (LBFGS_DEV_SEARCH=0) every case must give the same trajectory bit for bit
AND the same trial and commit counters (trial passes with f only, with f and g.d, commits): the
launch restates the host's caches, so it evaluates exactly the trial passes the host loop would.
The one pass it may add is d's materialisation (the host loop forms d on the fly for an
iteration's first two trial passes and its commit; the launch reads it from the buffer): at most
one per launch. Against the oracle's canonical restatement the trajectory is bit-exact.
lbfgs_search_stats shows the device form actually ran, and that its launches took the recommit."""
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


def solve(monkeypatch, dev, n, m, obj, ls, iters, seed, tol=1e-5):
    for k in ("LBFGS_DEV_SEARCH", "LBFGS_DEV_WOLFE", "LBFGS_SEARCH_TIMEOUT", "LBFGS_COOP", "LBFGS_SPEC"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("LBFGS_DEV_SEARCH", "1" if dev else "0")
    x0 = L.x0_uniform(n, seed, -2.0, 2.0)
    with L.Context(n, m) as c:
        r = c.minimize(obj, x0, ls, iters, tolerance=tol, trace=True)
        r["search"] = c.search_stats()
    return x0, r


def assert_same(a, b):
    for key in ("tr_f", "tr_gnorm", "x"):
        assert np.array_equal(bits(a[key]), bits(b[key])), key
    ta, tb = a["tr_alpha"], b["tr_alpha"]
    assert np.array_equal(np.isnan(ta), np.isnan(tb)) and np.array_equal(ta[~np.isnan(ta)], tb[~np.isnan(tb)])
    assert np.array_equal(a["tr_c1"], b["tr_c1"]) and np.array_equal(a["tr_c2"], b["tr_c2"])
    assert a["messages"] == b["messages"] and a["status"] == b["status"] and a["iterations"] == b["iterations"]


CASES = [  # n, m, objective, line search, iterations, seed
    (10_000, 5, "rosenbrock", "backtracking", 300, 42),       # 20 segments
    (10_000, 5, "rosenbrock", "interpolation", 300, 42),
    (10_000, 5, "rosenbrock", "wolfe", 300, 42),
    (10_000, 5, "rosenbrock", "backtracking_wolfe", 300, 42),
    (100_003, 10, "rosenbrock", "interpolation", 120, 7),     # 196 segments of 512
    (100_003, 10, "rosenbrock", "backtracking_wolfe", 120, 7),
    (300_001, 8, "quad_tridiag", "interpolation", 80, 3),     # 147 segments of 2048 (mid-n length)
    (300_001, 8, "quad_tridiag", "backtracking_wolfe", 80, 3),
    (30_001, 3, "quad_sep", "backtracking", 200, 11),         # (quad_sep: the device form may not be needed)
    (30_001, 3, "quad_sep", "interpolation", 200, 11),
    (30_001, 3, "quad_sep", "backtracking_wolfe", 200, 11),
    (257, 2, "rosenbrock", "backtracking_wolfe", 400, 5),     # one segment, partly filled
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c[0]}_m{c[1]}_{c[2]}_{c[3]}")
def test_device_search_matches_host_loop_and_oracle(monkeypatch, case):
    n, m, obj, ls, iters, seed = case
    x0, host = solve(monkeypatch, False, n, m, obj, ls, iters, seed)
    _, dev = solve(monkeypatch, True, n, m, obj, ls, iters, seed)
    assert host["search"] == (0, 0)
    launches, commits = dev["search"]
    if obj != "quad_sep":  # its first steps are accepted: no search beyond the commit's first trial
        assert launches > 0, "the device form never ran"
        assert 0 < commits <= launches
    assert commits <= launches
    assert_same(host, dev)
    for k in ("trials_f", "trials_fg", "commits"):
        assert host[k] == dev[k], (k, host[k], dev[k])
    assert 0 <= dev["passes"] - host["passes"] <= launches, (host["passes"], dev["passes"], launches)
    with np.errstate(all="ignore"):
        o = O.lbfgs(obj, x0, ls, m, iters, 1e-5, mode=O.CANON)
    assert np.array_equal(bits(dev["tr_f"]), bits(o["f"])) and np.array_equal(bits(dev["x"]), bits(o["x"]))
    assert dev["messages"] == o["messages"] and dev["iterations"] == o["iters"]


def test_standalone_line_search_on_the_device(monkeypatch):
    """lbfgs_line_search (the reference's free functions, line_search.cpp) along -g from a random
    point, where the first steps are rejected: the device form (no commit here) gives the host
    loop's step for all four searches"""
    n = 50_000
    x = L.x0_uniform(n, 17, -2.0, 2.0)
    for ls in ("backtracking", "interpolation", "wolfe", "backtracking_wolfe"):
        steps = []
        for dev in (False, True):
            monkeypatch.setenv("LBFGS_DEV_SEARCH", "1" if dev else "0")
            with L.Context(n, 5) as c:
                g = c.objective("rosenbrock", x)[1]
                steps.append(c.line_search("rosenbrock", ls, x, -g, g))
        assert np.array_equal(bits([steps[0]]), bits([steps[1]])), (ls, steps)
