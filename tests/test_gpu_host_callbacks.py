"""Host-callback objectives (LBFGS_OBJ_HOST): the callback sequence.

* LBFGS_FLAG_REFERENCE_CALLS: the device path calls f and grad exactly as the reference does,
  call for call - the oracle (oracle/lbfgs_oracle.c F()/G(), which restate every f / grad call of
  lbfgs.cpp and line_search.cpp and reproduce the reference's own f_calls / grad logs bit for
  bit, tests/test_oracle_golden.py) driven by the same Python callables in the canonical order
  must log the identical sequence: the kind of each call, the checksum of the point it was
  called at and, for f, the value.
* Default: one f and at most one grad call per distinct point, the same trajectory bit for bit.
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


class Log:
    def __init__(self, obj):
        self.obj = obj
        self.calls = []

    def f(self, x):
        v = O.f(self.obj, x, O.CANON)
        self.calls.append(("f", O.np_checksum(x), float(v)))
        return v

    def grad(self, x):
        self.calls.append(("g", O.np_checksum(x), None))
        return O.grad(self.obj, x)


CASES = [("rosenbrock", 2000, 5, "backtracking", 40), ("rosenbrock", 2000, 5, "wolfe", 40),
         ("rosenbrock", 2000, 5, "interpolation", 40), ("rosenbrock", 2000, 5, "backtracking_wolfe", 25),
         ("quad_tridiag", 1000, 10, "wolfe", 30), ("rosenbrock", 3, 1, "wolfe", 60),
         ("quad_sep", 1000, 5, "backtracking", 20)]


@pytest.mark.parametrize("obj,n,m,ls,iters", CASES)
def test_reference_call_sequence(obj, n, m, ls, iters):
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    lo = Log(obj)
    o = O.lbfgs("host", x0, ls, m, iters, 1e-5, mode=O.CANON, f=lo.f, grad=lo.grad)
    lg = Log(obj)
    with L.Context(n, m) as c:
        r = c.minimize("host", x0, ls, iters, f=lg.f, grad=lg.grad, trace=True, reference_calls=True)
    assert len(lg.calls) == len(lo.calls)
    for i, (a, b) in enumerate(zip(lg.calls, lo.calls)):
        assert a[0] == b[0] and a[1] == b[1], (i, a, b)
        if a[0] == "f":
            assert bits([a[2]])[0] == bits([b[2]])[0], (i, a, b)
    assert r["f_calls"] == o["nf_total"] == sum(1 for k in lg.calls if k[0] == "f")
    assert r["grad_calls"] == o["ng_total"] == sum(1 for k in lg.calls if k[0] == "g")
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
    assert r["messages"] == o["messages"]


@pytest.mark.parametrize("obj,n,m,ls,iters", CASES)
def test_default_one_call_per_point(obj, n, m, ls, iters):
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    la, lb = Log(obj), Log(obj)
    with L.Context(n, m) as c:
        ra = c.minimize("host", x0, ls, iters, f=la.f, grad=la.grad, trace=True,
                        reference_calls=True)
        rb = c.minimize("host", x0, ls, iters, f=lb.f, grad=lb.grad, trace=True)
    for key in ("tr_f", "tr_gnorm", "x"):
        assert np.array_equal(bits(ra[key]), bits(rb[key])), key
    assert ra["messages"] == rb["messages"]
    fpts = [k[1] for k in lb.calls if k[0] == "f"]
    gpts = [k[1] for k in lb.calls if k[0] == "g"]
    assert len(fpts) == len(set(fpts)) and len(gpts) == len(set(gpts))  # no point twice
    assert set(fpts) <= {k[1] for k in la.calls if k[0] == "f"}
    assert rb["f_calls"] == len(fpts) < ra["f_calls"]
    assert rb["grad_calls"] == len(gpts) <= ra["grad_calls"]


# goldens whose canonical-order run ends the way the reference's does, with the number of leading
# f calls that agree with the reference's own f_calls log within 1e-10 (measured on the CPU with
# the oracle's canonical order, which the device path reproduces call for call above)
GOLDEN_CALLS = {"qsep_main": 5, "qtri_n1e4_m10_bt": 48, "qtri_n1e4_m20_wolfe": 24, "rosen_n2_m3_bt": 95,
                "rosen_n1_bt": 1}


@pytest.mark.parametrize("name", sorted(GOLDEN_CALLS))
def test_golden_call_counts_reference_calls(name):
    """The reference's own logs (tests/golden: every f value it computed, one row per grad call)
    against the device path in the reference call order with the reference's sequential f as the
    callable: the same number of f and grad calls, the values agreeing over the leading calls."""
    meta, g = O.load_golden(name)
    n, obj = meta["n"], meta["objective"]
    x0 = O.x0_uniform(n, meta["seed"], meta["lo"], meta["hi"])
    fv = []

    def f(x):
        v = O.f(obj, x, O.SEQ)
        fv.append(v)
        return v

    with L.Context(n, meta["m"]) as c:
        r = c.minimize("host", x0, meta["method"], meta["maxit"], f=f, grad=lambda x: O.grad(obj, x),
                       tolerance=meta["tol"], reference_calls=True)
    ref = g["f_calls"]
    assert r["f_calls"] == len(fv) == len(ref)
    assert r["grad_calls"] == len(g["grad_c"])
    k = GOLDEN_CALLS[name]
    rel = np.abs(np.array(fv[:k]) - ref[:k]) / np.maximum(np.abs(ref[:k]), 1e-300)
    assert np.all(rel <= 1e-10), (int(np.argmax(rel)), float(rel.max()))
    assert r["messages"].strip().splitlines()[-1] == meta["stdout"].strip().splitlines()[-1]
