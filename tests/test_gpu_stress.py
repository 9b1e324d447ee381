"""The reference's guard paths on the GPU (SURVEY §5 failure detection: "same guards, with
identical messages"): invalid rho / gamma (lbfgs.cpp:102-124), non-descent direction (:148-153),
line-search failure (:164-168), skipped updates (:192-195). The stress objectives
(tests/golden/stress_*, produced by the reference itself through oracle/ref_driver.cpp) run as
host callbacks through the device path:
  * the whole stdout equals the reference's, message for message;
  * in the reference call order, as many f and grad calls as the reference made;
  * the trajectory is the canonical oracle's bit for bit.
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


@pytest.mark.parametrize("refcalls", [False, True])
@pytest.mark.parametrize("name", O.stress_cases())
def test_guard_paths_match_reference(name, refcalls):
    meta, g = O.load_golden(name)
    n = meta["n"]
    x0 = O.x0_uniform(n, meta["seed"], meta["lo"], meta["hi"])
    device = meta["objective"] in L.OBJECTIVES  # a benchmark objective: the fused device path
    if device and refcalls:
        pytest.skip("device objective: no callbacks")
    with np.errstate(all="ignore"):
        if device:
            o = O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"], mode=O.CANON)
            with L.Context(n, meta["m"]) as c:
                r = c.minimize(meta["objective"], x0, meta["method"], meta["maxit"], tolerance=meta["tol"], trace=True)
        else:
            f, grad = O.stress_objective(meta["objective"])
            o = O.lbfgs("host", x0, meta["method"], meta["m"], meta["maxit"], meta["tol"], mode=O.CANON, f=f,
                        grad=grad)
            with L.Context(n, meta["m"]) as c:
                r = c.minimize("host", x0, meta["method"], meta["maxit"], tolerance=meta["tol"], f=f, grad=grad,
                               trace=True, reference_calls=refcalls)
    assert r["messages"] == meta["stdout"]  # the reference's own output
    assert r["messages"] == o["messages"] and r["status"] == o["status"] and r["iterations"] == o["iters"]
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(r["tr_c1"], o["c1"]) and np.array_equal(r["tr_c2"], o["c2"])
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
    if refcalls:
        assert r["f_calls"] == len(g["f_calls"]) and r["grad_calls"] == len(g["grad_c"])
    if device:  # the unfused launch structure and one trial pass per step reach the same guards
        for kw, env in ((dict(unfused=True), None), ({}, "0")):
            if env is not None:
                os.environ["LBFGS_BATCH"] = env
            try:
                with np.errstate(all="ignore"), L.Context(n, meta["m"]) as c:
                    r2 = c.minimize(meta["objective"], x0, meta["method"], meta["maxit"], tolerance=meta["tol"],
                                    trace=True, **kw)
            finally:
                os.environ.pop("LBFGS_BATCH", None)
            assert r2["messages"] == meta["stdout"]
            assert np.array_equal(bits(r2["tr_f"]), bits(o["f"])) and np.array_equal(bits(r2["x"]), bits(o["x"]))
