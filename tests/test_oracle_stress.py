"""The reference's guard paths (lbfgs.cpp:102-124 invalid rho / gamma, :148-153 non-descent,
:164-168 line-search failure, :192-195 skipped updates), pinned by goldens the reference itself
produced on stress objectives (tests/golden/stress_*, oracle/ref_driver.cpp): the oracle in the
reference's order, driven by the same objectives as host callables, reproduces every f value the
reference computed, every grad call's point and |g|, and the whole stdout."""
import numpy as np
import pytest

import oracle_lib as O


@pytest.mark.parametrize("name", O.stress_cases())
def test_oracle_reproduces_reference_guard_paths(name):
    meta, g = O.load_golden(name)
    x0 = O.x0_uniform(meta["n"], meta["seed"], meta["lo"], meta["hi"])
    with np.errstate(all="ignore"):
        if meta["objective"] in O.OBJ:  # a benchmark objective at a stress scale
            o = O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"], mode=O.SEQ,
                        log_calls=True)
        else:
            f, grad = O.stress_objective(meta["objective"])
            o = O.lbfgs("host", x0, meta["method"], meta["m"], meta["maxit"], meta["tol"], mode=O.SEQ, f=f,
                        grad=grad, log_calls=True)
    assert np.array_equal(o["flog"].view(np.uint64), g["f_calls"].view(np.uint64))
    assert np.array_equal(o["glog"][:, :2], g["grad_c"])
    assert np.array_equal(o["glog"][:, 2].view(np.float64).view(np.uint64), g["grad_norm"].view(np.uint64))
    assert o["messages"] == meta["stdout"]


def test_every_guard_message_is_pinned():
    out = "".join(O.load_golden(n)[0]["stdout"] for n in O.stress_cases())
    for msg in ("Warning: Invalid rho at iteration", "Warning: Invalid gamma at iteration",
                "Warning: Not a descent direction, using gradient", "Warning: Line search failed at iteration",
                "Warning: Skipping update, sy ="):
        assert msg in out, msg
