"""Pin the oracle (our C restatement) against traces of the REFERENCE itself.

Fixtures in tests/golden/ were produced by tests/golden/make_golden.py from oracle/_ref/ref_lbfgs,
i.e. the reference's own sequential-implementation sources. In ORC_SEQ mode the oracle must
reproduce every objective call the reference makes, bit for bit: the f-call value sequence,
the checksum of every x passed to grad(), |grad|, the returned x and the printed messages.
"""
import numpy as np
import pytest

import oracle_lib as O


@pytest.mark.parametrize("name", ["kat_n1000", "kat_n5"])
def test_kat_objectives_bit_exact(name):
    meta, g = O.load_golden(name)
    x = g["x"]
    # x0 generator == std::mt19937 + uniform_real_distribution (benchmark driver uses it too)
    assert np.array_equal(O.x0_uniform(meta["n"], meta["seed"], -2.0, 2.0), x)
    assert O.f("rosenbrock", x, O.SEQ) == g["f_rosen"][0]
    assert O.f("quad_tridiag", x, O.SEQ) == g["f_qtri"][0]
    assert O.f("quad_sep", x, O.SEQ) == g["f_qsep"][0]
    assert np.array_equal(O.grad("rosenbrock", x).view(np.uint64), g["g_rosen"].view(np.uint64))
    assert np.array_equal(O.grad("quad_tridiag", x).view(np.uint64), g["g_qtri"].view(np.uint64))
    assert np.array_equal(O.grad("quad_sep", x).view(np.uint64), g["g_qsep"].view(np.uint64))


def test_checksum_matches_numpy():
    x = O.x0_uniform(777, 5, -3.0, 1.0)
    assert O.checksum(x) == O.np_checksum(x)


@pytest.mark.parametrize("name", O.golden_cases())
def test_oracle_reproduces_reference_trace(name):
    meta, g = O.load_golden(name)
    n = meta["n"]
    x0 = O.x0_uniform(n, meta["seed"], meta["lo"], meta["hi"])
    if g["x_full"].shape[0] > 0:
        assert np.array_equal(g["x_full"][0], x0)
    r = O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"],
                mode=O.SEQ, log_calls=True)
    # every f() value, in call order
    ref_f = g["f_calls"]
    assert len(r["flog"]) == len(ref_f)
    assert np.array_equal(r["flog"].view(np.uint64), ref_f.view(np.uint64))
    # every grad() argument (checksums) and |grad| (bits)
    ref_gc, ref_gn = g["grad_c"], g["grad_norm"]
    assert r["glog"].shape[0] == ref_gc.shape[0]
    assert np.array_equal(r["glog"][:, 0:2], ref_gc)
    assert np.array_equal(r["glog"][:, 2], ref_gn.view(np.uint64))
    # returned x
    assert O.checksum(r["x"]) == tuple(int(v) for v in g["ret_c"])
    if "ret_x" in g:
        assert np.array_equal(r["x"], g["ret_x"])
    # messages (the reference's non-verbose stdout)
    assert r["messages"] == meta["stdout"]
