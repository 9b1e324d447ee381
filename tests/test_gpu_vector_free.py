"""Vector-free mode (LBFGS_FLAG_VECTOR_FREE): the two-loop recursion over the Gram matrix of
the basis {s_i, y_i, g} on the host, one fused device pass per iteration (direction formed on
the fly from the basis, first trial, commit, new Gram rows).

  * bit-exact against the oracle's restatement of the same algorithm in the canonical order
    (oracle/lbfgs_oracle.c orc_lbfgs_vf): f, |g|, alpha, x checksums, final x, messages;
  * against the reference's own sequential runs: f and |g| within 1e-10 relative for the first
    K_f / K_g iterations and the same outcome — the same contract as the default mode, with
    horizons measured per case (they match the canonical order's to within a few iterations).
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

# (K_f, K_g) of the vector-free order against the reference (measured with the oracle)
HORIZON_VF = {"qsep_main": (2, 2), "qtri_n1e4_m10_bt": (10, 10), "qtri_n1e4_m20_wolfe": (2, 3),
              "qtri_n1e5_m20_wolfe": (2, 3), "rosen_n100_m5_bt": (47, 39), "rosen_n1_bt": (1, 1),
              "rosen_n1e3_m10_bt_conv": (49, 35), "rosen_n1e4_m5_bt": (67, 45),
              "rosen_n1e4_m5_btw": (68, 45), "rosen_n1e4_m5_interp": (67, 45),
              "rosen_n1e4_m5_wolfe": (28, 15), "rosen_n1e5_m10_bt": (61, 25),
              "rosen_n2_m3_bt": (30, 31), "rosen_n3_m1_wolfe": (8, 8),
              "rosen_n4097_m7_interp": (70, 44)}


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def run_gpu(meta):
    x0 = L.x0_uniform(meta["n"], meta["seed"], meta["lo"], meta["hi"])
    with L.Context(meta["n"], meta["m"]) as c:
        return c.minimize(meta["objective"], x0, meta["method"], meta["maxit"], tolerance=meta["tol"],
                          trace=True, vector_free=True)


def run_oracle(meta):
    x0 = O.x0_uniform(meta["n"], meta["seed"], meta["lo"], meta["hi"])
    return O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"],
                   mode=O.CANON, vector_free=True)


@pytest.mark.parametrize("name", sorted(HORIZON_VF))
def test_vector_free_bit_exact_vs_oracle(name):
    meta, _ = O.load_golden(name)
    r = run_gpu(meta)
    o = run_oracle(meta)
    assert r["status"] == o["status"] and r["iterations"] == o["iters"]
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
    a1, a2 = r["tr_alpha"], o["alpha"]
    assert np.array_equal(np.isnan(a1), np.isnan(a2))
    assert np.array_equal(a1[~np.isnan(a1)], a2[~np.isnan(a2)])
    assert np.array_equal(r["tr_c1"], o["c1"]) and np.array_equal(r["tr_c2"], o["c2"])
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
    assert r["messages"] == o["messages"]


@pytest.mark.parametrize("name", sorted(HORIZON_VF))
def test_vector_free_vs_reference_golden(name):
    meta, g = O.load_golden(name)
    r = run_gpu(meta)
    Kf, Kg = HORIZON_VF[name]
    x0 = O.x0_uniform(meta["n"], meta["seed"], meta["lo"], meta["hi"])
    s = O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"], mode=O.SEQ)
    ref_f, ref_g = s["f"], s["gnorm"]
    rel_f = np.abs(r["tr_f"][:Kf] - ref_f[:Kf]) / np.maximum(np.abs(ref_f[:Kf]), 1e-300)
    rel_g = np.abs(r["tr_gnorm"][:Kg] - ref_g[:Kg]) / np.maximum(np.abs(ref_g[:Kg]), 1e-300)
    assert np.all(rel_f <= 1e-10) and np.all(rel_g <= 1e-10)
    final = meta["stdout"].strip().splitlines()[-1]
    assert r["messages"].strip().splitlines()[-1] == final


def test_vector_free_at_scale_bit_exact():
    """n = 3e6 + 1 (odd, 8192 segments minus a partial one), m = 10, 14 iterations (h reaches
    the bucket 10 kernel), every line search kind's rejected-first-trial path via Wolfe"""
    n, m = 3_000_001, 10
    x0 = L.x0_uniform(n, 11, -2.0, 2.0)
    for ls in ("backtracking", "wolfe"):
        with L.Context(n, m) as c:
            r = c.minimize("rosenbrock", x0, ls, 14, trace=True, vector_free=True)
        o = O.lbfgs("rosenbrock", x0, ls, m, 14, 1e-5, mode=O.CANON, vector_free=True)
        assert np.array_equal(bits(r["tr_f"]), bits(o["f"])), ls
        assert np.array_equal(bits(r["x"]), bits(o["x"])), ls


def test_vector_free_nontemporal_bit_exact(monkeypatch):
    meta, _ = O.load_golden("rosen_n1e4_m5_interp")
    monkeypatch.setenv("LBFGS_NT", "1")
    r = run_gpu(meta)
    monkeypatch.delenv("LBFGS_NT")
    o = run_oracle(meta)
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))


def test_vector_free_rejects_unsupported():
    with L.Context(100, 3) as c:  # host callbacks, unfused + vector-free, m > 20
        with pytest.raises(L.LbfgsError):
            c.minimize("host", np.zeros(100), "backtracking", 5, f=lambda x: 0.0, grad=lambda x: x,
                       vector_free=True)
        with pytest.raises(L.LbfgsError):
            c.minimize("rosenbrock", np.zeros(100), "backtracking", 5, vector_free=True, unfused=True)
    with L.Context(100, 21) as c:
        with pytest.raises(L.LbfgsError):
            c.minimize("rosenbrock", np.zeros(100), "backtracking", 5, vector_free=True)


@pytest.mark.parametrize("ticket", ["0", "1"])
@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("obj,ls", [("rosenbrock", "backtracking"), ("rosenbrock", "wolfe"),
                                    ("quad_tridiag", "wolfe")])
def test_vector_free_sharded_emulated_bit_exact(world, obj, ls, ticket, monkeypatch):
    """Sharded vector-free mode (one wide all-gather per commit carrying the reductions and the
    ranks' edge values of x, g, s, y into the neighbours' ghost cells) with `world` emulated
    ranks on this GPU gives the single-GPU trajectory bit for bit."""
    import threading

    n = 4_000_003
    m, iters = 5, 12
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    with L.Context(n, m) as c:
        ref = c.minimize(obj, x0, ls, iters, trace=True, vector_free=True)
    monkeypatch.setenv("LBFGS_TICKET", ticket)
    grp = L.HostGroup(world)
    ctxs = [L.Context(n, m, rank=r, group=grp) for r in range(world)]
    out = [None] * world
    err = [None] * world

    def run(r):
        try:
            out[r] = ctxs[r].minimize(obj, x0, ls, iters, trace=True, vector_free=True)
        except Exception as e:  # pragma: no cover
            err[r] = e

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not any(err), err
    x = np.zeros(n)
    for r in range(world):
        o = out[r]
        for key in ["tr_f", "tr_gnorm", "tr_alpha"]:
            assert np.array_equal(bits(o[key]), bits(ref[key])), (r, key)
        assert np.array_equal(o["tr_c1"], ref["tr_c1"]) and np.array_equal(o["tr_c2"], ref["tr_c2"])
        lo, nl = ctxs[r].elem_lo, ctxs[r].n_loc
        x[lo:lo + nl] = o["x"][lo:lo + nl]
    assert np.array_equal(bits(x), bits(ref["x"]))
    for c in ctxs:
        c.close()
    grp.close()


@pytest.mark.parametrize("m,ls", [(20, "backtracking"), (14, "wolfe"), (16, "interpolation")])
def test_vector_free_large_history_buckets(m, ls):
    """h grows to m over the run, so every register bucket up to 20 (12, 16, 20: the
    AGPR-spilling instantiations) is exercised; bit-exact vs the oracle's restatement."""
    n, iters = 50_001, m + 8
    x0 = L.x0_uniform(n, 5, -2.0, 2.0)
    with L.Context(n, m) as c:
        r = c.minimize("rosenbrock", x0, ls, iters, trace=True, vector_free=True)
    o = O.lbfgs("rosenbrock", x0, ls, m, iters, 1e-5, mode=O.CANON, vector_free=True)
    assert r["iterations"] == o["iters"] == iters
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
    assert "Skipping" not in o["messages"]  # the history really reaches h = m


@pytest.mark.parametrize("ticket", [None, "0", "1"])
@pytest.mark.parametrize("n", [65_535, 65_536, 131_073, 262_143, 262_144])
def test_vector_free_geometry_edges_bit_exact(monkeypatch, n, ticket):
    """The edges of the mid-n segment rules (ORC_MIDL_LO = 65536: canonical segments grow to 2048
    while the vector-free commit keeps 512; ORC_VFL_LO = 262144: the vector-free base length
    follows the canonical one; just over 131072 the canonical grid drops under the ticket
    threshold and the vector-free grid does not), under both stage-2 forms and the default
    choice: bit-exact against the oracle's ORC_CANON_VF restatement."""
    if ticket is not None:
        monkeypatch.setenv("LBFGS_TICKET", ticket)
    x0 = L.x0_uniform(n, 9, -2.0, 2.0)
    with L.Context(n, 8) as c:
        r = c.minimize("rosenbrock", x0, "backtracking", 25, trace=True, vector_free=True)
    o = O.lbfgs("rosenbrock", x0, "backtracking", 8, 25, 1e-5, mode=O.CANON, vector_free=True)
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
    assert np.array_equal(r["tr_c1"], o["c1"]) and np.array_equal(r["tr_c2"], o["c2"])
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
