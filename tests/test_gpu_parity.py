"""GPU parity tests: the HIP path (through the C ABI) against the oracle.

Contract:
  * elementwise results (gradients, trial gradients, two-loop direction) are BIT-EXACT
    against the reference formulas;
  * every reduction is BIT-EXACT against the oracle's canonical-order restatement, so whole
    L-BFGS trajectories are bit-exact (f, |g|, alpha and the x checksum at every iteration);
  * against the reference's own sequential traces (tests/golden) the trajectory agrees within
    1e-10 relative in f for the first K iterations, K = the measured horizon of the canonical
    order (no parallel reduction order can reproduce a left-to-right sum), and ends in the
    same outcome.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402
import oracle_lib as O  # noqa: E402

pytestmark = pytest.mark.gpu

OBJS = ["rosenbrock", "quad_tridiag", "quad_sep"]
_ctx = {}


def ctx(n, m=5):
    key = (n, m)
    if key not in _ctx:
        if len(_ctx) > 6:
            for k in list(_ctx):
                _ctx.pop(k).close()
        _ctx[key] = L.Context(n, m)
    return _ctx[key]


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


SIZES = [1, 2, 3, 5, 127, 128, 129, 255, 511, 512, 513, 4095, 4097, 10000, 65537, 524289,
         3_000_017]


@pytest.mark.parametrize("n", SIZES)
def test_dot_bit_exact_canonical(n):
    rs = np.random.RandomState(n)
    a = rs.uniform(-3, 3, n)
    b = rs.uniform(-3, 3, n)
    got = ctx(n).dot(a, b)
    want = O.dot(a, b, O.CANON)
    assert bits([got])[0] == bits([want])[0], (got, want)
    # and numerically close to an exact-ish reference
    ref = float(np.dot(a.astype(np.longdouble), b.astype(np.longdouble)))
    assert abs(got - ref) <= 2 * n * np.finfo(float).eps * np.sum(np.abs(a * b)) + 1e-300


@pytest.mark.parametrize("obj", OBJS)
@pytest.mark.parametrize("n", [1, 2, 3, 129, 513, 4097, 100_003, 1_048_577])
def test_objective_bit_exact(obj, n):
    x = np.random.RandomState(n + 1).uniform(-2, 2, n)
    f, g = ctx(n).objective(obj, x)
    assert np.array_equal(bits(g), bits(O.grad(obj, x)))
    assert bits([f])[0] == bits([O.f(obj, x, O.CANON)])[0]


@pytest.mark.parametrize("name", ["kat_n1000", "kat_n5"])
def test_objective_vs_reference_kat(name):
    """Gradients bit-exact against the reference's own functions; f within the sum-order bound."""
    meta, g = O.load_golden(name)
    x = g["x"]
    for obj, gk, fk in [("rosenbrock", "g_rosen", "f_rosen"), ("quad_tridiag", "g_qtri", "f_qtri"),
                        ("quad_sep", "g_qsep", "f_qsep")]:
        f, gr = ctx(len(x)).objective(obj, x)
        assert np.array_equal(bits(gr), bits(g[gk]))
        assert abs(f - g[fk][0]) <= 1e-13 * abs(g[fk][0])


@pytest.mark.parametrize("obj", OBJS)
@pytest.mark.parametrize("n", [2, 129, 4097, 200_001])
def test_trial_bit_exact(obj, n):
    rs = np.random.RandomState(7 * n)
    x = rs.uniform(-2, 2, n)
    d = rs.uniform(-1, 1, n)
    alpha = 0.37
    f, gt, dphi = ctx(n).trial(obj, x, d, alpha)
    xt = x + alpha * d  # add(x, scalarProduct(alpha, d)) rounding
    assert bits([f])[0] == bits([O.f(obj, xt, O.CANON)])[0]
    gref = O.grad(obj, xt)
    assert np.array_equal(bits(gt), bits(gref))
    assert bits([dphi])[0] == bits([O.dot(gref, d, O.CANON)])[0]


@pytest.mark.parametrize("h", [1, 2, 5])
@pytest.mark.parametrize("n", [3, 1000, 70_001])
def test_twoloop_bit_exact(h, n):
    rs = np.random.RandomState(100 * h + n)
    g = rs.uniform(-1, 1, n)
    S = [rs.uniform(-1, 1, n) for _ in range(h)]
    Y = [s * rs.uniform(0.5, 2.0, n) + 0.01 * rs.uniform(-1, 1, n) for s in S]  # s.y > 0
    d, gd = ctx(n, 5).twoloop(g, S, Y)
    dref, gdref = O.twoloop(g, S, Y, O.CANON)
    assert np.array_equal(bits(d), bits(dref))
    assert bits([gd])[0] == bits([gdref])[0]


@pytest.mark.parametrize("k", [10, 30, 60])
def test_one_step_from_reference_state(k):
    """SURVEY 8c parity item 3: one L-BFGS step from the reference's own state. The sequential
    oracle (bit-exact with the reference, tests/test_oracle_golden.py) gives x_j for
    j = k-m .. k+1 of Rosenbrock n=1e4, m=5, backtracking, hence g_j, s_j, y_j exactly as the
    reference holds them; the device two-loop from (g_k, s, y) with the reference's accepted
    step gives x_{k+1} within 1e-12 relative (norm-wise; elementwise is meaningless for
    components near 0) of the reference's x_{k+1}, and the step itself within 1e-12. Measured
    on CPU with the canonical restatement: 6e-16 and 6e-15."""
    n, m = 10_000, 5
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    xs = {j: O.lbfgs("rosenbrock", x0, "backtracking", m, j, 1e-5, mode=O.SEQ)["x"]
          for j in range(k - m, k + 2)}
    run = O.lbfgs("rosenbrock", x0, "backtracking", m, k + 1, 1e-5, mode=O.SEQ)
    assert "Skipping" not in run["messages"]  # the ring holds the last m pairs
    gs = {j: O.grad("rosenbrock", xs[j]) for j in xs}
    S = [xs[j + 1] - xs[j] for j in range(k - m, k)]
    Y = [gs[j + 1] - gs[j] for j in range(k - m, k)]
    d, _ = ctx(n, m).twoloop(gs[k], S, Y)
    alpha = run["alpha"][k]
    x1 = xs[k] + alpha * d
    assert np.linalg.norm(x1 - xs[k + 1]) <= 1e-12 * np.linalg.norm(xs[k + 1])
    step = xs[k + 1] - xs[k]
    assert np.linalg.norm(alpha * d - step) <= 1e-12 * np.linalg.norm(step)


def _run_gpu(meta):
    n = meta["n"]
    x0 = L.x0_uniform(n, meta["seed"], meta["lo"], meta["hi"])
    c = ctx(n, meta["m"])
    return c.minimize(meta["objective"], x0, meta["method"], meta["maxit"],
                      tolerance=meta["tol"], trace=True)


@pytest.mark.parametrize("name", O.golden_cases())
def test_trajectory_bit_exact_vs_canonical_oracle(name):
    meta, _ = O.load_golden(name)
    r = _run_gpu(meta)
    x0 = O.x0_uniform(meta["n"], meta["seed"], meta["lo"], meta["hi"])
    o = O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"],
                mode=O.CANON)
    assert r["status"] == o["status"]
    assert r["iterations"] == o["iters"]
    assert len(r["tr_f"]) == len(o["f"])
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
    a1, a2 = r["tr_alpha"], o["alpha"]
    assert np.array_equal(np.isnan(a1), np.isnan(a2))
    assert np.array_equal(a1[~np.isnan(a1)], a2[~np.isnan(a2)])
    assert np.array_equal(r["tr_c1"], o["c1"]) and np.array_equal(r["tr_c2"], o["c2"])
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
    assert r["messages"] == o["messages"]


# Measured horizons (K_f, K_g) of the canonical order against the reference: the first
# iterations for which f and |g| agree within 1e-10 relative. The GPU is
# bit-exact with the canonical oracle, so these are its horizons. No parallel reduction order
# can extend them much: they are set by the reference's own left-to-right rounding.
HORIZON = {"qsep_main": (2, 2), "qtri_n1e4_m10_bt": (10, 10), "qtri_n1e4_m20_wolfe": (2, 3),
           "qtri_n1e5_m20_wolfe": (2, 3), "rosen_n100_m5_bt": (47, 39), "rosen_n1_bt": (1, 1),
           "rosen_n1e3_m10_bt_conv": (49, 35), "rosen_n1e4_m5_bt": (67, 45),
           "rosen_n1e4_m5_btw": (68, 45), "rosen_n1e4_m5_interp": (67, 45),
           "rosen_n1e4_m5_wolfe": (28, 15), "rosen_n1e5_m10_bt": (61, 26),
           "rosen_n2_m3_bt": (24, 24), "rosen_n3_m1_wolfe": (15, 15),
           "rosen_n4097_m7_interp": (61, 38)}


HORIZONS = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "horizons.json")))


def _horizon(a, b, tol=1e-10):
    k = min(len(a), len(b))
    r = np.abs(a[:k] - b[:k]) / np.maximum(np.abs(b[:k]), 1e-300)
    bad = np.nonzero(r > tol)[0]
    return int(bad[0]) if len(bad) else int(k)


@pytest.mark.parametrize("name", O.golden_cases())
def test_trajectory_vs_reference_golden(name):
    meta, g = O.load_golden(name)
    r = _run_gpu(meta)
    Kf, Kg = HORIZON[name]
    # the reference's per-iteration f and |g|: from its own trace where one grad() call per
    # iteration makes the mapping direct, else from the sequential oracle, which reproduces
    # every reference call bit-exactly (tests/test_oracle_golden.py)
    if meta["method"] in ("backtracking", "interpolation"):
        gnf = g["grad_nf"].astype(np.int64)
        ref_f = g["f_calls"][gnf - 1]
        ref_g = g["grad_norm"]
    else:
        x0 = O.x0_uniform(meta["n"], meta["seed"], meta["lo"], meta["hi"])
        o = O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"],
                    mode=O.SEQ)
        ref_f, ref_g = o["f"], o["gnorm"]
    assert len(r["tr_f"]) >= Kf and len(ref_f) >= Kf
    rel_f = np.abs(r["tr_f"][:Kf] - ref_f[:Kf]) / np.maximum(np.abs(ref_f[:Kf]), 1e-300)
    rel_g = np.abs(r["tr_gnorm"][:Kg] - ref_g[:Kg]) / np.maximum(np.abs(ref_g[:Kg]), 1e-300)
    assert np.all(rel_f <= 1e-10), (int(np.argmax(rel_f)), float(rel_f.max()))
    assert np.all(rel_g <= 1e-10), (int(np.argmax(rel_g)), float(rel_g.max()))
    # the device run's own horizon is at least the reference's against itself under another
    # summation order (K_ref, tests/golden/horizons.json, tests/test_oracle_horizons.py)
    kf, kg = HORIZONS[name]["ref"]
    assert _horizon(r["tr_f"], ref_f) >= kf and _horizon(r["tr_gnorm"], ref_g) >= kg
    # same outcome as the reference run
    final = meta["stdout"].strip().splitlines()[-1]
    assert r["messages"].strip().splitlines()[-1] == final
    if final == "Converged!":
        assert r["gnorm"] < meta["tol"]


def test_reference_x_trajectory_small():
    """n=100: the full iterate x_k of the reference for k < 40 (its measured x horizon)
    within 1e-10 relative."""
    meta, g = O.load_golden("rosen_n100_m5_bt")
    n = meta["n"]
    c = ctx(n, meta["m"])
    x0 = L.x0_uniform(n, meta["seed"], meta["lo"], meta["hi"])
    c.init("rosenbrock", x0, "backtracking", meta["tol"])
    xs = g["x_full"]
    for k in range(0, 40):
        x = c.get_x()
        err = np.max(np.abs(x - xs[k])) / np.max(np.abs(xs[k]))
        assert err <= 1e-10, (k, err)
        c.step(1)


def test_deterministic_repeat_large():
    """n = 3e6: two runs give bit-identical trajectories (ticketed group reduction is
    placement/timing independent) and match the canonical oracle for the first iterations."""
    n = 3_000_000
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    c = ctx(n, 10)
    r1 = c.minimize("rosenbrock", x0, "backtracking", 12, trace=True)
    r2 = c.minimize("rosenbrock", x0, "backtracking", 12, trace=True)
    for key in ["tr_f", "tr_gnorm", "tr_alpha"]:
        assert np.array_equal(bits(r1[key]), bits(r2[key]))
    assert np.array_equal(r1["tr_c1"], r2["tr_c1"])
    o = O.lbfgs("rosenbrock", x0, "backtracking", 10, 12, 1e-5, mode=O.CANON)
    assert np.array_equal(bits(r1["tr_f"]), bits(o["f"]))
    assert np.array_equal(r1["tr_c1"], o["c1"]) and np.array_equal(r1["tr_c2"], o["c2"])


def test_host_callback_objective_matches_device_objective():
    """LBFGS_OBJ_HOST (user callbacks) drives the same device two-loop: with the reference's
    own formulas as callbacks, the trajectory stays within 1e-12 of the device objective."""
    n = 2000
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    c = ctx(n, 5)

    def f(x):
        return O.f("rosenbrock", x, O.CANON)

    def grad(x):
        return O.grad("rosenbrock", x)

    rh = c.minimize("host", x0, "backtracking", 30, f=f, grad=grad, trace=True)
    rd = c.minimize("rosenbrock", x0, "backtracking", 30, trace=True)
    assert np.array_equal(bits(rh["tr_f"]), bits(rd["tr_f"]))
    assert np.array_equal(rh["tr_c1"], rd["tr_c1"])


@pytest.mark.parametrize("ticket", ["0", "1"])
@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("obj,ls", [("rosenbrock", "backtracking"), ("rosenbrock", "wolfe"),
                                    ("quad_tridiag", "wolfe")])
def test_sharded_emulated_bit_exact(world, obj, ls, ticket, monkeypatch):
    """The sharded data path (group ownership, halo of d through the all-gathered slot,
    x ghosts, per-rank slices) with `world` emulated ranks on this GPU — threads with one
    stream each, exchanging through host memory exactly where RCCL all-gathers — must give
    the single-GPU trajectory bit for bit: the canonical order does not depend on the rank
    count."""
    import threading

    n = 4_000_003  # every one of 8 ranks owns segments (n > 7 * 1024 * 512)
    m, iters = 5, 12
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    ref = ctx(n, m).minimize(obj, x0, ls, iters, trace=True)
    monkeypatch.setenv("LBFGS_TICKET", ticket)  # both stage-2 forms under sharding (read at creation)
    grp = L.HostGroup(world)
    ctxs = [L.Context(n, m, rank=r, group=grp) for r in range(world)]
    out = [None] * world
    err = [None] * world

    def run(r):
        try:
            out[r] = ctxs[r].minimize(obj, x0, ls, iters, trace=True)
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
            a, b = bits(o[key]), bits(ref[key])
            assert np.array_equal(a, b), (r, key)
        assert np.array_equal(o["tr_c1"], ref["tr_c1"]) and np.array_equal(o["tr_c2"], ref["tr_c2"])
        lo, nl = ctxs[r].elem_lo, ctxs[r].n_loc
        x[lo:lo + nl] = o["x"][lo:lo + nl]
    assert np.array_equal(bits(x), bits(ref["x"]))
    for c in ctxs:
        c.close()
    grp.close()


@pytest.mark.parametrize("n,m,ls", [(10_000, 5, "backtracking"), (30_001, 16, "wolfe"), (4097, 7, "interpolation"),
                                    (20_000, 10, "backtracking_wolfe"), (32_768, 1, "backtracking"),
                                    (100_000, 10, "backtracking"), (200_001, 6, "wolfe")])
def test_cooperative_iteration_bit_exact(monkeypatch, n, m, ls):
    """The cooperative multi-workgroup iteration (LBFGS_COOP: one workgroup per segment, grid
    barriers between passes, the whole two-loop and the commit at a0 in one launch) against the
    multi-launch sequence and the oracle: identical bits."""
    x0 = L.x0_uniform(n, 3, -2.0, 2.0)
    out = []
    for coop in ("0", "512"):  # LBFGS_COOP = the largest segment count that runs cooperatively
        monkeypatch.setenv("LBFGS_COOP", coop)
        with L.Context(n, m) as c:
            out.append(c.minimize("rosenbrock", x0, ls, 60, trace=True))
    a, b = out
    assert b["passes"] < a["passes"]  # the cooperative path really ran
    for key in ("tr_f", "tr_gnorm", "x"):
        assert np.array_equal(bits(a[key]), bits(b[key])), key
    assert np.array_equal(a["tr_c1"], b["tr_c1"]) and a["messages"] == b["messages"]
    o = O.lbfgs("rosenbrock", x0, ls, m, 60, 1e-5, mode=O.CANON)
    assert np.array_equal(bits(b["tr_f"]), bits(o["f"]))


@pytest.mark.parametrize("n,m,ls,obj", [(700_001, 10, "backtracking", "rosenbrock"),
                                        (1_000_001, 5, "wolfe", "rosenbrock"),
                                        (2_000_000, 7, "interpolation", "quad_tridiag")])
def test_deferred_stage2_bit_exact(monkeypatch, n, m, ls, obj):
    """Deferred stage 2 (LBFGS_DEFER: every workgroup of the consuming pass forms the previous
    pass's total from its partials; no reduce launch between two-loop passes) against the
    reduce-kernel sequence and the oracle: identical bits."""
    x0 = L.x0_uniform(n, 5, -2.0, 2.0)
    out = []
    monkeypatch.setenv("LBFGS_TICKET", "0")  # deferral replaces the reduce kernel, not tickets
    for defer in ("0", "8192"):
        monkeypatch.setenv("LBFGS_DEFER", defer)
        with L.Context(n, m) as c:
            c.prof_reset()
            c.prof_enable(True)
            r = c.minimize(obj, x0, ls, 14, trace=True)
            r["reduce_launches"] = c.prof_get("group_reduce")["launches"]
            out.append(r)
    a, b = out
    assert b["reduce_launches"] < a["reduce_launches"]  # the deferred path really ran
    for key in ("tr_f", "tr_gnorm", "x"):
        assert np.array_equal(bits(a[key]), bits(b[key])), key
    assert np.array_equal(a["tr_c1"], b["tr_c1"]) and a["messages"] == b["messages"]
    o = O.lbfgs(obj, x0, ls, m, 14, 1e-5, mode=O.CANON)
    assert np.array_equal(bits(b["tr_f"]), bits(o["f"]))


@pytest.mark.parametrize("n,m,ls,obj,vf", [(3_000_000, 10, "backtracking", "rosenbrock", False),
                                           (5_000_000, 5, "wolfe", "quad_tridiag", False),
                                           (2_500_000, 7, "interpolation", "rosenbrock", True)])
def test_ticket_stage2_one_rank_bit_exact(monkeypatch, n, m, ls, obj, vf):
    """In-launch tickets on ONE rank over several groups (LBFGS_TICKET=1; the default only up to
    64 segments): each group's last arriver forms its tree, and the host may read a result slot
    only once every group has. Round 3 found the single completion word of the one-group case
    releasing the host after the first group here (NaN trajectories at n = 2.5e6 .. 3e7); the
    trajectories must be the reduce-kernel sequence's bit for bit."""
    x0 = L.x0_uniform(n, 11, -2.0, 2.0)
    out = []
    for ticket in ("0", "1"):
        monkeypatch.setenv("LBFGS_TICKET", ticket)
        with L.Context(n, m) as c:
            c.prof_reset()
            c.prof_enable(True)
            r = c.minimize(obj, x0, ls, 12, trace=True, vector_free=vf)
            r["reduce_launches"] = c.prof_get("group_reduce")["launches"]
            out.append(r)
    a, b = out
    assert b["reduce_launches"] < a["reduce_launches"]  # the ticket path really ran
    for key in ("tr_f", "tr_gnorm", "x"):
        assert np.array_equal(bits(a[key]), bits(b[key])), key
    assert np.array_equal(a["tr_c1"], b["tr_c1"]) and a["messages"] == b["messages"]
    assert np.all(np.isfinite(b["tr_f"]))


@pytest.mark.parametrize("vector_free", [False, True])
def test_full_run_to_convergence_bit_exact(vector_free):
    """BASELINE configs[0] to convergence (Rosenbrock n=1e4, m=5, backtracking, tol 1e-5: ~17k
    iterations through the cooperative kernel, or the vector-free commit): every f, |g|, alpha,
    the final x and the whole message stream bit-identical to the oracle's restatement."""
    n, m = 10_000, 5
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    with L.Context(n, m) as c:
        r = c.minimize("rosenbrock", x0, "backtracking", 30_000, trace=True, vector_free=vector_free)
    o = O.lbfgs("rosenbrock", x0, "backtracking", m, 30_000, 1e-5, mode=O.CANON, vector_free=vector_free)
    assert r["status"] == o["status"] == "converged" and r["iterations"] == o["iters"] > 15_000
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
    assert np.array_equal(bits(r["x"]), bits(o["x"]))
    assert r["messages"] == o["messages"]
