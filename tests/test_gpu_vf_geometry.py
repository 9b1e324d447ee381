"""The vector-free commit's own segment geometry (lbk_vf_factor / orc_vf_factor): segments of
F = 1, 2, 4 or 8 canonical segments, 1024 / F of them per group, chosen from n alone. Checked
bit for bit against the oracle's restatement at sizes that select F = 2, 8 and 4, on one GPU
and sharded over emulated ranks (the ranks own the same elements in both geometries)."""
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


@pytest.mark.parametrize("n,F", [(1_500_000, 2), (4_194_304, 8), (10_000_000, 4)])
def test_vector_free_long_segments_bit_exact(n, F):
    assert O.vf_factor(n) == F
    m = 6
    x0 = L.x0_uniform(n, 7, -2.0, 2.0)
    with L.Context(n, m) as c:
        r = c.minimize("rosenbrock", x0, "backtracking", 10, trace=True, vector_free=True)
    o = O.lbfgs("rosenbrock", x0, "backtracking", m, 10, 1e-5, mode=O.CANON, vector_free=True)
    assert np.array_equal(bits(r["tr_f"]), bits(o["f"]))
    assert np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
    assert np.array_equal(bits(r["x"]), bits(o["x"]))


@pytest.mark.parametrize("ticket", ["0", "1"])
def test_vector_free_long_segments_sharded(ticket, monkeypatch):
    """F = 8 with 8 emulated ranks: each rank owns exactly one group of 128 long segments."""
    import threading

    n, m, iters, world = 4_194_304, 5, 8, 8
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    with L.Context(n, m) as c:
        ref = c.minimize("rosenbrock", x0, "backtracking", iters, trace=True, vector_free=True)
    monkeypatch.setenv("LBFGS_TICKET", ticket)
    grp = L.HostGroup(world)
    ctxs = [L.Context(n, m, rank=r, group=grp) for r in range(world)]
    out, err = [None] * world, [None] * world

    def run(r):
        try:
            out[r] = ctxs[r].minimize("rosenbrock", x0, "backtracking", iters, trace=True, vector_free=True)
        except Exception as e:  # pragma: no cover
            err[r] = e

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(err), err
    x = np.zeros(n)
    for r in range(world):
        assert np.array_equal(bits(out[r]["tr_f"]), bits(ref["tr_f"])), r
        lo, nl = ctxs[r].elem_lo, ctxs[r].n_loc
        x[lo:lo + nl] = out[r]["x"][lo:lo + nl]
    assert np.array_equal(bits(x), bits(ref["x"]))
    for c in ctxs:
        c.close()
    grp.close()
