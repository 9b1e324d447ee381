"""Contexts created after others were destroyed give the same bits (round 6).

With physically contiguous vectors freed back to the driver (LBFGS_VEC_ALLOC=contiguous, A/B only),
tools/repeat_stress.py found the emulated 4-rank vector-free solve's f(x0) / |g(x0)| wrong right
after a context of n = 300,007 had been solved and destroyed (99 of 400 repetitions), and never
with plain allocations (profiles/r06/alloc_reuse/). The shipped allocation pools
contiguous vectors and never frees them. This runs that sequence - a small context solved and
destroyed, then four emulated ranks, each trajectory bit-identical to the one-rank run, four times
over - with the default allocation (these sizes are below the pool's 64 MiB: plain) and with every
vector pooled (LBFGS_VEC_POOL_MIN_MB=0), which makes each context reuse the previous ones' vectors.
"""
import os
import sys
import threading

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


@pytest.mark.parametrize("pool_all", [False, True])
def test_vectors_freed_then_reallocated_give_the_same_bits(monkeypatch, pool_all):
    monkeypatch.setenv("LBFGS_TICKET", "0")
    monkeypatch.delenv("LBFGS_VEC_ALLOC", raising=False)
    if pool_all:
        monkeypatch.setenv("LBFGS_VEC_POOL_MIN_MB", "0")
    n, m, iters = 4_000_003, 5, 12
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    with L.Context(n, m) as c:
        ref = c.minimize("rosenbrock", x0, "backtracking", iters, trace=True, vector_free=True)
    for rep in range(4):
        nc = 300_007
        with L.Context(nc, 5) as c:
            c.minimize("rosenbrock", L.x0_uniform(nc, rep, -2.0, 2.0), "wolfe", 5, trace=True)
        grp = L.HostGroup(4)
        ctxs = [L.Context(n, m, rank=r, group=grp) for r in range(4)]
        out, err = [None] * 4, [None] * 4

        def run(r):
            try:
                out[r] = ctxs[r].minimize("rosenbrock", x0, "backtracking", iters, trace=True, vector_free=True)
            except Exception as e:  # pragma: no cover
                err[r] = e

        th = [threading.Thread(target=run, args=(r,)) for r in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        modes = [c.vector_pool for c in ctxs]
        for c in ctxs:
            c.close()
        grp.close()
        assert not any(err), err
        assert all(md[0] == "pool" for md in modes), modes
        if pool_all:  # every vector came from (or went into) the pool
            assert all(md[1] > 0 for md in modes), modes
        for r in range(4):
            for key in ("tr_f", "tr_gnorm", "tr_alpha"):
                assert np.array_equal(bits(out[r][key]), bits(ref[key])), (rep, r, key)
