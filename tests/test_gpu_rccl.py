"""The sharded exchange's RCCL leg, executed on a one-GPU box, and configs[4]'s shard geometry.

* A world = 1 context created with an RCCL unique id owns a one-rank communicator and sends every
  reduction through the sharded path's in-place ncclAllGather (lbfgs_kernels.hip exchange_buf) and
  the trajectory checksum through ncclAllReduce, with the one-rank shortcuts (cooperative
  iteration, deferred / host-mirrored stage 2) off. Its trajectory must be the unsharded one bit
  for bit. Two ranks cannot share one device under RCCL ("Duplicate GPU detected"), so this is as
  far as RCCL itself runs here; the multi-rank data path is pinned by the emulated ranks below
  and in test_gpu_parity.py, which exchange the same slot layout where RCCL all-gathers.
* configs[4] (n = 1e9, m = 10, 8 ranks) shards with segments of L >= 8192 elements and the
  in-launch ticket stage 2 (lbk_create's rule for world > 1, L >= 8192). n = 8192^2 + 1 is the
  smallest n with that geometry (L = 8320); 8 emulated ranks at m = 10 must reproduce the
  single-GPU run and the canonical oracle bit for bit.
"""
import os
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402
import oracle_lib as O  # noqa: E402

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def same_run(a, b):
    for key in ("tr_f", "tr_gnorm", "x"):
        assert np.array_equal(bits(a[key]), bits(b[key])), key
    ta, tb = a["tr_alpha"], b["tr_alpha"]
    assert np.array_equal(np.isnan(ta), np.isnan(tb))
    assert np.array_equal(ta[~np.isnan(ta)], tb[~np.isnan(tb)])
    assert np.array_equal(a["tr_c1"], b["tr_c1"]) and np.array_equal(a["tr_c2"], b["tr_c2"])
    assert a["messages"] == b["messages"] and a["status"] == b["status"]


CASES = [(4_000_003, 5, "rosenbrock", "backtracking", 12, False, None),
         (100_000, 10, "rosenbrock", "wolfe", 40, False, None),        # cooperative when unsharded
         (700_001, 10, "rosenbrock", "backtracking", 14, False, None),  # deferred stage 2 unsharded
         (2_000_000, 7, "quad_tridiag", "interpolation", 12, False, "1"),
         (1_000_001, 6, "rosenbrock", "backtracking_wolfe", 12, False, "0"),
         (3_000_000, 10, "rosenbrock", "backtracking", 12, True, None)]


@pytest.mark.parametrize("n,m,obj,ls,iters,vf,ticket", CASES)
def test_rccl_one_rank_bit_identical(monkeypatch, n, m, obj, ls, iters, vf, ticket):
    if ticket is not None:
        monkeypatch.setenv("LBFGS_TICKET", ticket)
    x0 = L.x0_uniform(n, 11, -2.0, 2.0)
    with L.Context(n, m) as c:
        ref = c.minimize(obj, x0, ls, iters, trace=True, vector_free=vf)
    with L.Context(n, m, world=1, uid=L.unique_id()) as c:
        assert c.backend == "rccl"
        c.prof_reset()
        c.prof_enable(True)
        got = c.minimize(obj, x0, ls, iters, trace=True, vector_free=vf)
        c.prof_enable(False)
        us = c.exchange_latency("rccl", components=8, iters=50)
    same_run(got, ref)
    assert us > 0.0


_STALL_CHILD = r"""
import json, os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "cuda-lbfgs_amd"))
import lbfgs_amd as L
n = 1_000_003
x0 = L.x0_uniform(n, 5, -2.0, 2.0)
out = {}
try:
    with L.Context(n, 5, world=1, uid=L.unique_id()) as c:
        out["backend"] = c.backend
        t0 = time.monotonic()
        try:
            c.minimize("rosenbrock", x0, "backtracking", 10)
            out["error"] = None
        except L.LbfgsError as e:
            out["error"] = str(e)
        out["took"] = time.monotonic() - t0
except Exception as e:
    out["setup_error"] = repr(e)
print(json.dumps(out), flush=True)
os._exit(0)  # an abandoned RCCL thread must not hold the interpreter's teardown
"""


def test_rccl_stalled_collective_mid_solve_fails_bounded():
    """A collective that does not complete mid-solve (a peer that stops answering) ends the solve
    with LBFGS_ERR_RCCL within the RCCL bound instead of hanging the rank: every host
    wait on a stream that carries RCCL work is bounded (lbfgs_kernels_impl.h stream_wait). The
    stalled peer is stood in for by a device-side sleep queued ahead of each collective, longer than
    the bound of the waits on collectives (LBFGS_DEBUG_RCCL_STALL="stall_ms,wait_s"); the sleep ends
    on its own. The communicator's init keeps its own bound (LBFGS_RCCL_TIMEOUT, 60 s). Runs in a
    child process under a time limit, so nothing RCCL leaves behind can hold this one."""
    import json
    import subprocess
    env = dict(os.environ, LBFGS_DEBUG_RCCL_STALL="4000,0.5")
    p = subprocess.run([sys.executable, "-c", _STALL_CHILD, ROOT], env=env, capture_output=True, text=True,
                       timeout=150)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    out = json.loads(lines[-1])
    assert "setup_error" not in out and out["backend"] == "rccl", out
    err = out["error"] or ""
    assert "(-3)" in err and "did not complete" in err, out
    assert out["took"] < 3.5, out  # the 0.5 s bound (twice at most), not the 4 s stall, nor a hang


N4 = 8192 * 8192 + 1  # smallest n whose canonical segments are >= 8192 long (L = 8320)


def test_config4_geometry():
    for world in (1, 8):
        lo, nl = L.shard_range(N4, 0, world)
        assert lo == 0
    # 8066 segments of 8320: ranks 0..6 own 1024 each, rank 7 the remaining 898 (the last short)
    spans = [L.shard_range(N4, r, 8) for r in range(8)]
    assert sum(nl for _, nl in spans) == N4
    assert all(lo == r * 1024 * 8320 for r, (lo, _) in enumerate(spans))
    assert all(nl == 1024 * 8320 for _, nl in spans[:7])
    assert spans[7][1] == N4 - 7 * 1024 * 8320 > 897 * 8320


_single = {}


def _single_run(ls, iters):
    key = (ls, iters)
    if key not in _single:
        x0 = L.x0_uniform(N4, 42, -2.0, 2.0)
        with L.Context(N4, 10) as c:
            _single[key] = c.minimize("rosenbrock", x0, ls, iters, trace=True)
    return _single[key]


@pytest.mark.parametrize("ls", ["backtracking", "wolfe"])
def test_config4_shard_geometry_8_ranks_m10(ls):
    """8 emulated ranks (threads, one stream each, exchanging through host memory exactly where
    the ranks all-gather) at m = 10 on configs[4]'s segment geometry (L = 8320, ticket stage 2):
    the single-GPU trajectory bit for bit over 12 iterations (h reaches m = 10)."""
    iters, world = 12, 8
    x0 = L.x0_uniform(N4, 42, -2.0, 2.0)
    ref = _single_run(ls, iters)
    grp = L.HostGroup(world)
    ctxs = [L.Context(N4, 10, rank=r, group=grp) for r in range(world)]
    out, err = [None] * world, [None] * world

    def run(r):
        try:
            out[r] = ctxs[r].minimize("rosenbrock", x0, ls, iters, trace=True)
        except Exception as e:  # pragma: no cover
            err[r] = e

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(err), err
    x = np.zeros(N4)
    for r in range(world):
        o = out[r]
        for key in ("tr_f", "tr_gnorm", "tr_alpha"):
            assert np.array_equal(bits(o[key]), bits(ref[key])), (r, key)
        assert np.array_equal(o["tr_c1"], ref["tr_c1"]) and np.array_equal(o["tr_c2"], ref["tr_c2"])
        assert o["h_max"] == ref["h_max"] == 10  # the ring is full by the last iterations
        lo, nl = ctxs[r].elem_lo, ctxs[r].n_loc
        x[lo:lo + nl] = o["x"][lo:lo + nl]
    assert np.array_equal(bits(x), bits(ref["x"]))
    for c in ctxs:
        c.close()
    grp.close()


def test_config4_shard_geometry_vs_canonical_oracle():
    """The same geometry against the CPU oracle's canonical order (ORC_CANON): f, |g| and the
    x checksum of every iteration, bit for bit (10 iterations; ~1 min of oracle time)."""
    iters = 10
    ref = _single_run("backtracking", 12)
    x0 = O.x0_uniform(N4, 42, -2.0, 2.0)
    o = O.lbfgs("rosenbrock", x0, "backtracking", 10, iters, 1e-5, mode=O.CANON)
    k = len(o["f"]) - 1  # the oracle's trace ends with the max-iterations entry
    assert np.array_equal(bits(ref["tr_f"][:k]), bits(o["f"][:k]))
    assert np.array_equal(bits(ref["tr_gnorm"][:k]), bits(o["gnorm"][:k]))
    assert np.array_equal(ref["tr_c1"][:k], o["c1"][:k]) and np.array_equal(ref["tr_c2"][:k], o["c2"][:k])
