"""Sharded solves over the xGMI peer exchange (lbfgs_xgmi.hip), one process per rank, no RCCL:
bit-exact with the single-GPU trajectory.

The box has one GPU, so every rank runs on device 0 and the mailboxes are IPC-mapped between
processes of the same device: the kernel, wire format, epoch/parity protocol, bootstrap and
self-test are exactly those of the cross-GPU case; only the xGMI hop itself is not exercised.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

pytestmark = pytest.mark.gpu
WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "xgmi_worker.py")


def bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def run_ranks(tmp_path, world, n, m, obj, ls, iters, mode, env=None, unset=(), timeout=150):
    e = {k: v for k, v in os.environ.items() if k not in unset}
    e.setdefault("LBFGS_XGMI_TIMEOUT", "20")  # a lost exchange fails the test instead of hanging it
    e.update(env or {})
    procs = [subprocess.Popen([sys.executable, WORKER, str(tmp_path), str(r), str(world), str(n), str(m), obj, ls,
                               str(iters), mode], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=e)
             for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:  # pragma: no cover
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for r, p in enumerate(procs):
        assert p.returncode == 0, (r, outs[r][-3000:])
    return [dict(np.load(os.path.join(tmp_path, f"out{r}.npz"))) for r in range(world)]


@pytest.mark.parametrize("world,obj,ls,mode,ticket", [
    (2, "rosenbrock", "backtracking", "default", "0"),
    (2, "quad_tridiag", "wolfe", "default", "1"),
    (4, "rosenbrock", "backtracking", "default", "1"),
    (4, "rosenbrock", "wolfe", "default", "0"),
    (2, "rosenbrock", "backtracking", "vf", "0"),
    (4, "rosenbrock", "interpolation", "vf", "1"),
    (8, "rosenbrock", "backtracking", "default", "1"),
    (8, "quad_tridiag", "wolfe", "vf", "0"),
])
def test_xgmi_sharded_bit_exact(tmp_path, world, obj, ls, mode, ticket):
    n = 4_000_003  # every one of up to 8 ranks owns segments
    m, iters = 5, 12
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    with L.Context(n, m) as c:
        ref = c.minimize(obj, x0, ls, iters, trace=True, vector_free=(mode == "vf"))
    outs = run_ranks(tmp_path, world, n, m, obj, ls, iters, mode,
                     env={"LBFGS_TICKET": ticket})
    x = np.zeros(n)
    for r, o in enumerate(outs):
        for key in ("tr_f", "tr_gnorm", "tr_alpha"):
            assert np.array_equal(bits(o[key]), bits(ref[key])), (r, key)
        assert np.array_equal(o["tr_c1"], ref["tr_c1"]) and np.array_equal(o["tr_c2"], ref["tr_c2"]), r
        lo = int(o["lo"])
        x[lo:lo + len(o["x"])] = o["x"]
        assert str(o["messages"]) == ref["messages"]
    assert np.array_equal(bits(x), bits(ref["x"]))


@pytest.mark.parametrize("world,obj,ls,mode", [
    (2, "rosenbrock", "backtracking", "default"),
    (4, "quad_tridiag", "wolfe", "default"),
    (8, "rosenbrock", "interpolation", "default"),
    (2, "rosenbrock", "backtracking", "vf"),
])
def test_xgmi_folded_exchange_bit_exact(tmp_path, world, obj, ls, mode):
    """The two-loop's exchanges folded into the passes (LBFGS_XGMI_FOLD=2 forces it for ranks
    sharing this one GPU; it is the default when every rank has a GPU of its own): the producing
    pass's stage 2 pushes its group value, an r pass its rank edges, straight into the peers'
    mailboxes, and the consuming pass polls them in its prologue. In-launch (ticket) stage 2, as
    every sharded run with segments >= 8192 elements uses. Bit-identical to one GPU."""
    n, m, iters = 4_000_003, 5, 12
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    with L.Context(n, m) as c:
        ref = c.minimize(obj, x0, ls, iters, trace=True, vector_free=(mode == "vf"))
    outs = run_ranks(tmp_path, world, n, m, obj, ls, iters, mode, env={"LBFGS_TICKET": "1", "LBFGS_XGMI_FOLD": "2"})
    x = np.zeros(n)
    for r, o in enumerate(outs):
        assert bool(o["folded"])  # vector-free runs fold nothing but report the setting
        for key in ("tr_f", "tr_gnorm", "tr_alpha"):
            assert np.array_equal(bits(o[key]), bits(ref[key])), (r, key)
        assert np.array_equal(o["tr_c1"], ref["tr_c1"]) and np.array_equal(o["tr_c2"], ref["tr_c2"]), r
        lo = int(o["lo"])
        x[lo:lo + len(o["x"])] = o["x"]
        assert str(o["messages"]) == ref["messages"]
    assert np.array_equal(bits(x), bits(ref["x"]))


@pytest.mark.parametrize("world,obj,ls,mode", [
    (2, "rosenbrock", "backtracking", "default"),
    (4, "rosenbrock", "wolfe", "default"),
    (8, "rosenbrock", "backtracking", "default"),
    (8, "quad_tridiag", "wolfe", "default"),
    (4, "rosenbrock", "interpolation", "default"),
    (4, "rosenbrock", "backtracking", "vf"),
    (8, "rosenbrock", "backtracking_wolfe", "vf"),
])
@pytest.mark.parametrize("ticket", ["0", "1"])
def test_xgmi_ungated_fold_cu_partitioned(tmp_path, world, obj, ls, mode, ticket):
    """The folded exchanges exactly as ranks on distinct GPUs run them: the library's default fold
    setting (LBFGS_XGMI_FOLD unset) with every rank's stream confined to its own 1/world of the
    CUs (LBFGS_CU_PARTITION=1), so no collect gate runs before a consuming pass and its workgroups
    wait for the peers' pushes in their prologue (src_total_mailbox) while those producers run on
    CUs of their own. Both producers: the reduce kernel's workgroups (ticket 0) and the group's
    last arriving workgroup (ticket 1). Bit-identical to one GPU."""
    n, m, iters = 4_000_003, 5, 12
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    with L.Context(n, m) as c:
        ref = c.minimize(obj, x0, ls, iters, trace=True, vector_free=(mode == "vf"))
    outs = run_ranks(tmp_path, world, n, m, obj, ls, iters, mode,
                     env={"LBFGS_TICKET": ticket, "LBFGS_CU_PARTITION": "1"}, unset=("LBFGS_XGMI_FOLD",))
    x = np.zeros(n)
    for r, o in enumerate(outs):
        assert bool(o["folded"]) and int(o["cu_part"]) == int(outs[0]["cu_part"]) > 0, (r, o["folded"], o["cu_part"])
        for key in ("tr_f", "tr_gnorm", "tr_alpha"):
            assert np.array_equal(bits(o[key]), bits(ref[key])), (r, key)
        assert np.array_equal(o["tr_c1"], ref["tr_c1"]) and np.array_equal(o["tr_c2"], ref["tr_c2"]), r
        lo = int(o["lo"])
        x[lo:lo + len(o["x"])] = o["x"]
        assert str(o["messages"]) == ref["messages"]
    assert np.array_equal(bits(x), bits(ref["x"]))


def test_xgmi_fold_off_on_a_shared_gpu(tmp_path):
    """Ranks sharing one GPU do not fold by default (a pass's spinning workgroups could hold the CUs
    the peer's producing kernel waits for); the exchange kernel carries their reductions."""
    outs = run_ranks(tmp_path, 2, 4_000_003, 5, "rosenbrock", "backtracking", 3, "default", unset=("LBFGS_XGMI_FOLD",))
    assert not any(bool(o["folded"]) for o in outs)


def test_xgmi_soak_8_ranks_bit_exact(tmp_path):
    """A long sharded solve (8 ranks, 1500 iterations, ~2e4 mailbox exchanges per rank through
    both parities) stays bit-identical to one GPU: a protocol race (epoch reuse, a stale
    mailbox word) would show as a wrong value or a timeout."""
    n, m, iters = 4_000_003, 5, 1500
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)  # the worker's seed
    with L.Context(n, m) as c:
        ref = c.minimize("rosenbrock", x0, "backtracking", iters, trace=True)
    outs = run_ranks(tmp_path, 8, n, m, "rosenbrock", "backtracking", iters, "default",
                     env={"LBFGS_TICKET": "1"}, timeout=280)
    x = np.zeros(n)
    for r, o in enumerate(outs):
        for key in ("tr_f", "tr_gnorm", "tr_alpha"):
            assert np.array_equal(bits(o[key]), bits(ref[key])), (r, key)
        lo = int(o["lo"])
        x[lo:lo + len(o["x"])] = o["x"]
    assert np.array_equal(bits(x), bits(ref["x"]))


def test_xgmi_silent_peer_times_out(tmp_path):
    """A peer that publishes its handle but never exchanges must not hang the others: rank 0's
    self-test gives up after its timeout (LBFGS_XGMI_SELFTEST_TIMEOUT) and no rank enables the
    peer exchange."""
    e = dict(os.environ, LBFGS_XGMI_SELFTEST_TIMEOUT="3")
    args = [str(tmp_path), "", "2", "4000003", "5", "rosenbrock", "backtracking", "3", "default"]
    procs = []
    for r, mode in ((0, "default"), (1, "silent")):
        a = list(args)
        a[1], a[8] = str(r), mode
        procs.append(subprocess.Popen([sys.executable, WORKER] + a, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True, env=e))
    outs = [p.communicate(timeout=180)[0] for p in procs]
    assert procs[0].returncode == 3, outs[0][-2000:]
    assert "timed out" in outs[0], outs[0][-2000:]
    assert procs[1].returncode == 0, outs[1][-2000:]


@pytest.mark.parametrize("fold", ["0", "2", "cu"])
def test_xgmi_stalled_peer_fails_once(tmp_path, fold):
    """A peer that connects and then stops exchanging: the solving rank's first wait times out
    (LBFGS_XGMI_TIMEOUT = 3 s) and every exchange queued behind it ends within ~1/65536 of that
    once the error word is set, so the solve fails in about one timeout, not one per exchange
    queued before the host's next synchronisation (with the fold forced, the gated consumers'
    collect launches wait the same way; "cu": the CUs partitioned, the fold ungated as across
    GPUs, so the consuming passes' own prologues time out). The stalled rank stays alive
    meanwhile, so its mailbox stays mapped."""
    e = dict(os.environ, LBFGS_XGMI_TIMEOUT="3", XGMI_STALL_S="25")
    if fold == "cu":
        e.pop("LBFGS_XGMI_FOLD", None)
        e["LBFGS_CU_PARTITION"] = "1"
    else:
        e["LBFGS_XGMI_FOLD"] = fold
    args = [str(tmp_path), "", "2", "4000003", "5", "rosenbrock", "backtracking", "40", ""]
    procs = []
    for r, mode in ((0, "expect_fail"), (1, "stall")):
        a = list(args)
        a[1], a[8] = str(r), mode
        procs.append(subprocess.Popen([sys.executable, WORKER] + a, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True, env=e))
    outs = [p.communicate(timeout=180)[0] for p in procs]
    assert procs[0].returncode == 4, outs[0][-2000:]
    took = float(outs[0].split("failed after ")[1].split(" s")[0])
    assert took < 15.0, outs[0][-2000:]
    assert procs[1].returncode == 0, outs[1][-2000:]


def test_xgmi_exchange_latency_collective(tmp_path):
    """lbfgs_exchange_latency (bench.py's exchange_latency_us) runs as a collective on every rank
    and returns a positive per-exchange time for both slot widths."""
    outs = run_ranks(tmp_path, 2, 4_000_003, 5, "rosenbrock", "backtracking", 1, "latency")
    for o in outs:
        assert 0.0 < float(o["us8"]) < 1e5 and 0.0 < float(o["us96"]) < 1e5
