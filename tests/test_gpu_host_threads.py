"""A solve keeps one host thread busy (the one polling the completion words) and no runtime thread
spinning beside it (DESIGN.md §5 "Host side"): slot fetches without a completion word of their
own poll one written by k_slot_publish instead of synchronising the stream - each stream
synchronisation registered an asynchronous handler with the runtime, and the runtime thread that
serves them spun at ~1 core within a second of solving (profiles/r05/config4_cpu/). n = 1e7 has
7813 segments in 8 groups, so every fetch of the iteration takes that path. n = 1e5 under Wolfe
runs the cooperative iteration and the device-resident line search (k_coop_search), whose host
wait polls the completion word its block 0 writes."""
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

pytestmark = pytest.mark.gpu


def thread_ticks():
    out = {}
    for t in os.listdir("/proc/self/task"):
        try:
            s = open(f"/proc/self/task/{t}/stat").read()
        except OSError:
            continue
        f = s[s.rindex(")") + 2:].split()
        out[int(t)] = int(f[11]) + int(f[12])
    return out


@pytest.mark.parametrize("n,ls,vector_free", [(10 ** 7, "backtracking", False), (10 ** 7, "backtracking", True),
                                               (10 ** 5, "wolfe", False)])
def test_no_runtime_thread_spins_during_a_solve(n, ls, vector_free):
    m = 10
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    hz = os.sysconf("SC_CLK_TCK")
    with L.Context(n, m) as c:
        c.init("rosenbrock", x0, ls, tolerance=1e-5, vector_free=vector_free)
        c.step(m)
        t_end = time.perf_counter() + 1.5  # past the ~1 s after which the spinning used to start
        while time.perf_counter() < t_end:
            c.step(50)
        c.sync()
        a, t0 = thread_ticks(), time.perf_counter()
        t_end = t0 + 1.5
        while time.perf_counter() < t_end:
            r = c.step(50)
        c.sync()
        dt = time.perf_counter() - t0
        b = thread_ticks()
    assert r["status"] == "running"
    busy = sorted(((b[k] - a.get(k, 0)) / hz / dt for k in b), reverse=True)
    # the polling thread (~1 core) and nothing else near it
    assert len(busy) < 2 or busy[1] < 0.3, busy[:4]
