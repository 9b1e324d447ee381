"""A/B of the vectors' placement in HBM (LBFGS_ALLOC, lbfgs_driver.c ctx_create), alternating in one
process: configs[2]'s geometry (n = 1e8, m = 10), history filled, 40 timed steps (wall clock, no
events), 10 steps with per-launch events (k_axpy_dot / k_axpy2_dot / k_commit durations), and the
probe's stream over the solver's q against a fresh scratch vector.
usage: python tools/alloc_ab.py out.json [modes, e.g. 0,1,2,3] [rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402


def one(mode, x0, n, m):
    os.environ["LBFGS_ALLOC"] = str(mode)
    with L.Context(n, m) as c:
        c.init("rosenbrock", x0, "backtracking", tolerance=1e-5)
        c.step(m + 10)
        c.sync()
        t0 = time.perf_counter()
        c.step(40)
        c.sync()
        wall = (time.perf_counter() - t0) / 40
        c.prof_reset()
        c.prof_enable(True)
        c.step(10)
        c.sync()
        c.prof_enable(False)
        k = {kind: round(c.prof_get(kind)["ms"] / max(c.prof_get(kind)["launches"], 1) * 1e3, 1)
             for kind in ("axpy_dot", "axpy2_dot", "mid", "commit")}
        SCR = 8 + 2 * (m + 1)
        pq = c.stream_probe_vectors(5, 15, 12, 10)
        ps = c.stream_probe_vectors(SCR, 15, 12, 10)
        addr = {i: hex(c.vector_address(i)) for i in (0, 5, 6, 8, 9, 28, 29)}
    return dict(mode=mode, it_s=round(1.0 / wall, 3), ms=round(wall * 1e3, 3), kernels_us=k,
                probe_q_us=round(pq, 1), probe_scratch_us=round(ps, 1), addr=addr)


def main():
    out = sys.argv[1]
    modes = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2,3").split(",")]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    n, m = 10 ** 8, 10
    L.lib()
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    res = []
    for r in range(rounds):
        for mode in (modes if r % 2 == 0 else modes[::-1]):
            d = one(mode, x0, n, m)
            d["round"] = r
            res.append(d)
            print(json.dumps(d), flush=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
