"""Which of the context's vectors stream slowly together (the pass-vs-probe gap).

One context at configs[2]'s geometry (n = 1e8, m = 10) with its history filled; then the probe's
3 R + 1 W stream (alpha = 0) over chosen triplets of the context's own vectors
(lbfgs_stream_probe_vectors), 10 launches each, alternating:
  * the written vector q over the work vectors and a fresh scratch allocation, (y, s) fixed;
  * (y_p, s_{p-1}) over the pool with the solver's q, and with the scratch vector.
Prints and writes (argv[1]) the times with every vector's device address.
usage: python tools/placement_probe.py out.json [n]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

NAMES = ["x", "g", "xn", "gn", "d", "q", "r", "gt"]


def main():
    out = sys.argv[1]
    n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10 ** 8
    m = 10
    SCR = 8 + 2 * (m + 1)
    name = {k: v for k, v in enumerate(NAMES)}
    for p in range(m + 1):
        name[8 + 2 * p], name[9 + 2 * p] = f"S{p}", f"Y{p}"
    name[SCR] = "scratch"
    L.lib()
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    res = {"n": n, "m": m, "addresses": {}, "q_sweep": {}, "pair_sweep_q": {}, "pair_sweep_scratch": {}}
    with L.Context(n, m) as c:
        c.init("rosenbrock", x0, "backtracking", tolerance=1e-5)
        del x0
        c.step(m + 4)
        c.sync()
        for k in range(SCR):
            a = c.vector_address(k)
            res["addresses"][name[k]] = hex(a) if a else None
        y, s = 9 + 2 * 3, 8 + 2 * 2  # Y3, S2
        for rnd in range(3):
            for qk in [5, 6, 4, 2, 3, 7, SCR]:
                res["q_sweep"].setdefault(name[qk], []).append(round(c.stream_probe_vectors(qk, y, s, 10), 1))
            for p in range(1, m + 1):
                yk, sk = 9 + 2 * p, 8 + 2 * (p - 1)
                key = f"{name[yk]},{name[sk]}"
                res["pair_sweep_q"].setdefault(key, []).append(round(c.stream_probe_vectors(5, yk, sk, 10), 1))
                res["pair_sweep_scratch"].setdefault(key, []).append(round(c.stream_probe_vectors(SCR, yk, sk, 10), 1))
            print(f"round {rnd}: q sweep " + ", ".join(f"{k} {v[-1]}" for k, v in res["q_sweep"].items()), flush=True)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    for key in ("q_sweep", "pair_sweep_q", "pair_sweep_scratch"):
        res[key + "_median"] = {k: med(v) for k, v in res[key].items()}
    res["build"] = L.build_info()[0]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["q_sweep_median"]))
    print("pairs with q:", json.dumps(res["pair_sweep_q_median"]))
    print("pairs with scratch:", json.dumps(res["pair_sweep_scratch_median"]))
    print(json.dumps(res["addresses"]))


if __name__ == "__main__":
    main()
