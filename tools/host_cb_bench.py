#!/usr/bin/env python3
"""Host-callback objectives (LBFGS_OBJ_HOST) at scale: Rosenbrock n = 1e7, m = 10
with numpy callables, the default call policy (one f and at most one grad per distinct point)
against the reference's call sequence (LBFGS_FLAG_REFERENCE_CALLS), backtracking and Wolfe.
Reports seconds per iteration, f / grad calls per iteration, and the same solve with the device
objective for scale. Trajectories are checked identical between the two call policies.

usage: python tools/host_cb_bench.py [out.json] [--n N] [--iters K]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

L.lib()


def f_np(x):  # benchmark.cpp:58-68 (vectorised; the rounding of a numpy sum, not the reference's)
    t1 = x[1:] - x[:-1] * x[:-1]
    t2 = 1.0 - x[:-1]
    return float(np.sum(100.0 * t1 * t1 + t2 * t2))


def g_np(x):  # benchmark.cpp:70-81
    g = np.zeros_like(x)
    t2 = x[1:] - x[:-1] * x[:-1]
    g[:-1] = 2.0 * (x[:-1] - 1.0) - 400.0 * x[:-1] * t2
    g[1:] += 200.0 * t2
    return g


def main():
    n = int(float(sys.argv[sys.argv.index("--n") + 1])) if "--n" in sys.argv else 10**7
    iters = int(sys.argv[sys.argv.index("--iters") + 1]) if "--iters" in sys.argv else 20
    outp = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else None
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    res = dict(n=n, m=10, iterations=iters, objective="rosenbrock via numpy callables")
    with L.Context(n, 10) as c:
        for ls in ("backtracking", "wolfe"):
            runs = {}
            for policy in ("default", "reference_calls"):
                cnt = {"f": 0, "g": 0}

                def f(x):
                    cnt["f"] += 1
                    return f_np(x)

                def g(x):
                    cnt["g"] += 1
                    return g_np(x)

                t0 = time.perf_counter()
                r = c.minimize("host", x0, ls, iters, f=f, grad=g, trace=True,
                               reference_calls=policy == "reference_calls")
                dt = time.perf_counter() - t0
                k = max(r["iterations"], 1)
                runs[policy] = dict(seconds=dt, s_per_iter=dt / k, iterations=r["iterations"],
                                    f_calls=r["f_calls"], grad_calls=r["grad_calls"],
                                    f_per_iter=r["f_calls"] / k, grad_per_iter=r["grad_calls"] / k,
                                    f=r["f"], tr_f=r["tr_f"])
                assert cnt["f"] == r["f_calls"] and cnt["g"] == r["grad_calls"]
            a, b = runs["default"], runs["reference_calls"]
            same = bool(np.array_equal(a.pop("tr_f").view(np.uint64), b.pop("tr_f").view(np.uint64)))
            t0 = time.perf_counter()
            rd = c.minimize("rosenbrock", x0, ls, iters)
            dd = time.perf_counter() - t0
            res[ls] = dict(default=a, reference_calls=b, same_trajectory=same,
                           speedup_default_over_reference_calls=b["seconds"] / a["seconds"],
                           device_objective=dict(seconds=dd, s_per_iter=dd / max(rd["iterations"], 1)))
            print(ls, json.dumps(res[ls]), flush=True)
    if outp:
        with open(outp, "w") as fp:
            json.dump(res, fp, indent=1)


if __name__ == "__main__":
    main()
