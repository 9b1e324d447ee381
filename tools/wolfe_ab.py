#!/usr/bin/env python3
"""A/B of the device-resident Wolfe search at small n (LBFGS_DEV_WOLFE=0 / 1, alternating, twice):
microseconds per iteration of 1000 Rosenbrock iterations (m = 5) after 50 warm-up ones, Wolfe and,
as the control, backtracking; the Wolfe trajectories must be bit-identical.

usage: python tools/wolfe_ab.py <n>
"""
import sys, time, os
sys.path.insert(0, 'cuda-lbfgs_amd')
import lbfgs_amd as L, numpy as np
n, m = int(float(sys.argv[1])), 5
x0 = L.x0_uniform(n, 42, -2.0, 2.0)
res = {}
for rep in range(2):
    for dw in ("0", "1"):
        os.environ["LBFGS_DEV_WOLFE"] = dw
        with L.Context(n, m) as c:
            for ls in ["wolfe", "backtracking"]:
                c.minimize("rosenbrock", x0, ls, 50)
                t = time.perf_counter(); r = c.minimize("rosenbrock", x0, ls, 1000, trace=True); dt = time.perf_counter() - t
                key = (dw, ls)
                if key in res:
                    assert np.array_equal(res[key][1].view(np.uint64), r["tr_f"].view(np.uint64))
                res[key] = (dt, r["tr_f"])
                print(f"n={n} dev_wolfe={dw} {ls}: {dt/r['iterations']*1e6:.1f} us/it trials_fg={r['trials_fg']} passes={r['passes']}", flush=True)
a, b = res[("0", "wolfe")][1], res[("1", "wolfe")][1]
print("wolfe trajectories bit-identical:", np.array_equal(a.view(np.uint64), b.view(np.uint64)))
