#!/usr/bin/env python3
"""A/B of the device-resident line searches at small n (LBFGS_DEV_SEARCH=0 / 1, alternating, twice):
microseconds per iteration of 1000 Rosenbrock iterations (m = 5) after 50 warm-up ones, for each of
the four searches; the trajectories and the trial / commit counters must be identical between the two. Also
prints how many iterations needed the device search and how many of its launches took the commit.

usage: python tools/search_ab.py <n> [out.json]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402
import numpy as np  # noqa: E402

n, m = int(float(sys.argv[1])), 5
x0 = L.x0_uniform(n, 42, -2.0, 2.0)
SEARCHES = ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"]
res, rows = {}, []
for rep in range(2):
    for dv in ("0", "1"):
        os.environ["LBFGS_DEV_SEARCH"] = dv
        with L.Context(n, m) as c:
            for ls in SEARCHES:
                c.minimize("rosenbrock", x0, ls, 50)
                t = time.perf_counter()
                r = c.minimize("rosenbrock", x0, ls, 1000, trace=True)
                dt = time.perf_counter() - t
                sl, sc = c.search_stats()
                key = (dv, ls)
                # (passes may differ by d's materialisation, at most one per device launch)
                sig = (r["tr_f"].view(np.uint64).tobytes(), r["trials_f"], r["trials_fg"], r["commits"])
                if key in res:
                    assert res[key] == sig
                res[key] = sig
                us = dt / r["iterations"] * 1e6
                rows.append(dict(n=n, dev_search=int(dv), ls=ls, rep=rep, us_per_it=round(us, 2),
                                 iterations=r["iterations"], trials_f=r["trials_f"], trials_fg=r["trials_fg"],
                                 passes=r["passes"], device_searches=sl, device_commits=sc))
                print(f"n={n} dev_search={dv} {ls:19s}: {us:7.1f} us/it  trials_f={r['trials_f']} "
                      f"trials_fg={r['trials_fg']} passes={r['passes']} device searches={sl} commits={sc}", flush=True)
same = {ls: res[("0", ls)] == res[("1", ls)] for ls in SEARCHES}
print("trajectories and counters identical:", same)
if len(sys.argv) > 2:
    with open(sys.argv[2], "w") as fp:
        json.dump(dict(tool="tools/search_ab.py", n=n, m=m, rows=rows, identical=same, build=L.build_info()[0]), fp)
sys.exit(0 if all(same.values()) else 1)
