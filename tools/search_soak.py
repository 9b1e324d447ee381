#!/usr/bin/env python3
"""Soak of the device-resident line searches: seeded random cooperative sizes
(n up to 131 072, <= 256 segments), histories 1..20, every objective, every line search, random
tolerances and caps, in the default mode; each solve compared bit for bit with the oracle's
canonical restatement (trace f / |g| / step / x checksums, final x, messages, status, iterations),
and the host loop (LBFGS_DEV_SEARCH=0) on every tenth draw. Prints progress and one JSON summary.

usage: python tools/search_soak.py [cases] [out.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lbfgs_amd as L  # noqa: E402
import oracle_lib as O  # noqa: E402


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def same(r, o):
    a1, a2 = r["tr_alpha"], o["alpha"]
    return (r["status"] == o["status"] and r["iterations"] == o["iters"]
            and np.array_equal(bits(r["tr_f"]), bits(o["f"])) and np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
            and np.array_equal(np.isnan(a1), np.isnan(a2)) and np.array_equal(a1[~np.isnan(a1)], a2[~np.isnan(a2)])
            and np.array_equal(r["tr_c1"], o["c1"]) and np.array_equal(r["tr_c2"], o["c2"])
            and np.array_equal(bits(r["x"]), bits(o["x"])) and r["messages"] == o["messages"])


def solve(n, m, obj, ls, x0, maxit, tol, dev):
    os.environ["LBFGS_DEV_SEARCH"] = "1" if dev else "0"
    with L.Context(n, m) as c:
        r = c.minimize(obj, x0, ls, maxit, tolerance=tol, trace=True)
        r["search"] = c.search_stats()
        return r


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rs = np.random.RandomState(9090)
    objs = ["rosenbrock", "quad_tridiag", "quad_sep"]
    searches = ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"]
    bad, trials, launches, commits, t0 = [], 0, 0, 0, time.time()
    for i in range(cases):
        n = int(rs.choice([rs.randint(1, 600), rs.randint(600, 20001), rs.randint(20001, 131073)]))
        m, obj, seed = int(rs.randint(1, 21)), objs[rs.randint(3)], int(rs.randint(1, 1 << 30))
        ls = searches[rs.randint(4)]
        if obj == "quad_sep" and ls == "wolfe":  # diverges to NaN (the reference too)
            obj = "rosenbrock"
        maxit, tol = int(rs.choice([20, 100, 400])), float(10.0 ** rs.uniform(-10, -3))
        x0 = O.x0_uniform(n, seed, -2.0, 2.0)
        with np.errstate(all="ignore"):
            o = O.lbfgs(obj, x0, ls, m, maxit, tol, mode=O.CANON)
            r = solve(n, m, obj, ls, x0, maxit, tol, True)
            ok = same(r, o)
            if ok and i % 10 == 0:
                h = solve(n, m, obj, ls, x0, maxit, tol, False)
                ok = (same(h, o) and all(h[k] == r[k] for k in ("trials_f", "trials_fg", "commits"))
                      and 0 <= r["passes"] - h["passes"] <= r["search"][0])
        trials += int(r["trials_fg"]) + int(r["trials_f"])
        launches += r["search"][0]
        commits += r["search"][1]
        if not ok:
            bad.append(dict(n=n, m=m, obj=obj, ls=ls, seed=seed, maxit=maxit, tol=tol))
        if (i + 1) % 50 == 0:
            print(f"{i + 1}/{cases} solves, {len(bad)} mismatches, {time.time() - t0:.0f} s", flush=True)
    out = dict(tool="tools/search_soak.py", cases=cases, mismatches=len(bad), bad=bad[:20], trial_passes=trials,
               device_searches=launches, device_commits=commits,
               seconds=round(time.time() - t0, 1), build=L.build_info()[0])
    line = json.dumps(out)
    print(line)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fp:
            fp.write(line + "\n")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
