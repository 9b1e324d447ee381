#!/usr/bin/env python3
"""Soak of the small-n launches queued ahead: seeded random sizes (nseg <= 256),
histories 1..16, every objective and line search, a few hundred runs with LBFGS_SPEC=1 and =0:
trajectories, messages, x must match bit for bit. Prints one JSON summary line.

usage: python tools/spec_soak.py [cases] [out.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402


def run(spec, n, m, obj, ls, iters, seed):
    os.environ["LBFGS_SPEC"] = spec
    x0 = L.x0_uniform(n, seed, -2.0, 2.0)
    with L.Context(n, m) as c:
        r = c.minimize(obj, x0, ls, iters, trace=True)
        r["spec"] = c.spec_stats()
    return r


def bits(a):
    return np.asarray(a, np.float64).view(np.uint64)


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rs = np.random.RandomState(777)
    objs, lss = ["rosenbrock", "quad_tridiag", "quad_sep"], list(L.LINE_SEARCHES)
    bad, taken, dropped, t0 = [], 0, 0, time.time()
    for i in range(cases):
        n, m = int(rs.randint(1000, 131073)), int(rs.randint(1, 17))
        obj, ls, seed = objs[rs.randint(3)], lss[rs.randint(4)], int(rs.randint(1, 1 << 30))
        if obj == "quad_sep" and ls == "wolfe":
            continue
        iters = int(rs.randint(20, 200))
        with np.errstate(all="ignore"):
            a = run("0", n, m, obj, ls, iters, seed)
            b = run("1", n, m, obj, ls, iters, seed)
        ok = all(np.array_equal(bits(a[k]), bits(b[k])) for k in ("tr_f", "tr_gnorm", "tr_alpha", "x"))
        ok = ok and a["messages"] == b["messages"] and a["iterations"] == b["iterations"]
        taken += b["spec"][0]
        dropped += b["spec"][1]
        if not ok:
            bad.append(dict(n=n, m=m, obj=obj, ls=ls, seed=seed, iters=iters))
        if i % 25 == 0:
            print(f"{i}/{cases} taken {taken} dropped {dropped} bad {len(bad)} ({time.time() - t0:.0f} s)", flush=True)
    out = dict(cases=cases, taken=taken, dropped=dropped, mismatches=bad, seconds=round(time.time() - t0, 1))
    print(json.dumps(out), flush=True)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fp:
            json.dump(out, fp, indent=1)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
