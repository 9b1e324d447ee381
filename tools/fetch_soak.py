#!/usr/bin/env python3
"""Soak of the slot fetches that poll a k_slot_publish word (DESIGN.md §5 "Host side"): seeded
random sizes with more than 1024 segments (n in [6e5, 4e6], so stage 2 runs in several groups and
every fetch of the iteration takes that path), histories 1..20, every objective and line search,
the default and vector-free modes, LBFGS_DIRECT=1 and =0 (pinned mirrors or none); each solve
compared bit for bit with the oracle's canonical restatement (f trace, final x, messages,
iterations; a diverging solve's NaNs match any NaN, see same()). Prints progress and one JSON summary line.

usage: python tools/fetch_soak.py [cases] [out.json]
"""
import json
import os
import random
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


def same(a, b):
    """bit for bit, except that any NaN matches any NaN: a diverging solve's NaNs carry the sign
    of the operation that made them, which x86 and the GPU set differently (0x7ff8... against
    0xfff8...); the separable quadratic under Wolfe diverges to NaN in the reference too"""
    a, b = np.ascontiguousarray(a, np.float64), np.ascontiguousarray(b, np.float64)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    return bool(np.array_equal(na, nb) and np.array_equal(bits(a[~na]), bits(b[~nb])))


def msgs(s):
    return s.replace("-nan", "nan")


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    rnd = random.Random(20261018)
    objs = ["rosenbrock", "quad_tridiag", "quad_sep"]
    lss = ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"]
    bad, rows, t0 = [], [], time.time()
    for i in range(cases):
        n = rnd.randint(600_000, 4_000_000)
        m = rnd.randint(1, 20)
        obj, ls = rnd.choice(objs), rnd.choice(lss)
        vf = rnd.random() < 0.3 and m <= 20
        direct = "0" if rnd.random() < 0.3 else "1"
        iters = rnd.randint(10, 40)
        seed = rnd.randint(1, 10 ** 6)
        os.environ["LBFGS_DIRECT"] = direct
        x0 = L.x0_uniform(n, seed, -2.0, 2.0)
        with L.Context(n, m) as c:
            r = c.minimize(obj, x0, ls, iters, tolerance=1e-5, trace=True, vector_free=vf)
        with np.errstate(all="ignore"):
            o = O.lbfgs(obj, x0, ls, m, iters, 1e-5, mode=O.CANON, vector_free=vf)
        ok = (same(r["tr_f"], o["f"]) and same(r["x"], o["x"]) and msgs(r["messages"]) == msgs(o["messages"])
              and r["iterations"] == o["iters"])
        nan = bool(np.isnan(r["tr_f"]).any())
        row = dict(i=i, n=n, m=m, obj=obj, ls=ls, vector_free=vf, direct=direct, iters=iters, seed=seed,
                   gpu_iterations=r["iterations"], nan_states=nan, ok=bool(ok))
        rows.append(row)
        if not ok:
            bad.append(row)
        print(json.dumps(row), flush=True)
    os.environ.pop("LBFGS_DIRECT", None)
    out = dict(tool="tools/fetch_soak.py", cases=cases, mismatches=len(bad), bad=bad,
               seconds=round(time.time() - t0, 1), build=L.build_info()[0])
    if len(sys.argv) > 2:
        json.dump(dict(out, rows=rows), open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
