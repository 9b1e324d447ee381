#!/usr/bin/env python3
"""Soak of the CUDA-path modes (LBFGS_FLAG_CUDA_COMPAT, with and without LBFGS_FLAG_CUDA_VARIANT;
DESIGN.md §4.5): seeded random sizes 1 .. 3e5, histories 1..20, every objective and line search,
random tolerances and iteration caps, each solve compared bit for bit with the oracle's
restatement (tests/oracle_lib.py, ORC_CANON, cuda = 1 or 2): trace f / |g| / step / x checksums,
the final x, messages, status and iteration count. Prints progress and one JSON summary line.

usage: python tools/cuda_soak.py [cases] [out.json]
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
    return (r["status"] == o["status"] and r["iterations"] == o["iters"]
            and np.array_equal(bits(r["tr_f"]), bits(o["f"])) and np.array_equal(bits(r["tr_gnorm"]), bits(o["gnorm"]))
            and np.array_equal(bits(r["tr_alpha"]), bits(o["alpha"]))
            and np.array_equal(r["tr_c1"], o["c1"]) and np.array_equal(r["tr_c2"], o["c2"])
            and np.array_equal(bits(r["x"]), bits(o["x"])) and r["messages"] == o["messages"])


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rs = np.random.RandomState(4242)
    objs, lss = ["rosenbrock", "quad_tridiag", "quad_sep"], list(L.LINE_SEARCHES)
    consts = L.constants("cuda")
    bad, iters_total, skips, statuses, t0 = [], 0, 0, {}, time.time()
    for i in range(cases):
        n = int(rs.choice([rs.randint(1, 65), rs.randint(65, 20001), rs.randint(20001, 300001)]))
        m, cuda = int(rs.randint(1, 21)), int(rs.randint(1, 3))
        obj, ls, seed = objs[rs.randint(3)], lss[rs.randint(4)], int(rs.randint(1, 1 << 30))
        maxit = int(rs.choice([5, 30, 200, 1000 if n <= 64 else 200]))
        tol = float(10.0 ** rs.uniform(-12, -3))
        x0 = O.x0_uniform(n, seed, -2.0, 2.0)
        o = O.lbfgs(obj, x0, ls, m, maxit, tol, mode=O.CANON, cuda=cuda, consts=O.CONSTANTS_H)
        with L.Context(n, m) as c:
            r = c.minimize(obj, x0, ls, maxit, tolerance=tol, trace=True, cuda_compat=True,
                           cuda_variant=cuda == 2, consts=consts)
        iters_total += o["iters"]
        skips += int(o["skips"])
        statuses[o["status"]] = statuses.get(o["status"], 0) + 1
        if not same(r, o):
            bad.append(dict(n=n, m=m, obj=obj, ls=ls, seed=seed, maxit=maxit, tol=tol, cuda=cuda))
        if (i + 1) % 25 == 0:
            print(f"{i + 1}/{cases} solves, {len(bad)} mismatches, {time.time() - t0:.0f} s", flush=True)
    out = dict(tool="tools/cuda_soak.py", cases=cases, mismatches=len(bad), bad=bad[:20], iterations=iters_total,
               skipped_pairs=skips, statuses=statuses, seconds=round(time.time() - t0, 1),
               build=L.build_info()[0])
    line = json.dumps(out)
    print(line)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fp:
            fp.write(line + "\n")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
