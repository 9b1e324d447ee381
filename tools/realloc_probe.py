#!/usr/bin/env python3
"""Does a large solve run slower when its vectors are allocated after an earlier large solve's were
freed in the same process (DESIGN.md §5, configs[4] on one card)? Solves of n = 1e9 / 1e8,
Rosenbrock, m = 10, backtracking, back to back in ONE process: each creates its context (all vectors
allocated), fills the history (m iterations), takes 2 warm-up steps and times 5, then frees
everything. Prints one line per solve and one JSON summary.

usage: python tools/realloc_probe.py [out.json]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

L.lib()
M = 10
x9 = L.x0_uniform(10 ** 9, 42, -2.0, 2.0)
rows = []
for n in (10 ** 9, 10 ** 9, 10 ** 8, 10 ** 9):
    t_alloc = time.perf_counter()
    with L.Context(n, M) as c:
        c.init("rosenbrock", x9[:n], "backtracking")
        t_alloc = time.perf_counter() - t_alloc
        c.step(M)
        c.step(2)
        c.sync()
        t = time.perf_counter()
        r = c.step(5)
        c.sync()
        dt = (time.perf_counter() - t) / 5
    row = dict(n=n, ms_per_it=round(dt * 1e3, 2), it_per_s=round(1 / dt, 3), gbps=round(r["bytes"] / 5 / dt / 1e9, 1),
               setup_s=round(t_alloc, 2), h_min=r.get("h_min"), h_max=r.get("h_max"))
    rows.append(row)
    print(row, flush=True)
out = dict(tool="tools/realloc_probe.py", rows=rows, build=L.build_info()[0])
print(json.dumps(out))
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as fp:
        json.dump(out, fp)
