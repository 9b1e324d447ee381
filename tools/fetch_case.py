#!/usr/bin/env python3
"""One tools/fetch_soak.py case in detail: the GPU trajectory against the oracle's canonical one
under LBFGS_DIRECT=1 and =0, the first differing state printed with both values (bits and NaNs).

usage: python tools/fetch_case.py n m objective line_search iterations seed [vector_free]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lbfgs_amd as L  # noqa: E402
import oracle_lib as O  # noqa: E402

n, m, obj, ls, iters, seed = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5]), int(sys.argv[6])
vf = len(sys.argv) > 7 and sys.argv[7] == "1"
x0 = L.x0_uniform(n, seed, -2.0, 2.0)
with np.errstate(all="ignore"):
    o = O.lbfgs(obj, x0, ls, m, iters, 1e-5, mode=O.CANON, vector_free=vf)
print("oracle iterations", o["iters"], "messages", repr(o["messages"][-200:]))
for direct in ("1", "0"):
    os.environ["LBFGS_DIRECT"] = direct
    with L.Context(n, m) as c:
        r = c.minimize(obj, x0, ls, iters, tolerance=1e-5, trace=True, vector_free=vf)
    a, b = np.asarray(r["tr_f"]), np.asarray(o["f"])
    k = min(len(a), len(b))
    diff = [i for i in range(k) if a[i].view(np.uint64) != b[i].view(np.uint64)]
    xb = np.array_equal(np.asarray(r["x"]).view(np.uint64), np.asarray(o["x"]).view(np.uint64))
    xnan = np.array_equal(np.isnan(r["x"]), np.isnan(o["x"]))
    print(f"DIRECT={direct}: gpu iterations {r['iterations']} trace {len(a)} vs {len(b)}; f differs at {diff[:5]};"
          f" x bit-identical {xb}, same NaN positions {xnan}, messages equal {r['messages'] == o['messages']}")
    for i in diff[:2]:
        print(f"   state {i}: gpu {a[i]!r} ({int(a[i].view(np.uint64)):#x}) oracle {b[i]!r} ({int(b[i].view(np.uint64)):#x})")
    if r["messages"] != o["messages"]:
        print("   gpu messages tail", repr(r["messages"][-200:]))
