#!/usr/bin/env python3
"""Golden fixtures (test infrastructure) for the CUDA path's line searches, the host searches that
parallel-implementation/L-BFGS.cu:293 calls: parallel-implementation/line_search.cpp, which differs
from the sequential file (0.5 floors after backtracking and interpolation, a cached bisection
backtracking-Wolfe search with constants of its own, a safeguarded cubic in the Wolfe search).

For each case (Rosenbrock, x / d / g built as below) and each of the four searches this runs the
reference's own line_search.cpp, compiled here unmodified (oracle/_ref/ref_cuda_ls, oracle/Makefile),
and records the returned step and every f() value and grad() call; the oracle's restatement
(orc_cuda_line_search, ORC_SEQ) must reproduce them bit for bit (tests/test_oracle_cuda_path.py).

  first       x0, g = grad(x0), d = -g                      (the CUDA loop's iteration 0)
  stale       x1 = x0 + 1e-3 d0, g = grad(x0), d = -grad(x1) (every later iteration: the line
                                                             search gets the iteration-0 gradient)
  short       x0, g = grad(x0), d = -1e-3 g                  (the first trial taken)
  ascent      x0, g = grad(x0), d = +g                      (no descent: the floors and minima)
  wide        x0, g = grad(x0), d = -1e-4 g, n = 2           (the Wolfe searches' expansion)

usage: python tests/golden/make_cuda_ls.py   (writes tests/golden/cuda_ls.json and cuda_ls.npz)
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_cuda_ls")
METHODS = ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"]


def cases():
    out = {}
    for n, seed in ((1000, 42), (5, 7), (64, 3)):
        x0 = O.x0_uniform(n, seed, -2.0, 2.0)
        g0 = O.grad("rosenbrock", x0)
        d0 = -g0
        x1 = x0 + 1e-3 * d0
        out[f"first_n{n}"] = (x0, d0, g0)
        out[f"stale_n{n}"] = (x1, -O.grad("rosenbrock", x1), g0)
        out[f"short_n{n}"] = (x0, -1e-3 * g0, g0)
        out[f"ascent_n{n}"] = (x0, g0.copy(), g0)
    x0 = O.x0_uniform(2, 11, -2.0, 2.0)
    g0 = O.grad("rosenbrock", x0)
    out["wide_n2"] = (x0, -1e-4 * g0, g0)
    return out


def run_ref(method, x, d, g, tmp):
    inp = os.path.join(tmp, "in.bin")
    with open(inp, "wb") as fp:
        np.array([len(x)], np.int64).tofile(fp)
        for v in (x, d, g):
            np.ascontiguousarray(v, np.float64).tofile(fp)
    pre = os.path.join(tmp, "out")
    subprocess.run([REF_BIN, method, inp, pre], check=True)
    a = np.fromfile(pre + ".alpha.bin", np.float64)[0]
    f = np.fromfile(pre + ".f.bin", np.float64)
    g = np.fromfile(pre + ".g.bin", np.uint64).reshape(-1, 3)
    return a, f, g


def hexbits(a):
    return [f"{int(u):016x}" for u in np.atleast_1d(np.asarray(a, np.float64)).view(np.uint64)]


def main():
    if not os.path.exists(REF_BIN):
        sys.exit("build the reference first: make -C oracle ref")
    cs = cases()
    meta, arrays = {}, {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, (x, d, g) in cs.items():
            arrays[name + "_x"], arrays[name + "_d"], arrays[name + "_g"] = x, d, g
            for mth in METHODS:
                a, f, gl = run_ref(mth, x, d, g, tmp)
                meta[f"{name}/{mth}"] = dict(alpha=hexbits(a)[0], f_calls=hexbits(f),
                                             grad_calls=[[str(int(v)) for v in row] for row in gl])
                print(f"{name:12s} {mth:18s} alpha {a!r:24} {len(f)} f, {len(gl)} grad calls")
    doc = dict(generator="tests/golden/make_cuda_ls.py: oracle/_ref/ref_cuda_ls (the reference's "
                         "parallel-implementation/line_search.cpp, vector_utils.cpp, functions.cpp)",
               cases=meta)
    with open(os.path.join(HERE, "cuda_ls.json"), "w") as fp:
        json.dump(doc, fp, indent=1)
    np.savez_compressed(os.path.join(HERE, "cuda_ls.npz"), **arrays)


if __name__ == "__main__":
    main()
