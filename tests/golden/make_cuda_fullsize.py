#!/usr/bin/env python3
"""Full-size fixtures (test infrastructure) for the CUDA-path mode (LBFGS_FLAG_CUDA_COMPAT, DESIGN.md
§4.5) at configs[2]'s size: Rosenbrock n = 1e8, m = 10, x0 ~ U(-2, 2) from std::mt19937(42),
12 iterations (the history fills at k = 10), in the oracle's ORC_CANON order, which the GPU must
reproduce bit for bit:

  cuda_bt         orc_opts.cuda = 1: L-BFGS.cu's loop with line_search.cpp's backtracking search
                  (the iteration-0 gradient in every search, the 0.5 floor)
  cuda_btw        orc_opts.cuda = 1: the same loop with line_search.cpp's cached bisection
                  backtracking-Wolfe search (C2 = 0.9 of its own)
  cuda_wolfe      orc_opts.cuda = 1: the same loop with line_search.cpp's Wolfe search (the
                  safeguarded cubic, the iteration-0 gradient)
  variant_wolfe   orc_opts.cuda = 2: L-BFGS-Wolfe.cu's loop and inline search (the current
                  gradient, f(x_host) of the last transferred trial point, f_lo from f(x0))

(L-BFGS-Backtracking.cu's, L-BFGS-Interpolation.cu's and L-BFGS-Backtracking_Wolfe.cu's own searches
accept the same steps as cuda_bt on this run, so they add no trajectory of their own here; the four
trajectories above all differ.)

Each case stores the trace (f, |g|, alpha as 16-hex-digit IEEE bit patterns, the x checksums as
decimal strings), status, iteration count and messages. The restatement's line searches are pinned
to the reference's line_search.cpp (tests/golden/cuda_ls.json); the loop is parity unpinned.
The oracle holds ~30 vectors of 800 MB per case; the cases run one at a time (~3-4 min each).

usage: python tests/golden/make_cuda_fullsize.py [case ...]   (writes tests/golden/fullsize/cuda_n1e8.json;
       named cases are recomputed and merged into the existing file, cases no longer listed dropped)
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

OUT = os.path.join(HERE, "fullsize", "cuda_n1e8.json")
N, M, ITERS, TOL = 10 ** 8, 10, 12, 1e-5
CASES = {"cuda_bt": (1, "backtracking"), "cuda_btw": (1, "backtracking_wolfe"), "cuda_wolfe": (1, "wolfe"),
         "variant_wolfe": (2, "wolfe")}


def hexbits(a):
    return [f"{int(u):016x}" for u in np.ascontiguousarray(a, np.float64).view(np.uint64)]


def main():
    x0 = O.x0_uniform(N, 42, -2.0, 2.0)
    doc = dict(n=N, m=M, iterations=ITERS, tol=TOL, objective="rosenbrock", seed=42,
               generator="tests/golden/make_cuda_fullsize.py (oracle ORC_CANON, constants.h profile)", cases={})
    names = sys.argv[1:] or list(CASES)
    if sys.argv[1:] and os.path.exists(OUT):
        old = json.load(open(OUT))
        doc["cases"] = {k: v for k, v in old["cases"].items() if k in CASES}
    for name in names:
        cuda, ls = CASES[name]
        t = time.time()
        r = O.lbfgs("rosenbrock", x0, ls, M, ITERS, TOL, mode=O.CANON, cuda=cuda, consts=O.CONSTANTS_H)
        doc["cases"][name] = dict(cuda=cuda, method=ls, status=r["status"], iterations=int(r["iters"]),
                                  f=hexbits(r["f"]), gnorm=hexbits(r["gnorm"]), alpha=hexbits(r["alpha"]),
                                  c1=[str(int(v)) for v in r["c1"]], c2=[str(int(v)) for v in r["c2"]],
                                  messages=r["messages"])
        print(f"{name}: {r['status']} after {r['iters']} iterations, f {r['f'][-1]:.6g}, "
              f"{time.time() - t:.0f} s", flush=True)
        del r
    doc["cases"] = {k: doc["cases"][k] for k in CASES if k in doc["cases"]}
    with open(OUT, "w") as fp:
        json.dump(doc, fp, indent=1)


if __name__ == "__main__":
    main()
