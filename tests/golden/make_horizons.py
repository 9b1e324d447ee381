#!/usr/bin/env python3
"""Horizon fixture (test infrastructure): for every golden case, how many leading iterations of
the reference's own run (the oracle's ORC_SEQ order, bit-exact with the reference per
tests/test_oracle_golden.py) survive a change of summation order alone, f and |g| within 1e-10
relative:
  canon  the product's canonical device order (the GPU is bit-exact with it)
  pair   recursive pairwise sums (8-term sequential leaves)
  rev    right-to-left sums
  fma    left-to-right with the products fused (the reference built with FMA contraction)
  ref    the smallest horizon over pair / rev / fma: how far the reference agrees with itself
         under an equally valid order - the yardstick the GPU's horizon is held to.
Writes tests/golden/horizons.json.  usage: python tests/golden/make_horizons.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

ALT = {"pair": O.PAIR, "rev": O.REV, "fma": O.FMA}


def horizon(a, b, tol=1e-10):
    k = min(len(a), len(b))
    r = np.abs(a[:k] - b[:k]) / np.maximum(np.abs(b[:k]), 1e-300)
    bad = np.nonzero(r > tol)[0]
    return int(bad[0]) if len(bad) else int(k)


def case_horizons(name):
    meta, _ = O.load_golden(name)
    x0 = O.x0_uniform(meta["n"], meta["seed"], meta["lo"], meta["hi"])

    def run(mode):
        return O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"], mode=mode)

    seq = run(O.SEQ)
    out = {}
    for key, mode in [("canon", O.CANON)] + list(ALT.items()):
        r = run(mode)
        out[key] = [horizon(r["f"], seq["f"]), horizon(r["gnorm"], seq["gnorm"])]
    out["ref"] = [min(out[k][i] for k in ALT) for i in (0, 1)]
    out["iterations"] = len(seq["f"])
    return out


def main():
    res = {name: case_horizons(name) for name in O.golden_cases()}
    with open(os.path.join(HERE, "horizons.json"), "w") as fp:
        json.dump(res, fp, indent=1, sort_keys=True)
    for k, v in res.items():
        print(k, v)


if __name__ == "__main__":
    main()
