#!/usr/bin/env python3
"""Extract the dense quadratic known-answer data of the reference's
sequential-implementation/matrices.h (mat<n>, linear<n>, minimum<n> for n in 2..500) into
tests/golden/matrices.npz. The header's problems are f(x) = x^T A x + b^T x with
2 A x* + b = 0; its literals carry an `f` suffix, so every value is the float32 rounding of the
printed decimal, kept as such here (float64 arrays holding float32 values).

Data only (numbers, not source). Run in the container that has /root/reference:
    python tests/golden/make_matrices.py
"""
import os
import re

import numpy as np

SRC = "/root/reference/sequential-implementation/matrices.h"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "matrices.npz")


def main():
    text = open(SRC).read()
    blocks = re.findall(r"(mat|linear|minimum)(\d+)(?:\[\d+\])?\s*=\s*\{([^}]*)\}", text)
    arrs = {}
    for kind, n, body in blocks:
        vals = [float(v.rstrip("f")) for v in re.findall(r"[-+]?\d+\.\d*(?:[eE][-+]?\d+)?f?", body)]
        a = np.asarray(vals, dtype=np.float32).astype(np.float64)
        n = int(n)
        if kind == "mat":
            a = a.reshape(n, n)
        assert a.size == (n * n if kind == "mat" else n), (kind, n, a.size)
        arrs[f"{kind}{n}"] = a
    np.savez_compressed(OUT, **arrs)
    print(OUT, sorted(arrs))


if __name__ == "__main__":
    main()
