#!/usr/bin/env python3
"""The reference's published comparison (cuda_lbfgs.pdf p.5 Table I): Rosenbrock
n=1e4, one row per line search, GPU against the sequential CPU code. Here the GPU is one MI355X
(default and vector-free modes), the CPU is the reference's own sequential sources compiled
unmodified (oracle/_ref/ref_lbfgs) on one core of the same box.

Each cell is the time of the same 1000 iterations (m = 5, x0 from std::mt19937(42), tol 1e-5 —
none of the four converges within 1000 iterations at this n, so every run takes exactly 1000
steps), best of 3 runs on each side (the box's shared host cores make single CPU timings vary by
±20 %), and the table reports the speedups.

usage: python tools/paper_table.py [out.json]
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

L.lib()
import numpy as np  # noqa: E402

N, M, ITERS = 10_000, 5, 1000
PUBLISHED = {"backtracking": 1.12, "interpolation": 1.11, "backtracking_wolfe": 3.55, "wolfe": 1.79}


def gpu(ls, vector_free):
    x0 = L.x0_uniform(N, 42, -2.0, 2.0)
    with L.Context(N, M) as c:
        c.init("rosenbrock", x0, ls, tolerance=1e-5, vector_free=vector_free)
        c.sync()
        t0 = time.perf_counter()
        r = c.step(ITERS)
        c.sync()
        dt = time.perf_counter() - t0
    return dict(seconds=dt, iterations=r["iterations"], status=r["status"], f=r["f"])


def cpu(ls):
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_lbfgs")
    with tempfile.TemporaryDirectory() as tmp:
        pre = os.path.join(tmp, "c")
        cmd = [ref, "rosenbrock", str(N), str(M), ls, str(ITERS), "1e-5", "42", "-2", "2", pre, "0"]
        try:
            subprocess.run(["taskset", "-c", "0"] + cmd, check=True, capture_output=True, timeout=900)
        except (FileNotFoundError, subprocess.CalledProcessError):
            subprocess.run(cmd, check=True, capture_output=True, timeout=900)
        g = np.fromfile(pre + ".g.bin", dtype=np.uint64).reshape(-1, 5)
        t = g[:, 3].copy().view(np.float64)
        nf = g[:, 4].copy().view(np.int64) if g.shape[1] > 4 else None
    # grad() timestamps: the first is the initial gradient, the rest one per accepted step
    # (backtracking / interpolation) or per f+grad trial (Wolfe variants): time from the first
    # to the last call over the iterations it covers
    return dict(seconds=float(t[-1] - t[0]), grad_calls=len(t))


def main():
    rows = {}
    for ls in ["backtracking", "interpolation", "backtracking_wolfe", "wolfe"]:
        best = lambda f: min((f() for _ in range(3)), key=lambda r: r["seconds"])  # noqa: E731
        gd = best(lambda: gpu(ls, False))
        gv = best(lambda: gpu(ls, True))
        c = best(lambda: cpu(ls))
        rows[ls] = dict(published_speedup_T4=PUBLISHED[ls], cpu_reference=c, gpu_default=gd, gpu_vector_free=gv,
                        speedup_default=c["seconds"] / gd["seconds"], speedup_vector_free=c["seconds"] / gv["seconds"])
        print(ls, json.dumps(rows[ls]), flush=True)
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
