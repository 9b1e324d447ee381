#!/usr/bin/env python3
"""The reference's benchmark protocol (sequential-implementation/main.cpp:24-55, benchmark.cpp:83-105;
paper p.4 "five independent runs"): seeds 42, 365, 12345, 777777, 10000, each a full LBFGS call
timed end to end, averaged. Two workloads:
  main_cpp   : main.cpp as shipped — separable quadratic, n = 1e4, x0 ~ U(-1000, 1000), m = 10,
               tol 1e-8, max 15000 iterations, backtracking
  rosenbrock : Rosenbrock n = 1e4, x0 ~ U(-2, 2), m = 5, tol 1e-5, max 30000, backtracking (the
               BASELINE configs[0] case, to convergence)
GPU: one MI355X, default and vector-free modes, time of minimize() (x0 upload and result download
included, as the reference's timer includes its copies). CPU: the reference's own sequential code
(oracle/_ref/ref_lbfgs), first to last grad() call on one core.

usage: python tools/seeds5.py [out.json]
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

SEEDS = [42, 365, 12345, 777777, 10000]
CASES = {
    "main_cpp": dict(obj="quad_sep", n=10_000, lo=-1000.0, hi=1000.0, m=10, tol=1e-8, maxit=15000),
    "rosenbrock": dict(obj="rosenbrock", n=10_000, lo=-2.0, hi=2.0, m=5, tol=1e-5, maxit=30000),
}


def gpu(case, seed, vector_free):
    x0 = L.x0_uniform(case["n"], seed, case["lo"], case["hi"])
    with L.Context(case["n"], case["m"]) as c:
        t0 = time.perf_counter()
        r = c.minimize(case["obj"], x0, "backtracking", case["maxit"], tolerance=case["tol"], vector_free=vector_free)
        dt = time.perf_counter() - t0
    return dict(seconds=dt, iterations=r["iterations"], status=r["status"], f=r["f"])


def cpu(case, seed):
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_lbfgs")
    with tempfile.TemporaryDirectory() as tmp:
        pre = os.path.join(tmp, "c")
        cmd = [ref, case["obj"], str(case["n"]), str(case["m"]), "backtracking", str(case["maxit"]), repr(case["tol"]),
               str(seed), repr(case["lo"]), repr(case["hi"]), pre, "0"]
        try:
            subprocess.run(["taskset", "-c", "0"] + cmd, check=True, capture_output=True, timeout=1200)
        except (FileNotFoundError, subprocess.CalledProcessError):
            subprocess.run(cmd, check=True, capture_output=True, timeout=1200)
        g = np.fromfile(pre + ".g.bin", dtype=np.uint64).reshape(-1, 5)
        t = g[:, 3].copy().view(np.float64)
    return dict(seconds=float(t[-1] - t[0]), grad_calls=len(t))


def main():
    out = {}
    for name, case in CASES.items():
        gpu(case, 1, False)  # untimed warm-up: the first launch of each kernel loads its code object
        gpu(case, 1, True)
        runs = {"gpu_default": [], "gpu_vector_free": [], "cpu_reference": []}
        for seed in SEEDS:
            runs["gpu_default"].append(gpu(case, seed, False))
            runs["gpu_vector_free"].append(gpu(case, seed, True))
            runs["cpu_reference"].append(cpu(case, seed))
            print(name, seed, {k: round(v[-1]["seconds"], 4) for k, v in runs.items()},
                  runs["gpu_default"][-1]["iterations"], runs["gpu_vector_free"][-1]["iterations"], flush=True)
        mean = {k: float(np.mean([r["seconds"] for r in v])) for k, v in runs.items()}
        out[name] = dict(case=case, seeds=SEEDS, runs=runs, mean_seconds=mean,
                         speedup_default=mean["cpu_reference"] / mean["gpu_default"],
                         speedup_vector_free=mean["cpu_reference"] / mean["gpu_vector_free"])
        print(name, json.dumps({k: round(v, 4) for k, v in mean.items()}),
              "speedups", round(out[name]["speedup_default"], 2), round(out[name]["speedup_vector_free"], 2), flush=True)
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
