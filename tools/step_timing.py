"""Wall time of individual solver steps (one iteration per lbfgs_solver_step call, synchronised
after each) against one multi-step call, default and vector-free mode: where does an
iteration's time go beyond its kernels? usage: python tools/step_timing.py [n] [steps] [default|vf|both]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402


def run(n, steps, vf):
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    out = {}
    with L.Context(n, 10) as c:
        c.init("rosenbrock", x0, "backtracking", tolerance=1e-5, vector_free=vf)
        c.step(10)
        w = c.step(12)
        c.sync()
        t0 = time.perf_counter()
        r = c.step(steps)
        c.sync()
        out["multi_ms_per_step"] = (time.perf_counter() - t0) / steps * 1e3
        out["multi_seconds_reported"] = r["seconds"]
        keys = ("commits", "passes", "trials_f", "trials_fg")
        out["multi_counts"] = {k: r[k] - w[k] for k in keys}  # cumulative counters
        if os.environ.get("STEP_TIMING_MULTI_AGAIN"):  # the multi-step call again, later in the run
            t0 = time.perf_counter()
            r = c.step(steps)
            c.sync()
            out["multi2_ms_per_step"] = (time.perf_counter() - t0) / steps * 1e3
            out["multi2_counts"] = {k: r[k] for k in keys}
        single, kern = [], []
        for _ in range(steps):
            t0 = time.perf_counter()
            c.step(1)
            c.sync()
            single.append((time.perf_counter() - t0) * 1e3)
        out["single_ms"] = [round(s, 3) for s in single]
        out["single_median_ms"] = float(np.median(single))
        # the same again with every launch event-timed: per step, the kernels that ran and their times
        for _ in range(steps):
            c.prof_reset()
            c.prof_enable(True)
            t0 = time.perf_counter()
            c.step(1)
            c.sync()
            w = (time.perf_counter() - t0) * 1e3
            c.prof_enable(False)
            ks = {k: c.prof_get(k) for k in L.KERNELS}
            kern.append({"wall": round(w, 3), **{k: [v["launches"], round(v["ms"], 3)] for k, v in ks.items()
                                                 if v["launches"]}})
        out["single_kernels"] = kern
        c.prof_reset()
        c.prof_enable(True)
        t0 = time.perf_counter()
        c.step(steps)
        c.sync()
        wall = (time.perf_counter() - t0) * 1e3
        c.prof_enable(False)
        ks = {k: c.prof_get(k) for k in L.KERNELS}
        out["prof_wall_ms_per_step"] = wall / steps
        out["prof_kernels_ms_per_step"] = {k: round(v["ms"] / steps, 4) for k, v in ks.items() if v["launches"]}
        out["prof_launches_per_step"] = {k: v["launches"] / steps for k, v in ks.items() if v["launches"]}
    return out


if __name__ == "__main__":
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    import json

    mode = sys.argv[3] if len(sys.argv) > 3 else "both"
    for vf in {"default": (False,), "vf": (True,), "both": (False, True)}[mode]:
        print(json.dumps({"n": n, "vector_free": vf, "stagger": os.environ.get("LBFGS_STAGGER"),
                          **run(n, steps, vf)}), flush=True)
