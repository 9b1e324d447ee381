#!/usr/bin/env python3
"""Run BASELINE.json's configs on one GPU and write one JSON summary (profiles/<round>/configs.json).

  configs[0]  Rosenbrock n=1e4, m=5, backtracking (the reference's CPU case): GPU it/s, and the
              reference itself (oracle/_ref) on this host's core for the same 1000 iterations
  configs[1]  Rosenbrock n=1e7, m=10: it/s (20 warm-up + 200 timed), unfused per-vector kernels
              (LBFGS_FLAG_UNFUSED, as the config names) and the fused default; plus the unfused
              mode at n=1e8 for the fused/unfused ratio at configs[2]'s size
  configs[2]  Rosenbrock n=1e8, m=10: it/s (20 warm-up + 100 timed) — bench.py's headline
  configs[3]  tridiagonal quadratic (generate_quadratic_*) n=1e8, m=20, Wolfe: time to solution
  configs[4]  Rosenbrock n=1e9, m=10: the 8-GPU problem size, here on ONE GPU (240 GB resident;
              the sharded 8-GPU run is the driver's), 5 warm-up + 10 timed

usage: python tools/bench_configs.py [out.json] [--skip-1e9]
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


def timed_steps(n, m, obj, ls, warm, steps, tol=1e-5, unfused=False, vector_free=False):
    """m untimed iterations fill the history first (as bench.py), so every timed step has h = m;
    h_min / h_max of the timed steps are reported"""
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    with L.Context(n, m) as c:
        c.init(obj, x0, ls, tolerance=tol, unfused=unfused, vector_free=vector_free)
        del x0
        fill = c.step(m)
        c.step(warm)
        c.sync()
        t0 = time.perf_counter()
        r = c.step(steps)
        c.sync()
        dt = time.perf_counter() - t0
    done = steps if r["status"] == "running" else max(r["iterations"] - warm - fill["iterations"], 1)
    return dict(n=n, m=m, objective=obj, line_search=ls,
                kernels="unfused" if unfused else "vector_free" if vector_free else "fused",
                history_fill=fill["iterations"], warmup=warm, steps=done, h_min=r["h_min"], h_max=r["h_max"],
                steady_state=r["h_min"] == m, seconds=dt,
                iters_per_s=done / dt, ms_per_iter=1e3 * dt / done, gbps=r["bytes"] / dt / 1e9,
                status=r["status"], f=r["f"], gnorm=r["gnorm"])


def to_solution(n, m, obj, ls, maxit, tol=1e-5, vector_free=False):
    """time to solution through lbfgs_minimize (x0 upload and x download included), and the same
    solve with x0 already resident (lbfgs_solver_init untimed, then the steps)"""
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    with L.Context(n, m) as c:
        t0 = time.perf_counter()
        r = c.minimize(obj, x0, ls, maxit, tolerance=tol, vector_free=vector_free)
        dt = time.perf_counter() - t0
        c.init(obj, x0, ls, tolerance=tol, vector_free=vector_free)
        c.sync()
        t1 = time.perf_counter()
        r2 = c.step(maxit)
        c.sync()
        dt2 = time.perf_counter() - t1
    return dict(n=n, m=m, objective=obj, line_search=ls, kernels="vector_free" if vector_free else "fused",
                seconds=dt, seconds_x0_resident=dt2, iterations=r["iterations"],
                status=r["status"], f=r["f"], gnorm=r["gnorm"], trials_f=r["trials_f"],
                trials_fg=r["trials_fg"], gbps=r["bytes"] / dt / 1e9,
                same_result_resident=(r2["iterations"] == r["iterations"] and r2["f"] == r["f"]),
                note="seconds: lbfgs_minimize incl. x0 upload and result download; seconds_x0_resident: "
                     "the solve alone (init untimed, no download)")


def cpu_reference(n, m, iters):
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_lbfgs")
    if not os.path.exists(ref):
        return None
    with tempfile.TemporaryDirectory() as tmp:
        pre = os.path.join(tmp, "c")
        subprocess.run([ref, "rosenbrock", str(n), str(m), "backtracking", str(iters), "1e-5", "42", "-2",
                        "2", pre, "0"], check=True, capture_output=True, timeout=900)
        g = np.fromfile(pre + ".g.bin", dtype=np.uint64).reshape(-1, 5)
        t = g[:, 3].copy().view(np.float64)
    return dict(iters_per_s=(len(t) - 1) / (t[-1] - t[0]), seconds=float(t[-1] - t[0]), iterations=len(t) - 1,
                kind="reference (oracle/_ref, 1 core)")


def put(res, key, val):
    res[key] = val
    print(key, json.dumps(val), flush=True)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else None
    res = {}
    # the reference's own case to convergence (17042 iterations, 7.05 s on one core)
    put(res, "config0_rosen_1e4_m5_bt_to_solution", to_solution(10**4, 5, "rosenbrock", "backtracking", 30000))
    put(res, "config0_rosen_1e4_m5_bt_to_solution_vector_free",
        to_solution(10**4, 5, "rosenbrock", "backtracking", 30000, vector_free=True))
    put(res, "config0_rosen_1e4_m5_bt_vector_free", timed_steps(10**4, 5, "rosenbrock", "backtracking", 0, 1000,
                                                                vector_free=True))
    put(res, "config1_rosen_1e7_m10_vector_free", timed_steps(10**7, 10, "rosenbrock", "backtracking", 20, 200,
                                                              vector_free=True))
    put(res, "config2_rosen_1e8_m10_vector_free", timed_steps(10**8, 10, "rosenbrock", "backtracking", 20, 100,
                                                              vector_free=True))
    put(res, "config3_qtri_1e8_m20_wolfe_vector_free", to_solution(10**8, 20, "quad_tridiag", "wolfe", 1000,
                                                                   vector_free=True))
    if "--skip-1e9" not in sys.argv:
        put(res, "config4_rosen_1e9_m10_single_gpu_vector_free",
            timed_steps(10**9, 10, "rosenbrock", "backtracking", 5, 10, vector_free=True))
    res["config0_rosen_1e4_m5_bt"] = dict(gpu=timed_steps(10**4, 5, "rosenbrock", "backtracking", 0, 1000),
                                          cpu=cpu_reference(10**4, 5, 1000))
    print(json.dumps(res["config0_rosen_1e4_m5_bt"]), flush=True)
    res["config1_rosen_1e7_m10_unfused"] = timed_steps(10**7, 10, "rosenbrock", "backtracking", 20, 200,
                                                       unfused=True)
    print(json.dumps(res["config1_rosen_1e7_m10_unfused"]), flush=True)
    res["config1_rosen_1e7_m10_fused"] = timed_steps(10**7, 10, "rosenbrock", "backtracking", 20, 200)
    print(json.dumps(res["config1_rosen_1e7_m10_fused"]), flush=True)
    res["config2_rosen_1e8_m10_unfused"] = timed_steps(10**8, 10, "rosenbrock", "backtracking", 20, 100,
                                                       unfused=True)
    print(json.dumps(res["config2_rosen_1e8_m10_unfused"]), flush=True)
    res["config2_rosen_1e8_m10"] = timed_steps(10**8, 10, "rosenbrock", "backtracking", 20, 100)
    print(json.dumps(res["config2_rosen_1e8_m10"]), flush=True)
    res["config3_qtri_1e8_m20_wolfe"] = to_solution(10**8, 20, "quad_tridiag", "wolfe", 1000)
    print(json.dumps(res["config3_qtri_1e8_m20_wolfe"]), flush=True)
    if "--skip-1e9" not in sys.argv:
        res["config4_rosen_1e9_m10_single_gpu"] = timed_steps(10**9, 10, "rosenbrock", "backtracking", 5, 10)
        print(json.dumps(res["config4_rosen_1e9_m10_single_gpu"]), flush=True)
    if out:
        with open(out, "w") as fp:
            json.dump(res, fp, indent=1)


if __name__ == "__main__":
    main()
