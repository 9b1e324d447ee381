"""The gap between the two-loop pass k_axpy_dot and the box probe k_probe_stream.

One process, one context at configs[2]'s geometry (n = 1e8, m = 10, Rosenbrock, backtracking; the
history filled), then rounds of lbfgs_stream_probe_variant alternating its six variants - the
probe, the probe with alpha != 0, + the segment reduction stored plainly, + the collect stage 2,
the product's own k_axpy_dot launch with alpha = 0 and != 0 - each 20 launches timed by one event
pair, and between rounds 10 solver steps with per-launch events (the in-iteration k_axpy_dot,
k_axpy2_dot and k_commit); variant 6 is the commit's 4 R + 4 W mix (k_probe_commit) beside k_commit.
Writes one JSON document (argv[1]). Under rocprofv3 the kernel trace separates the variants by
kernel name (k_probe_stream / k_probe_stream2 / k_axpy_dot).

usage: python tools/gap_probe.py out.json [n] [rounds]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

NAMES = ["probe", "probe_alpha", "probe+partial_store", "probe+collect", "k_axpy_dot_alpha0", "k_axpy_dot",
         "commit_mix_4r4w", "probe_on_solver_q", "probe_alpha_on_solver_q", "k_axpy_dot_on_solver_q",
         "probe_scratch_random", "k_axpy_dot_scratch_random", "commit_mix_4r4w_x_random"]
# + 8: on the solver's own q; + 16: the scratch vector filled with a copy of y_0 (random data, not zeros)
VARIANTS = [0, 1, 2, 3, 4, 5, 6, 8, 9, 13, 16, 21, 22]


def main():
    out = sys.argv[1]
    n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10 ** 8
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    m = 10
    L.lib()
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    res = {"n": n, "m": m, "launches_per_sample": 20, "samples": {k: [] for k in NAMES}, "solver_axpy_dot_us": [],
           "solver_commit_us": [], "solver_axpy2_dot_us": []}
    with L.Context(n, m) as c:
        c.init("rosenbrock", x0, "backtracking", tolerance=1e-5)
        del x0
        c.step(m + 4)
        c.sync()
        for r in range(rounds):
            order = list(range(len(VARIANTS))) if r % 2 == 0 else list(range(len(VARIANTS) - 1, -1, -1))
            for v in order:
                p = c.stream_probe(20, variant=VARIANTS[v])
                res["samples"][NAMES[v]].append(round(p["avg_launch_us"], 2))
            c.prof_reset()
            c.prof_enable(True)
            c.step(10)
            c.sync()
            c.prof_enable(False)
            for kind in ("axpy_dot", "axpy2_dot", "commit"):
                a = c.prof_get(kind)
                res[f"solver_{kind}_us"].append(round(a["ms"] / a["launches"] * 1e3, 2))
            print(f"round {r}: " + ", ".join(f"{k} {v[-1]}" for k, v in res["samples"].items())
                  + f", in-solve k_axpy_dot {res['solver_axpy_dot_us'][-1]}", flush=True)
    res["median_us"] = {k: sorted(v)[len(v) // 2] for k, v in res["samples"].items()}
    for kind in ("axpy_dot", "axpy2_dot", "commit"):
        v = sorted(res[f"solver_{kind}_us"])
        res["median_us"][f"solver_k_{kind}"] = v[len(v) // 2]
    res["bytes_per_launch"] = {k: (64.0 if k in ("commit_mix_4r4w", "commit_mix_4r4w_x_random", "solver_k_commit") else 32.0) * n
                               for k in res["median_us"]}
    res["tbps_median"] = {k: round(res["bytes_per_launch"][k] / (v * 1e-6) / 1e12, 3)
                          for k, v in res["median_us"].items()}
    res["build"] = L.build_info()[0]
    res["time"] = time.strftime("%Y-%m-%d %H:%M:%S")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["median_us"]), json.dumps(res["tbps_median"]))


if __name__ == "__main__":
    main()
