"""Repeated solves in one process, each compared bit for bit with the first solve of its kind: a
wrong result that comes and goes shows up as a count, not as one red test (round 6: two suite
cases failed once each on the contiguous-vector library - a small-n interpolation trajectory and an
emulated 4-rank vector-free f(x0)).

Kinds, interleaved every repetition:
  small   rosen_n4097_m7_interp's problem (n = 4097, m = 7, interpolation, 150 iterations) on one
          long-lived context, as the parity suite runs it
  churn   a context of another size created, solved 5 iterations and destroyed (virtual addresses
          and physical pages of freed vectors come back to later allocations)
  vf4     the emulated 4-rank vector-free solve of test_vector_free_sharded_emulated_bit_exact
          (n = 4,000,003, m = 5, 12 iterations, backtracking, reduce-kernel stage 2), against the
          one-rank vector-free run
The environment (LBFGS_VEC_ALLOC=plain, ...) selects the library's mode; no oracle is used.

usage: python tools/repeat_stress.py out.json [reps] [kinds] [churn_alloc,vf_alloc] [scale]
  (the last argument sets LBFGS_VEC_ALLOC for the churn contexts and for the 4-rank contexts
  separately, e.g. "contiguous,plain": which side's allocations matter; "default,default" leaves
  the environment alone; scale multiplies the churn and 4-rank sizes, e.g. 10 puts them in the
  pool's 64 MiB+ range)
"""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402


def bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def same(a, b):
    keys = ("tr_f", "tr_gnorm", "tr_alpha")
    bad = [k for k in keys if not np.array_equal(bits(a[k]), bits(b[k]))]
    if not np.array_equal(a["tr_c1"], b["tr_c1"]) or not np.array_equal(a["tr_c2"], b["tr_c2"]):
        bad.append("checksums")
    first = None
    if bad:
        k = bad[0] if bad[0] != "checksums" else "tr_f"
        x, y = bits(a[k]), bits(b[k])
        d = np.nonzero(x[:min(len(x), len(y))] != y[:min(len(x), len(y))])[0]
        first = int(d[0]) if len(d) else min(len(x), len(y))
    return bad, first


def alloc_env(mode):
    if mode is None:
        return
    if mode == "default":
        os.environ.pop("LBFGS_VEC_ALLOC", None)
    else:
        os.environ["LBFGS_VEC_ALLOC"] = mode


def vf4(x0, ref, n, m, iters, mode=None):
    grp = L.HostGroup(4)
    alloc_env(mode)
    ctxs = [L.Context(n, m, rank=r, group=grp) for r in range(4)]
    out, err = [None] * 4, [None] * 4

    def run(r):
        try:
            out[r] = ctxs[r].minimize("rosenbrock", x0, "backtracking", iters, trace=True, vector_free=True)
        except Exception as e:  # noqa: BLE001
            err[r] = repr(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    for c in ctxs:
        c.close()
    grp.close()
    if any(err):
        return {"error": err}
    bad = {}
    for r in range(4):
        b, first = same(out[r], ref)
        if b:
            bad[r] = {"keys": b, "first": first, "f0": [float(out[r]["tr_f"][0]), float(ref["tr_f"][0])]}
    return bad


def main():
    out_path = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    kinds = sys.argv[3].split(",") if len(sys.argv) > 3 else ["small", "churn", "vf4"]
    modes = sys.argv[4].split(",") if len(sys.argv) > 4 else [None, None]
    modes = [None if md == "default" else md for md in modes]
    scale = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    env = {k: v for k, v in os.environ.items() if k.startswith("LBFGS_")}
    res = {"env": env, "reps": reps, "kinds": kinds, "alloc_modes": modes, "scale": scale, "fail": {k: 0 for k in kinds}, "runs": {k: 0 for k in kinds},
           "failures": [], "build": L.build_info()[0]}
    t0 = time.time()
    n_s, m_s = 4097, 7
    x_s = L.x0_uniform(n_s, 7, -2.0, 2.0)
    cs = L.Context(n_s, m_s)
    ref_s = cs.minimize("rosenbrock", x_s, "interpolation", 150, tolerance=1e-5, trace=True)
    n_v, m_v, it_v = 4_000_003 * scale, 5, 12
    x_v = L.x0_uniform(n_v, 42, -2.0, 2.0)
    ref_v = None
    if "vf4" in kinds:
        os.environ["LBFGS_TICKET"] = "0"
        with L.Context(n_v, m_v) as c:
            ref_v = c.minimize("rosenbrock", x_v, "backtracking", it_v, trace=True, vector_free=True)
    sizes = [k * scale for k in (100_003, 1_000_003, 65_537, 300_007)]
    for rep in range(reps):
        if "small" in kinds:
            r = cs.minimize("rosenbrock", x_s, "interpolation", 150, tolerance=1e-5, trace=True)
            res["runs"]["small"] += 1
            b, first = same(r, ref_s)
            if b:
                res["fail"]["small"] += 1
                res["failures"].append({"rep": rep, "kind": "small", "keys": b, "first": first})
        if "churn" in kinds:
            n = sizes[rep % len(sizes)]
            x = L.x0_uniform(n, rep, -2.0, 2.0)
            alloc_env(modes[0])
            with L.Context(n, 5) as c:
                a = c.minimize("rosenbrock", x, "wolfe", 5, trace=True)
                b2 = c.minimize("rosenbrock", x, "wolfe", 5, trace=True)
            res["runs"]["churn"] += 1
            b, first = same(a, b2)
            if b:
                res["fail"]["churn"] += 1
                res["failures"].append({"rep": rep, "kind": "churn", "n": n, "keys": b, "first": first})
        if "vf4" in kinds:
            bad = vf4(x_v, ref_v, n_v, m_v, it_v, modes[1])
            res["runs"]["vf4"] += 1
            if bad:
                res["fail"]["vf4"] += 1
                res["failures"].append({"rep": rep, "kind": "vf4", "bad": bad})
        print(f"rep {rep}: {res['fail']} after {time.time() - t0:.0f} s", flush=True)
    cs.close()
    res["seconds"] = round(time.time() - t0, 1)
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps({"fail": res["fail"], "runs": res["runs"]}))


if __name__ == "__main__":
    main()
