#!/usr/bin/env python3
"""Full-size parity fixtures (test infrastructure) for the two single-GPU BASELINE configs the
headline and the time-to-solution are quoted on:

  config1_n1e7  configs[1]: Rosenbrock n = 1e7, m = 10, backtracking, 12 iterations (the GPU test
                runs it through the unfused per-vector kernels, the CUDA path's launch shape)
  config2_n1e8  configs[2]: Rosenbrock n = 1e8, m = 10, backtracking, 12 iterations
                (the bench's history fill plus two steps; bench.py's CPU baseline runs the same)
  config3_n1e8  configs[3]: tridiagonal quadratic (benchmark.cpp:16-56) n = 1e8, m = 20, Wolfe,
                tol 1e-5, to convergence

x0 ~ U(-2, 2) from std::mt19937(42) in both. For each config this records

  reference  the reference ITSELF (oracle/_ref/ref_lbfgs: its sequential sources compiled
             unmodified, oracle/Makefile): every f() value, the checksum and |grad| of every
             grad() call, the returned x's checksum, its stdout;
  seq        the oracle's ORC_SEQ restatement, checked here call for call against `reference`
             (so the per-iteration f / |g| of the reference's run are known exactly, also where
             the Wolfe search calls grad() at trial points), as the per-iteration trace;
  canon      the oracle's ORC_CANON order: the product's canonical device order, which the GPU
             must reproduce bit for bit (f, |g|, alpha, x checksums, status, messages);
  horizons   how many leading iterations survive a change of summation order alone
             (tests/golden/make_horizons.py's yardstick, at full size).

Floats are stored as 16-hex-digit IEEE bit patterns, checksums as decimal strings (JSON ints
lose nothing either, but strings keep every reader honest). Writes tests/golden/fullsize/*.json.
Only runnable where /root/reference exists (this container): the reference needs ~15 s per
iteration at n = 1e8 and the m = 20 runs ~40 GB of host memory, so the cases run one at a time.

  config4_n1e9  configs[4]: Rosenbrock n = 1e9, m = 10, backtracking. A whole run does not fit
                this container (~62 GB; every vector is 8 GB), so the fixture holds the first two
                trace entries only: k = 0 (f, |g| and the x checksums at x0) and k = 1 (the first
                step alpha_0 and the state after it), in the canonical order, by `first_steps`
                below (3 vectors resident), which is checked bit for bit against the oracle's
                whole-run restatement at smaller n before it runs at 1e9; and f(x0), |g(x0)| of
                the reference itself (maxit = 0: it evaluates f and grad at x0 and stops).

usage: python tests/golden/make_fullsize.py [config1_n1e7] [config2_n1e8] [config3_n1e8] [config4_n1e9]
       python tests/golden/make_fullsize.py config4_deep OUT.json [iterations]   (a host with ~270 GB)
       python tests/golden/make_fullsize.py merge_config4_deep OUT.json
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_lbfgs")
OUT = os.path.join(HERE, "fullsize")

# name: (objective, n, m, method, maxit, tol, seed, lo, hi, baseline config)
CASES = {
    "config1_n1e7": ("rosenbrock", 10 ** 7, 10, "backtracking", 12, 1e-5, 42, -2.0, 2.0, "configs[1]"),
    "config2_n1e8": ("rosenbrock", 10 ** 8, 10, "backtracking", 12, 1e-5, 42, -2.0, 2.0, "configs[2]"),
    "config3_n1e8": ("quad_tridiag", 10 ** 8, 20, "wolfe", 1000, 1e-5, 42, -2.0, 2.0, "configs[3]"),
}
ALT = {"pair": O.PAIR, "rev": O.REV, "fma": O.FMA}


def hexbits(a):
    return [f"{int(u):016x}" for u in np.asarray(a, np.float64).view(np.uint64)]


def dec(a):
    return [str(int(u)) for u in np.asarray(a, np.uint64)]


def horizon(a, b, tol=1e-10):
    k = min(len(a), len(b))
    r = np.abs(a[:k] - b[:k]) / np.maximum(np.abs(b[:k]), 1e-300)
    bad = np.nonzero(r > tol)[0]
    return int(bad[0]) if len(bad) else int(k)


def run_reference(spec, tmp):
    obj, n, m, method, maxit, tol, seed, lo, hi, _ = spec
    prefix = os.path.join(tmp, "ref")
    t0 = time.time()
    out = subprocess.run([REF_BIN, obj, str(n), str(m), method, str(maxit), repr(tol), str(seed), repr(lo),
                          repr(hi), prefix, "0"], check=True, capture_output=True, text=True)
    f_calls = np.fromfile(prefix + ".f.bin", dtype=np.float64)
    g = np.fromfile(prefix + ".g.bin", dtype=np.uint64).reshape(-1, 5)
    ret = np.fromfile(prefix + ".ret.bin", dtype=np.uint64)[:2]
    return dict(f_calls=f_calls, grad_c=g[:, 0:2].copy(), grad_norm=g[:, 2].copy().view(np.float64),
                grad_nf=g[:, 4].copy(), ret_c=ret, stdout=out.stdout, seconds=time.time() - t0)


def make(name):
    spec = CASES[name]
    obj, n, m, method, maxit, tol, seed, lo, hi, cfg = spec
    with tempfile.TemporaryDirectory() as tmp:
        ref = run_reference(spec, tmp)
    print(f"{name}: reference {len(ref['f_calls'])} f / {len(ref['grad_c'])} grad calls in "
          f"{ref['seconds']:.0f} s: {ref['stdout'].strip()[-60:]!r}", flush=True)
    x0 = O.x0_uniform(n, seed, lo, hi)

    def run(mode, log=False):
        t0 = time.time()
        r = O.lbfgs(obj, x0, method, m, maxit, tol, mode=mode, log_calls=log)
        print(f"  oracle mode {mode}: {len(r['f'])} trace entries, {r['status']}, {time.time() - t0:.0f} s",
              flush=True)
        return r

    seq = run(O.SEQ, log=True)
    # pin: the restatement makes the reference's every call, bit for bit, at this size too
    assert np.array_equal(seq["flog"].view(np.uint64), ref["f_calls"].view(np.uint64)), "f calls differ"
    assert np.array_equal(seq["glog"][:, 0:2], ref["grad_c"]), "grad() arguments differ"
    assert np.array_equal(seq["glog"][:, 2], ref["grad_norm"].view(np.uint64)), "|grad| differs"
    assert O.checksum(seq["x"]) == tuple(int(v) for v in ref["ret_c"]), "returned x differs"
    assert seq["messages"] == ref["stdout"], "stdout differs"
    canon = run(O.CANON)
    hz = {"canon": [horizon(canon["f"], seq["f"]), horizon(canon["gnorm"], seq["gnorm"])]}
    for key, mode in ALT.items():
        r = run(mode)
        hz[key] = [horizon(r["f"], seq["f"]), horizon(r["gnorm"], seq["gnorm"])]
        del r
    hz["ref"] = [min(hz[k][i] for k in ALT) for i in (0, 1)]
    hz["iterations"] = len(seq["f"])

    def trace(r):
        return dict(f=hexbits(r["f"]), gnorm=hexbits(r["gnorm"]), alpha=hexbits(r["alpha"]),
                    c1=dec(r["c1"]), c2=dec(r["c2"]), iterations=r["iters"], status=r["status"],
                    messages=r["messages"], x_checksum=[str(v) for v in O.checksum(r["x"])],
                    nf_total=int(r["nf_total"]), ng_total=int(r["ng_total"]))

    meta = dict(case=name, baseline_config=cfg, objective=obj, n=n, m=m, method=method, maxit=maxit,
                tol=tol, seed=seed, lo=lo, hi=hi,
                reference=dict(f_calls=hexbits(ref["f_calls"]), grad_c1=dec(ref["grad_c"][:, 0]),
                               grad_c2=dec(ref["grad_c"][:, 1]), grad_norm=hexbits(ref["grad_norm"]),
                               grad_nf=[int(v) for v in ref["grad_nf"]],
                               ret_checksum=[str(int(v)) for v in ref["ret_c"]], stdout=ref["stdout"],
                               seconds_in_this_container=round(ref["seconds"], 1)),
                seq=trace(seq), canon=trace(canon), horizons=hz,
                generator=("tests/golden/make_fullsize.py: oracle/_ref/ref_lbfgs (the reference's "
                           "sequential sources) + oracle/lbfgs_oracle.c (ORC_SEQ checked against it "
                           "call for call; ORC_CANON; alternative orders for the horizons)"))
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, name + ".json"), "w") as fp:
        json.dump(meta, fp, indent=1)
    print(f"{name}: horizons {hz}", flush=True)


def first_steps(x0, backtracking=(1.0, 0.5, 1e-8, 1e-4)):
    """Trace entries k = 0 and k = 1 of ORC_CANON Rosenbrock with the backtracking search, with x0,
    g0 and one trial point resident (orc_lbfgs holds ~10 vectors): iteration 0 has no history, so
    d = -g0 (lbfgs.cpp:87-91); the search (line_search.cpp:19-30, oracle ls_backtracking) halves
    alpha while f(x) - f(x + alpha d) < c1 alpha g.d; x1 = x + alpha_0 d (lbfgs.cpp:159).
    x + alpha (-g) is formed as x - (alpha g): negation is exact, so the bits are the same, and
    g.d = -(g.g) bit for bit (the canonical sums are symmetric under negation); both identities
    are asserted against the oracle itself in check_first_steps."""
    a0, beta, tol_a, c1 = backtracking
    f0 = O.f("rosenbrock", x0)
    g = O.grad("rosenbrock", x0)
    gg = O.dot(g, g)
    gd = -gg
    alpha = a0
    t = np.empty_like(x0)
    while True:
        np.multiply(g, alpha, out=t)
        np.subtract(x0, t, out=t)
        ft = O.f("rosenbrock", t)
        if not (f0 - ft < c1 * alpha * gd):
            break
        alpha *= beta
        if alpha < tol_a:
            break
    np.multiply(g, alpha, out=t)
    np.subtract(x0, t, out=t)  # x1
    c0 = O.checksum(x0)
    del g
    f1 = O.f("rosenbrock", t)
    g1 = O.grad("rosenbrock", t)
    gg1 = O.dot(g1, g1)
    del g1
    c1_ = O.checksum(t)
    return dict(f=[f0, f1], gnorm=[float(np.sqrt(gg)), float(np.sqrt(gg1))], alpha=[alpha],
                c1=[c0[0], c1_[0]], c2=[c0[1], c1_[1]])


def check_first_steps(n, m=10):
    """first_steps against the oracle's whole run (ORC_CANON, 1 iteration), bit for bit"""
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    r = O.lbfgs("rosenbrock", x0, "backtracking", m, 1, 1e-5, mode=O.CANON)
    q = first_steps(x0)
    g = O.grad("rosenbrock", x0)
    assert np.float64(O.dot(g, -g)).view(np.uint64) == np.float64(-O.dot(g, g)).view(np.uint64)
    for k in range(2):
        assert np.float64(q["f"][k]).view(np.uint64) == r["f"][k:k + 1].view(np.uint64)[0], ("f", n, k)
        assert np.float64(q["gnorm"][k]).view(np.uint64) == r["gnorm"][k:k + 1].view(np.uint64)[0], ("g", n, k)
        assert q["c1"][k] == int(r["c1"][k]) and q["c2"][k] == int(r["c2"][k]), ("x", n, k)
    assert np.float64(q["alpha"][0]).view(np.uint64) == r["alpha"][0:1].view(np.uint64)[0], ("alpha", n)
    print(f"  first_steps == orc_lbfgs at n={n}: alpha_0 = {q['alpha'][0]!r}", flush=True)


def make_config4():
    """tests/golden/fullsize/config4_n1e9.json (see the module docstring)"""
    n, m, name = 10 ** 9, 10, "config4_n1e9"
    for small in (4_000_003, 8192 * 8192 + 1):
        check_first_steps(small, m)
    with tempfile.TemporaryDirectory() as tmp:
        ref = run_reference(("rosenbrock", n, m, "backtracking", 0, 1e-5, 42, -2.0, 2.0, "configs[4]"), tmp)
    print(f"{name}: reference f(x0), grad(x0) in {ref['seconds']:.0f} s", flush=True)
    t0 = time.time()
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    q = first_steps(x0)
    del x0
    print(f"{name}: canonical k = 0, 1 in {time.time() - t0:.0f} s: alpha_0 = {q['alpha'][0]!r}", flush=True)
    meta = dict(case=name, baseline_config="configs[4]", objective="rosenbrock", n=n, m=m, method="backtracking",
                maxit=1, tol=1e-5, seed=42, lo=-2.0, hi=2.0,
                reference=dict(f_calls=hexbits(ref["f_calls"]), grad_c1=dec(ref["grad_c"][:, 0]),
                               grad_c2=dec(ref["grad_c"][:, 1]), grad_norm=hexbits(ref["grad_norm"]),
                               stdout=ref["stdout"], seconds_in_this_container=round(ref["seconds"], 1),
                               note="maxit = 0: f and grad at x0 only (lbfgs.cpp:29-30)"),
                canon=dict(f=hexbits(q["f"]), gnorm=hexbits(q["gnorm"]), alpha=hexbits(q["alpha"]),
                           c1=[str(v) for v in q["c1"]], c2=[str(v) for v in q["c2"]], entries=2),
                generator=("tests/golden/make_fullsize.py make_config4: oracle/_ref/ref_lbfgs (the "
                           "reference's sequential sources) at maxit 0, and first_steps (ORC_CANON, "
                           "checked against orc_lbfgs at n = 4000003 and 8192^2 + 1)"))
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, name + ".json"), "w") as fp:
        json.dump(meta, fp, indent=1)


def make_config4_deep(out_path, iters=13):
    """configs[4]'s whole canonical run (ORC_CANON, the oracle's orc_lbfgs at n = 1e9, m = 10,
    backtracking, `iters` iterations: every trace entry, the history filled to h = m = 10 and three
    steps with the ring full). ~265 GB of host memory (30 resident vectors of 8 GB, the terms buffer,
    x0 and x): more than this container has, so it runs on a GPU box's host (tools/gpu_r06.sh
    config4deep, OpenMP over the oracle's vector loops) and writes `out_path`; `merge_config4_deep`
    adds it to tests/golden/fullsize/config4_n1e9.json as "canon_deep". Needs no reference build."""
    n, m = 10 ** 9, 10
    t0 = time.time()
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    print(f"config4 deep: x0 in {time.time() - t0:.0f} s", flush=True)
    t1 = time.time()
    r = O.lbfgs("rosenbrock", x0, "backtracking", m, iters, 1e-5, mode=O.CANON)
    del x0
    xc = [str(v) for v in O.checksum(r["x"])]
    deep = dict(f=hexbits(r["f"]), gnorm=hexbits(r["gnorm"]), alpha=hexbits(r["alpha"]), c1=dec(r["c1"]),
                c2=dec(r["c2"]), entries=len(r["f"]), iterations=r["iters"], status=r["status"],
                messages=r["messages"], x_checksum=xc, maxit=iters,
                seconds=round(time.time() - t1, 1), threads=os.environ.get("OMP_NUM_THREADS"),
                generator=("tests/golden/make_fullsize.py make_config4_deep: oracle/lbfgs_oracle.c orc_lbfgs "
                           "(ORC_CANON) at n = 1e9, m = 10, run on a GPU box's host"))
    with open(out_path, "w") as fp:
        json.dump(deep, fp, indent=1)
    print(f"config4 deep: {deep['entries']} trace entries in {deep['seconds']} s, {r['status']}", flush=True)


def merge_config4_deep(deep_path):
    """the deep run (make_config4_deep) into the fixture; its first two entries must be the
    fixture's first_steps entries bit for bit"""
    fx_path = os.path.join(OUT, "config4_n1e9.json")
    fx = json.load(open(fx_path))
    deep = json.load(open(deep_path))
    can = fx["canon"]
    for key in ("f", "gnorm", "c1", "c2"):
        assert deep[key][:2] == can[key], key
    assert deep["alpha"][:1] == can["alpha"]
    fx["canon_deep"] = deep
    with open(fx_path, "w") as fp:
        json.dump(fx, fp, indent=1)
    print(f"merged: {deep['entries']} entries", flush=True)


def main(argv):
    if argv[:1] == ["config4_deep"]:
        make_config4_deep(argv[1], int(argv[2]) if len(argv) > 2 else 13)
        return
    if argv[:1] == ["merge_config4_deep"]:
        merge_config4_deep(argv[1])
        return
    if not os.path.exists(REF_BIN):
        sys.exit("build the reference first: make -C oracle ref")
    for nm in argv or list(CASES) + ["config4_n1e9"]:
        if nm == "config4_n1e9":
            make_config4()
        else:
            make(nm)


if __name__ == "__main__":
    main(sys.argv[1:])
