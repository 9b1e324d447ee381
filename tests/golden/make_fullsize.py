#!/usr/bin/env python3
"""Full-size parity fixtures (test infrastructure) for the two single-GPU BASELINE configs the
headline and the time-to-solution are quoted on:

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

usage: python tests/golden/make_fullsize.py [config2_n1e8] [config3_n1e8]
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


def main(argv):
    if not os.path.exists(REF_BIN):
        sys.exit("build the reference first: make -C oracle ref")
    for nm in argv or list(CASES):
        make(nm)


if __name__ == "__main__":
    main(sys.argv[1:])
