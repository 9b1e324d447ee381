"""The oracle's restatement of the CUDA path (LBFGS_CUDA, parallel-implementation/L-BFGS.cu:105-380)
that the product's LBFGS_FLAG_CUDA_COMPAT mode is checked against.

* Its line searches (parallel-implementation/line_search.cpp) are pinned: for 13 inputs x 4 searches
  the restatement (orc_cuda_line_search, left-to-right sums) returns the step, and makes the f and
  grad calls, of the reference's own line_search.cpp compiled here (tests/golden/cuda_ls.json, made
  by tests/golden/make_cuda_ls.py from oracle/_ref/ref_cuda_ls), bit for bit.
* The loop itself runs on cuBLAS in the reference and cannot run here: parity unpinned. What is
  checked is its structure - the messages L-BFGS.cu prints, the convergence test after the step.
"""
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
FIX = json.load(open(os.path.join(HERE, "golden", "cuda_ls.json")))
ARR = np.load(os.path.join(HERE, "golden", "cuda_ls.npz"), allow_pickle=False)
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_cuda_ls")


def f64(hexes):
    return np.array([int(h, 16) for h in hexes], dtype=np.uint64).view(np.float64)


@pytest.mark.parametrize("key", sorted(FIX["cases"]))
def test_cuda_line_search_matches_reference(key):
    name, method = key.split("/")
    x, d, g = ARR[name + "_x"], ARR[name + "_d"], ARR[name + "_g"]
    want = FIX["cases"][key]
    a, flog, glog = O.cuda_line_search(method, x, d, g, mode=O.SEQ)
    assert np.float64(a).view(np.uint64) == f64([want["alpha"]]).view(np.uint64)[0], (a, f64([want["alpha"]]))
    assert np.array_equal(flog.view(np.uint64), f64(want["f_calls"]).view(np.uint64))
    assert np.array_equal(glog, np.array([[int(v) for v in r] for r in want["grad_calls"]], np.uint64).reshape(-1, 3))


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("key", ["stale_n1000/wolfe", "stale_n5/backtracking_wolfe", "ascent_n64/interpolation"])
def test_cuda_line_search_fixture_is_the_live_reference(key):
    """the committed fixture is what the reference's line_search.cpp, compiled here, returns"""
    name, method = key.split("/")
    with tempfile.TemporaryDirectory() as tmp:
        inp = os.path.join(tmp, "in.bin")
        with open(inp, "wb") as fp:
            np.array([len(ARR[name + "_x"])], np.int64).tofile(fp)
            for v in ("_x", "_d", "_g"):
                ARR[name + v].tofile(fp)
        subprocess.run([REF_BIN, method, inp, os.path.join(tmp, "o")], check=True)
        a = np.fromfile(os.path.join(tmp, "o.alpha.bin"), np.float64)
        f = np.fromfile(os.path.join(tmp, "o.f.bin"), np.float64)
    assert a.view(np.uint64)[0] == f64([FIX["cases"][key]["alpha"]]).view(np.uint64)[0]
    assert np.array_equal(f.view(np.uint64), f64(FIX["cases"][key]["f_calls"]).view(np.uint64))


@pytest.mark.parametrize("ls", ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"])
def test_cuda_path_loop_messages(ls):
    """L-BFGS.cu's stdout: "Starting", then per iteration "alpha: ..", "Iteration k: norm_g = ..",
    "Optimum value: .."; the trace entry k is the state printed after step k"""
    n = 64
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    r = O.lbfgs("rosenbrock", x0, ls, 5, 12, 1e-5, mode=O.CANON, cuda=True, consts=O.CONSTANTS_H)
    lines = r["messages"].strip().splitlines()
    assert lines[0] == "Starting"
    body = lines[1:]
    k = 0
    while body and body[0].startswith("alpha: "):
        assert body[1] == f"Iteration {k}: norm_g = {r['gnorm'][k]:g}"
        assert body[2] == f"Optimum value: {r['f'][k]:g}"
        assert float(body[0].split()[1]) == pytest.approx(r["alpha"][k], rel=1e-5)
        body = body[3:]
        k += 1
    assert k == len(r["f"]) == r["iters"]
    if r["status"] == "converged":
        assert body == [f"Convergence achieved at iteration {k - 1}"] and r["gnorm"][-1] <= 1e-5
    elif r["status"] == "max_iter":
        assert body == [] and k == 12
    else:
        assert body == [f"Warning: Line search failed at iteration {k}"]


def test_cuda_path_converges_with_le_after_the_step():
    """convergence is tested after the step with <= (L-BFGS.cu:353): a tolerance equal to the
    reached |g| stops the loop there"""
    n = 32
    x0 = O.x0_uniform(n, 5, -2.0, 2.0)
    r = O.lbfgs("rosenbrock", x0, "backtracking", 4, 6, 0.0, mode=O.CANON, cuda=True, consts=O.CONSTANTS_H)
    assert r["status"] == "max_iter" and len(r["gnorm"]) == 6
    tol = r["gnorm"][2]
    r2 = O.lbfgs("rosenbrock", x0, "backtracking", 4, 6, tol, mode=O.CANON, cuda=True, consts=O.CONSTANTS_H)
    assert r2["status"] == "converged" and r2["iters"] == 3
    assert np.array_equal(r2["f"].view(np.uint64), r["f"][:3].view(np.uint64))


@pytest.mark.parametrize("obj,n,m,ls,maxit,tol,want", [
    ("rosenbrock", 20, 3, "interpolation", 2000, 1e-13, 1332),
    ("rosenbrock", 100, 5, "backtracking", 3000, 1e-12, 3352),
    ("quad_tridiag", 4000, 7, "backtracking_wolfe", 300, 1e-10, 2023)])
def test_cuda_path_skips_pairs(obj, n, m, ls, maxit, tol, want):
    """pairs with s.y <= 1e-10 are skipped in the first loop with the slot's stale alpha / rho
    (L-BFGS.cu:222-223); these cases of tests/test_gpu_cuda_compat.py exercise that many times"""
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    r = O.lbfgs(obj, x0, ls, m, maxit, tol, mode=O.CANON, cuda=True, consts=O.CONSTANTS_H)
    assert r["skips"] == want


@pytest.mark.parametrize("ls", ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"])
def test_cuda_variant_loop_messages(ls):
    """the variant files (orc_opts.cuda = 2) print as L-BFGS.cu does; only L-BFGS-Backtracking.cu
    adds "Warning: Line search resulted in very small step size at iteration k" (:345-348) and
    never reports a failed search"""
    x0 = O.x0_uniform(64, 42, -2.0, 2.0)
    r = O.lbfgs("rosenbrock", x0, ls, 5, 12, 1e-5, mode=O.CANON, cuda=2, consts=O.CONSTANTS_H)
    lines = r["messages"].strip().splitlines()
    assert lines[0] == "Starting"
    body = [ln for ln in lines[1:] if not ln.startswith("Warning: Line search resulted")]
    for k in range(r["iters"]):
        a, it, opt = body[3 * k: 3 * k + 3]
        assert a.startswith("alpha: ") and it == f"Iteration {k}: norm_g = {r['gnorm'][k]:g}"
        assert opt == f"Optimum value: {r['f'][k]:g}"


def test_cuda_variant_backtracking_small_step_warning():
    """L-BFGS-Backtracking.cu's own search (correct-sign Armijo, 0.5 below 1e-10) takes steps in
    [1e-10, 1e-4) on this run and warns for each"""
    x0 = O.x0_uniform(5, 2, -2.0, 2.0)
    r = O.lbfgs("rosenbrock", x0, "backtracking", 2, 3000, 1e-14, mode=O.CANON, cuda=2, consts=O.CONSTANTS_H)
    warn = [ln for ln in r["messages"].splitlines() if ln.startswith("Warning: Line search resulted")]
    small = [a for a in r["alpha"] if a < 1e-4]
    assert warn and len(warn) == len(small)
    assert all(1e-10 <= a for a in r["alpha"])


def test_cuda_variant_differs_from_cuda_path():
    """the variants take the current gradient and their own searches: another trajectory than
    L-BFGS.cu's from the second iteration on"""
    x0 = O.x0_uniform(64, 42, -2.0, 2.0)
    a = O.lbfgs("rosenbrock", x0, "wolfe", 5, 10, 1e-5, mode=O.CANON, cuda=1, consts=O.CONSTANTS_H)
    b = O.lbfgs("rosenbrock", x0, "wolfe", 5, 10, 1e-5, mode=O.CANON, cuda=2, consts=O.CONSTANTS_H)
    assert not np.array_equal(a["f"], b["f"])


def test_cuda_fullsize_fixture_is_consistent():
    """tests/golden/fullsize/cuda_n1e8.json (the GPU's full-size CUDA-mode target): each case's
    printed lines are its own trace, and L-BFGS.cu's loop differs from the variant files'"""
    fx = json.load(open(os.path.join(HERE, "golden", "fullsize", "cuda_n1e8.json")))
    assert (fx["n"], fx["m"], fx["iterations"]) == (10 ** 8, 10, 12)
    for name, c in fx["cases"].items():
        f, gn, al = f64(c["f"]), f64(c["gnorm"]), f64(c["alpha"])
        assert len(f) == len(gn) == len(al) == len(c["c1"]) == c["iterations"] == 12, name
        lines = c["messages"].strip().splitlines()
        assert lines[0] == "Starting"
        body = [ln for ln in lines[1:] if not ln.startswith("Warning: Line search resulted")]
        for k in range(12):
            assert body[3 * k] == f"alpha: {al[k]:g}", (name, k)
            assert body[3 * k + 1] == f"Iteration {k}: norm_g = {gn[k]:g}", (name, k)
            assert body[3 * k + 2] == f"Optimum value: {f[k]:g}", (name, k)
    fs = [tuple(c["f"]) for c in fx["cases"].values()]
    assert len(set(fs)) == len(fs) == 4  # four distinct trajectories
