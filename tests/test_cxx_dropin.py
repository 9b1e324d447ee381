"""The C++ drop-in layer (include/lbfgs.h, benchmark.h, line_search.h, vector_utils.h,
config.h): a reference-style caller compiles against our headers (CPU) and, on the GPU, gives
the canonical-order results of the oracle."""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cuda-lbfgs_amd")
SRC = os.path.join(ROOT, "tests", "cxx", "dropin_main.cpp")


def _build(tmp):
    lib = os.path.join(PKG, "liblbfgs_hip.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)
    exe = os.path.join(tmp, "dropin_main")
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), SRC, "-o", exe, lib,
                    "-Wl,-rpath," + PKG], check=True, capture_output=True, text=True)
    return exe


def test_reference_style_caller_compiles(tmp_path):
    assert os.path.exists(_build(str(tmp_path)))


def _parse(out):
    d = {}
    for line in out.splitlines():
        if line.startswith("KEY "):
            parts = line.split(" ", 2)
            d[parts[1]] = parts[2]
    return d


def _fx(s):
    return float.fromhex(s)


def _ck(s):
    a, b = s.split()
    return int(a), int(b)


@pytest.mark.gpu
def test_cxx_dropin_on_gpu(tmp_path):
    exe = _build(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    k = _parse(r.stdout)
    n = 2000
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    o = O.lbfgs("rosenbrock", x0, "backtracking", 5, 30, 1e-5, mode=O.CANON)
    assert _ck(k["x_device"]) == O.checksum(o["x"])
    assert _fx(k["xh_minus_x_max"]) <= 1e-8  # host callbacks (sequential f) vs device f
    oq = O.lbfgs("quad_tridiag", x0, "wolfe", 20, 1000, 1e-5, mode=O.CANON)
    assert _ck(k["x_qtri"]) == O.checksum(oq["x"])
    assert _fx(k["dot"]) == O.dot(x0, x0, O.CANON)
    assert _fx(k["norm"]) == np.sqrt(O.dot(x0, x0, O.CANON))
    assert _ck(k["add"]) == O.checksum(x0 + x0)
    assert _ck(k["scal"]) == O.checksum(0.37 * x0)
    assert _ck(k["neg"]) == O.checksum(-x0)
    assert k["size_error"] == "Vectors must be of same size"
    # standalone line searches == the first step the oracle takes from x0 (d = -g)
    for ls in ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"]:
        ol = O.lbfgs("rosenbrock", x0, ls, 5, 1, 1e-5, mode=O.CANON)
        assert _fx(k["ls_" + ls]) == ol["alpha"][0], ls
    assert k["bad_method"] == "Unknown line search method: bogus"
    oc = O.lbfgs("rosenbrock", x0, "wolfe", 5, 20, 1e-5, mode=O.CANON, consts=dict(c2=0.7))
    assert _ck(k["x_cuda"]) == O.checksum(oc["x"])
    ob = O.lbfgs("rosenbrock", x0, "backtracking", 5, 20, 1e-5, mode=O.CANON, consts=dict(c2=0.7))
    assert _ck(k["x_cuda_bt"]) == O.checksum(ob["x"])
    assert _fx(k["C2"]) == 0.9
    assert "Maximum iterations reached" in r.stdout and "Converged!" in r.stdout


@pytest.mark.gpu
def test_cxx_dropin_vector_free_mode(tmp_path):
    """LBFGS_MODE=vector_free: the unchanged reference-style caller runs the vector-free mode for
    its device objectives (bit-exact with the oracle's restatement) and the default mode for its
    host-callback objective."""
    exe = _build(str(tmp_path))
    env = dict(os.environ, LBFGS_MODE="vector_free")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    k = _parse(r.stdout)
    x0 = O.x0_uniform(2000, 42, -2.0, 2.0)
    o = O.lbfgs("rosenbrock", x0, "backtracking", 5, 30, 1e-5, mode=O.CANON, vector_free=True)
    assert _ck(k["x_device"]) == O.checksum(o["x"])
    oq = O.lbfgs("quad_tridiag", x0, "wolfe", 20, 1000, 1e-5, mode=O.CANON, vector_free=True)
    assert _ck(k["x_qtri"]) == O.checksum(oq["x"])
