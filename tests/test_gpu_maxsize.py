"""n beyond 2^31 on one MI355X: the reference indexes with `int` (n < 2^31); this path uses
int64 throughout. At n = 2^31 + 2^20 + 3 (17.2 GB per vector, m = 1: 12 vectors, 206 GB resident)
the canonical segments are 268 288 elements long and element offsets pass INT32_MAX inside the
last ~1/8 of every vector. What a 32-bit offset anywhere in the kernels would break, checked
without a CPU oracle run at this size (the restatement would need ~200 GB of host memory):

  * f(x0) against numpy's float64 sum of the reference formula (chunked): within 1e-12 relative,
    so every element was reduced once;
  * the first backtracking step, x1 = x0 + (alpha * -g0) (d = -g0 at k = 0), element for element
    bit for bit at indices around 2^31 and at the end, with g0 from the reference formula
    (benchmark.cpp:70-81, fp-contract off);
  * three iterations on one rank against the same solve sharded over 8 emulated ranks, whose
    local offsets stay below 2^31: trace and final x bit for bit.
"""
import os
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

pytestmark = pytest.mark.gpu

N = 2 ** 31 + 2 ** 20 + 3
M = 1


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def rosen_f(x, chunk=1 << 27):
    """sum of 100 (x[i+1] - x[i]^2)^2 + (1 - x[i])^2, i < n - 1, in float64 chunks"""
    tot = 0.0
    for lo in range(0, len(x) - 1, chunk):
        hi = min(lo + chunk, len(x) - 1)
        a, b = x[lo:hi], x[lo + 1:hi + 1]
        t = b - a * a
        tot += float(np.sum(100.0 * (t * t) + (1.0 - a) * (1.0 - a)))
    return tot


def rosen_grad_at(x, idx):
    """benchmark.cpp:70-81 at the given indices: grad[i] = 200 (x_i - x_{i-1}^2) [i > 0] then
    + (2 (x_i - 1) - (400 x_i)(x_{i+1} - x_i^2)) [i < n - 1], in the reference's order"""
    n = len(x)
    g = np.zeros(len(idx))
    for j, i in enumerate(idx):
        v = 0.0
        if i > 0:
            v = v + 200.0 * (x[i] - x[i - 1] * x[i - 1])
        if i < n - 1:
            v = v + (2.0 * (x[i] - 1.0) - (400.0 * x[i]) * (x[i + 1] - x[i] * x[i]))
        g[j] = v
    return g


@pytest.mark.timeout(1500)
def test_n_beyond_int32():
    x0 = L.x0_uniform(N, 42, -2.0, 2.0)
    # one iteration: the first step, elementwise
    with L.Context(N, M) as c:
        r1 = c.minimize("rosenbrock", x0, "backtracking", 1, trace=True)
    f0 = rosen_f(x0)
    assert abs(r1["tr_f"][0] - f0) <= 1e-12 * abs(f0), (r1["tr_f"][0], f0)
    alpha = r1["tr_alpha"][0]
    idx = np.array([0, 1, 2 ** 31 - 3, 2 ** 31 - 2, 2 ** 31 - 1, 2 ** 31, 2 ** 31 + 1, 2 ** 31 + 2, N - 2, N - 1] +
                   list(np.random.RandomState(5).randint(0, N, 64)), dtype=np.int64)
    g0 = rosen_grad_at(x0, idx)
    want = x0[idx] + alpha * -g0
    assert np.array_equal(bits(r1["x"][idx]), bits(want)), np.nonzero(bits(r1["x"][idx]) != bits(want))
    del r1
    # three iterations: one rank against 8 emulated ranks (each < 2^31 elements)
    with L.Context(N, M) as c:
        ref = c.minimize("rosenbrock", x0, "backtracking", 3, trace=True)
    xs = np.zeros(N)
    grp = L.HostGroup(8)
    ctxs = [L.Context(N, M, rank=r, group=grp) for r in range(8)]
    out, err = [None] * 8, [None] * 8

    def run(r):
        try:
            out[r] = ctxs[r].minimize("rosenbrock", x0, "backtracking", 3, trace=True, out=xs)
        except Exception as e:  # pragma: no cover
            err[r] = e

    th = [threading.Thread(target=run, args=(r,)) for r in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=1200)
    assert not any(err), err
    for r in range(8):
        for key in ("tr_f", "tr_gnorm", "tr_alpha"):
            assert np.array_equal(bits(out[r][key]), bits(ref[key])), (r, key)
        assert np.array_equal(out[r]["tr_c1"], ref["tr_c1"]) and np.array_equal(out[r]["tr_c2"], ref["tr_c2"])
        assert ctxs[r].n_loc < 2 ** 31
    for c in ctxs:
        c.close()
    grp.close()
    assert np.array_equal(bits(xs), bits(ref["x"]))
