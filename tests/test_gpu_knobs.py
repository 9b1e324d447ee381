"""Every A/B knob of the device layer and the driver, alone and in the combinations that share
state, against the default path: identical trajectories, bit for bit (the canonical order does
not depend on how a pass is launched, where its stage 2 runs, which cache policy it streams with
or in which direction it walks). Round 3 found in-launch tickets on one rank releasing the host
after the first of several groups (LBFGS_TICKET=1 at mid n: NaN trajectories); this matrix is the
net for that class of interaction bug. Sizes cover each stage-2 regime of the default path:
cooperative (<= 256 segments), deferred (<= 1024), reduce kernel (> 1024, 512- and 640-element
segments).

The variants are the shipped forms (DESIGN.md §3 lists each stage-2 form's forward-progress
assumption and the test here that would catch a violation); LBFGS_PERSIST=1 is compiled out of the
shipped library (LBK_PERSIST_ITER) and must leave the default path untouched."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

pytestmark = pytest.mark.gpu

# every switch of the shipped library that changes how a one-rank solve runs;
# the sharded ones (LBFGS_XGMI_FOLD, LBFGS_CU_PARTITION, the time-outs of the exchanges) are
# covered by tests/test_gpu_xgmi.py and tests/test_gpu_rccl.py, the transfer paths (LBFGS_XFER)
# by tests/test_gpu_xfer.py. A/B forms measured slower are compiled into variant builds only
# (tools/build_variant.sh: LBK_PERSIST_ITER, LBK_PERSIST_STRIDE,
# LBK_PERSIST_ALT, LBK_PERSIST_LDS; the q/r ping-pong was removed).
KNOBS = ["LBFGS_TICKET", "LBFGS_DEFER", "LBFGS_REV", "LBFGS_NT", "LBFGS_DIRECT", "LBFGS_COOP",
         "LBFGS_PERSIST", "LBFGS_SPEC", "LBFGS_BATCH", "LBFGS_PERSIST_WG", "LBFGS_COLLECT",
         "LBFGS_COLLECT_TIMEOUT", "LBFGS_DEV_SEARCH", "LBFGS_DEV_WOLFE", "LBFGS_SEARCH_TIMEOUT", "LBFGS_WAIT"]

VARIANTS = {
    "ticket1": {"LBFGS_TICKET": "1"},
    "ticket0": {"LBFGS_TICKET": "0"},
    "defer0": {"LBFGS_DEFER": "0"},
    "defer_all": {"LBFGS_DEFER": "8192", "LBFGS_TICKET": "0"},
    "rev0": {"LBFGS_REV": "0"},
    "nt0": {"LBFGS_NT": "0"},
    "nt1": {"LBFGS_NT": "1"},
    "direct0": {"LBFGS_DIRECT": "0"},
    "coop0": {"LBFGS_COOP": "0"},
    "persist1_not_shipped": {"LBFGS_PERSIST": "1"},  # compiled out of the library: the default path runs
    "persist2": {"LBFGS_PERSIST": "2"},
    "persist2_wg1": {"LBFGS_PERSIST": "2", "LBFGS_PERSIST_WG": "1"},
    "persist2_nt1": {"LBFGS_PERSIST": "2", "LBFGS_NT": "1"},
    "collect1": {"LBFGS_COLLECT": "1"},
    "collect1_rev0_nt1": {"LBFGS_COLLECT": "1", "LBFGS_REV": "0", "LBFGS_NT": "1"},
    "collect1_defer0_batch0": {"LBFGS_COLLECT": "1", "LBFGS_DEFER": "0", "LBFGS_BATCH": "0"},
    "spec0": {"LBFGS_SPEC": "0"},
    "batch0": {"LBFGS_BATCH": "0"},
    "ticket1_direct0": {"LBFGS_TICKET": "1", "LBFGS_DIRECT": "0"},
    "ticket1_rev0_nt0": {"LBFGS_TICKET": "1", "LBFGS_REV": "0", "LBFGS_NT": "0"},
    "persist2_coop0_nt1": {"LBFGS_PERSIST": "2", "LBFGS_COOP": "0", "LBFGS_NT": "1"},
    "collect_timeout": {"LBFGS_COLLECT": "1", "LBFGS_COLLECT_TIMEOUT": "30"},
    "defer_all_rev0": {"LBFGS_DEFER": "8192", "LBFGS_TICKET": "0", "LBFGS_REV": "0"},
    "coop0_spec0_batch0": {"LBFGS_COOP": "0", "LBFGS_SPEC": "0", "LBFGS_BATCH": "0"},
    "devsearch0": {"LBFGS_DEV_SEARCH": "0"},
    "devsearch0_spec0": {"LBFGS_DEV_SEARCH": "0", "LBFGS_SPEC": "0"},
    "devwolfe0_round4_name": {"LBFGS_DEV_WOLFE": "0"},
    "search_timeout0": {"LBFGS_SEARCH_TIMEOUT": "0"},  # the device search gives up, the host loop redoes it
    "wait_spin": {"LBFGS_WAIT": "spin"},  # host waits spin throughout (no sleep phase)
}

CASES = [  # n, m, objective, line search, iterations
    (100_003, 5, "rosenbrock", "backtracking", 25),       # 196 segments: cooperative iteration
    (60_001, 5, "rosenbrock", "wolfe", 40),               # 118 segments: the device-resident line searches
    (30_001, 6, "quad_tridiag", "interpolation", 40),      # 59 segments: ... the interpolation search
    (20_001, 4, "rosenbrock", "backtracking_wolfe", 60),   # 40 segments: ... backtracking-Wolfe
    (700_001, 7, "quad_tridiag", "wolfe", 12),             # 342 segments of 2048: deferred stage 2
    (3_000_017, 5, "rosenbrock", "interpolation", 14),     # 5860 segments of 512: reduce kernel
    (5_000_000, 10, "rosenbrock", "backtracking", 14),     # 7813 segments of 640, h = m reached
]

_default = {}


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def solve(monkeypatch, case, env):
    n, m, obj, ls, iters = case
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    x0 = L.x0_uniform(n, 29, -2.0, 2.0)
    with L.Context(n, m) as c:  # knobs are read at creation and per solve
        return c.minimize(obj, x0, ls, iters, trace=True)


@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c[0]}_{c[2]}_{c[3]}")
def test_knob_bit_identical(monkeypatch, case, variant):
    if case not in _default:
        _default[case] = solve(monkeypatch, case, {})
    a = _default[case]
    b = solve(monkeypatch, case, VARIANTS[variant])
    assert np.all(np.isfinite(b["tr_f"])) and np.all(np.isfinite(b["tr_gnorm"]))
    for key in ("tr_f", "tr_gnorm", "x"):
        assert np.array_equal(bits(a[key]), bits(b[key])), key
    ta, tb = a["tr_alpha"], b["tr_alpha"]
    assert np.array_equal(np.isnan(ta), np.isnan(tb)) and np.array_equal(ta[~np.isnan(ta)], tb[~np.isnan(tb)])
    assert np.array_equal(a["tr_c1"], b["tr_c1"]) and np.array_equal(a["tr_c2"], b["tr_c2"])
    assert a["messages"] == b["messages"] and a["status"] == b["status"] and a["iterations"] == b["iterations"]
