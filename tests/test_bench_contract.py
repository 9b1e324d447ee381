"""bench.py's host-side pieces on CPU: the roofline object of the JSON line (achieved = algorithmic
bytes per launch / average launch time, frac against the 8 TB/s spec), the PMC traffic lookup
from the committed profiles, and the profile file tags. The GPU run itself is the driver's."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def bench():
    import bench as B  # loads liblbfgs_hip.so (no GPU needed to load it)

    return B


def test_ntag(bench):
    assert bench.ntag(10 ** 8) == "1e8"
    assert bench.ntag(10 ** 4) == "1e4"
    assert bench.ntag(12_500_000) == "12500000"


def test_roofline_object(bench):
    prof = {"axpy_dot": {"ms": 560.0, "launches": 1000, "bytes": 3.2e12},
            "commit": {"ms": 100.0, "launches": 100, "bytes": 6.4e11}}
    r = bench.roofline(prof, 10 ** 8, 1)
    assert r["kernel"] == "axpy_dot" and r["bound"] == "hbm" and r["unit"] == "GB/s"
    assert r["achieved"] == pytest.approx(3.2e9 / 0.56e-3 / 1e9, rel=1e-3)
    assert r["peak"] == 8000.0 and r["frac"] == pytest.approx(r["achieved"] / 8000.0, rel=1e-3)
    assert r["avg_launch_us"] == pytest.approx(560.0)
    assert sum(r["kernel_share"].values()) == pytest.approx(1.0, abs=1e-3)
    assert bench.roofline({}, 10 ** 8, 1) is None


def test_pmc_traffic_from_committed_profile(bench):
    traffic, src = bench.pmc_traffic("axpy_dot", 10 ** 8, 1)
    assert src and src.startswith("profiles/") and os.path.exists(os.path.join(ROOT, src))
    # corrected PMC bytes per launch within 1 % of the algorithmic 4 vectors x 800 MB
    assert traffic == pytest.approx(3.2e9, rel=0.01)
    vf, _ = bench.pmc_traffic("vf_commit", 10 ** 8, 1)
    assert vf == pytest.approx(26 * 8e8, rel=0.02)
    assert bench.pmc_traffic("axpy_dot", 10 ** 8, 8) == (None, None)  # per-rank PMC not committed


def test_cpu_baseline_runner(bench):
    """The reference timed on host cores beside the GPU run: child processes, steady iterations
    (h = m) averaged, pinning recorded (tiny sizes here; bench.py runs n = 1e8 and 1e7)."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "ref_lbfgs")):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    aff = os.sched_getaffinity(0)
    try:
        cb = bench.CpuBaseline([3000, 1000], 3)
        out = cb.collect(timeout=120)
    finally:
        os.sched_setaffinity(0, aff)
    assert [o["n"] for o in out] == [3000, 1000]
    for o in out:
        assert o["per_iter_s"] > 0 and o["iters_timed"] == 2 and isinstance(o["pinned"], bool)
