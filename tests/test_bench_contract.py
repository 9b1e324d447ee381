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
    import bench as B  # liblbfgs_hip.so loads on first use (no GPU needed to load it)

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


def test_pmc_traffic_requires_this_library(bench, tmp_path, monkeypatch):
    """traffic comes only from a PMC summary profiled on the loaded library (its `_build` carries
    the library's source hash); a summary of other code is refused and says why; the newest
    round wins; sharded lines have no per-rank PMC."""
    import json

    lib = bench.L.build_info()[0]
    (tmp_path / "profiles" / "r01").mkdir(parents=True)
    (tmp_path / "profiles" / "r02").mkdir(parents=True)
    entry = {"k_axpy_dot<true, false>": {"hbm_bytes_per_launch": 3.2e9}, "k_vf_commit<0, 10, true>":
             {"hbm_bytes_per_launch": 2.08e10}}
    (tmp_path / "profiles" / "r01" / "pmc_bench_n1e8.json").write_text(json.dumps(dict(entry, _build={"library": lib})))
    (tmp_path / "profiles" / "r02" / "pmc_bench_n1e8.json").write_text(
        json.dumps(dict(entry, _build={"library": "src=0000000000000000 built=x arch=gfx950"})))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    t, src, why = bench.pmc_traffic("axpy_dot", 10 ** 8, 1)
    assert t == 3.2e9 and src == "profiles/r01/pmc_bench_n1e8.json"
    assert bench.pmc_traffic("vf_commit", 10 ** 8, 1)[0] == 2.08e10
    (tmp_path / "profiles" / "r01" / "pmc_bench_n1e8.json").unlink()
    t, src, why = bench.pmc_traffic("axpy_dot", 10 ** 8, 1)
    assert t is None and src is None and "profiles/r02/pmc_bench_n1e8.json" in why and "src=0000" in why
    assert bench.pmc_traffic("axpy_dot", 10 ** 8, 8) == (None, None, None)  # per-rank PMC not committed
    r = bench.roofline({"axpy_dot": {"ms": 560.0, "launches": 1000, "bytes": 3.2e12}}, 10 ** 8, 1)
    assert r["traffic"] is None and r["traffic_refused"] == why


def test_committed_pmc_summaries_record_their_library(bench):
    """every committed PMC summary from round 4 on names the library it was profiled on"""
    import glob
    import json

    for fn in glob.glob(os.path.join(ROOT, "profiles", "r0[4-9]", "**", "pmc_bench_n*.json"), recursive=True):
        b = json.load(open(fn)).get("_build") or {}
        assert b.get("library", "").startswith("src="), fn


def test_box_fields(bench):
    p = {"avg_launch_us": 500.0, "bytes_per_launch": 3.2e9, "gbps": 6400.0, "gbps_min_over_ranks": 6400.0,
         "gbps_sum_over_ranks": 6400.0}
    f = bench.box_fields(p, 90.0, 5900.0, 1)
    assert f["box_copy_tbps"] == 6.4 and f["value_per_box_tbps"] == pytest.approx(90.0 / 6.4, rel=1e-3)
    assert f["hbm_frac_of_box"] == pytest.approx(5900.0 / 6400.0, rel=1e-3)
    assert bench.box_fields(None, 90.0, 5900.0, 1) == {"box_copy_tbps": None}
    # sharded: the ranks' concurrent probes add up to the box (8 GPUs, or one shared card)
    p8 = dict(p, gbps_min_over_ranks=5800.0, gbps_sum_over_ranks=8 * 6000.0)
    f8 = bench.box_fields(p8, 700.0, 40000.0, 8)
    assert f8["box_copy_tbps"] == 48.0 and f8["hbm_frac_of_box"] == pytest.approx(40000.0 / 48000.0, rel=1e-3)
    assert f8["box_probe"]["slowest_rank_gbps"] == 5800.0


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


def test_roofline_ignores_exchange_and_stage2(bench):
    """The dominant kernel is the streaming pass with the most time: a long exchange wait (bytes 0)
    or a stage-2 launch never becomes the roofline kernel."""
    prof = {"axpy_dot": {"ms": 560.0, "launches": 1000, "bytes": 3.2e12},
            "exchange": {"ms": 5000.0, "launches": 2000, "bytes": 0.0},
            "group_reduce": {"ms": 900.0, "launches": 900, "bytes": 0.0},
            "_exchange_share": {"share_max_over_ranks": 0.5}}
    assert bench.roofline(prof, 10 ** 8, 8)["kernel"] == "axpy_dot"


def _trajectory(o):
    return dict(tr_f=o["f"], tr_gnorm=o["gnorm"], tr_alpha=o["alpha"], tr_c1=o["c1"], tr_c2=o["c2"])


def test_reference_parity_live_and_fixture(bench):
    """reference_parity: the trajectory of the measured run (here the canonical-order oracle, which
    the GPU reproduces bit for bit) against the reference's live CPU-baseline run, and against a
    fixture of the canonical order (bit for bit; one flipped bit is caught)."""
    import numpy as np

    import oracle_lib as O

    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "ref_lbfgs")):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    n, m = 3000, 3
    aff = os.sched_getaffinity(0)
    try:
        live = bench.CpuBaseline([n], m).collect(timeout=120)[0]["trajectory"]
    finally:
        os.sched_setaffinity(0, aff)
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    can = O.lbfgs("rosenbrock", x0, "backtracking", m, 2 * m + 2, 1e-5, mode=O.CANON)
    traj = _trajectory(can)
    p = bench.reference_parity(traj, live, None, None)
    assert p["ok"] and p["iterations_compared"] == m + 3 and p["first_divergent_k"] is None
    assert p["max_rel_f"] <= 1e-10 and p["x_bit_identical_iterations"] >= 2  # x_0, x_1 = x_0 - g_0
    hexes = lambda a: [f"{int(u):016x}" for u in np.asarray(a, np.float64).view(np.uint64)]  # noqa: E731
    seq = O.lbfgs("rosenbrock", x0, "backtracking", m, m + 2, 1e-5, mode=O.SEQ)
    canon_short = O.lbfgs("rosenbrock", x0, "backtracking", m, m + 2, 1e-5, mode=O.CANON)
    fx = {"reference": {"grad_norm": hexes(live["gnorm"]), "grad_c1": [str(int(v)) for v in live["c1"]]},
          "seq": {"f": hexes(seq["f"]), "gnorm": hexes(seq["gnorm"]), "c1": [str(int(v)) for v in seq["c1"]],
                  "c2": [str(int(v)) for v in seq["c2"]]},
          "canon": {"f": hexes(canon_short["f"]), "gnorm": hexes(canon_short["gnorm"]),
                    "alpha": hexes(canon_short["alpha"]), "c1": [str(int(v)) for v in canon_short["c1"]],
                    "c2": [str(int(v)) for v in canon_short["c2"]]},
          "horizons": {"ref": [m + 3, m + 3]}}
    p = bench.reference_parity(traj, live, fx, "fixture.json")
    assert p["ok"] and p["canonical"]["bit_exact"] and p["live_reference_matches_fixture"]
    p = bench.reference_parity(traj, None, fx, "fixture.json")  # sharded lines: the fixture's reference
    assert p["ok"] and p["reference"].startswith("fixture")
    bad = dict(traj, tr_f=traj["tr_f"].copy())
    bad["tr_f"][2] = np.nextafter(bad["tr_f"][2], np.inf)
    p = bench.reference_parity(bad, live, fx, "fixture.json")
    assert not p["canonical"]["bit_exact"] and not p["ok"]
    # past the reference's own horizon a divergence is reported, not failed; before it, it fails
    far = dict(traj, tr_gnorm=traj["tr_gnorm"].copy())
    far["tr_gnorm"][m + 2] *= 1.0 + 1e-8
    fx2 = dict(fx, horizons={"ref": [m + 3, m + 2]})
    fx2["canon"] = dict(fx["canon"], gnorm=hexes(np.concatenate([canon_short["gnorm"][:m + 2], far["tr_gnorm"][m + 2:m + 3]])))
    p = bench.reference_parity(far, live, fx2, "fixture.json")
    assert p["first_divergent_k"] == m + 2 and p["within_tolerance_iterations"]["gnorm"] == m + 2 and p["ok"]
    p = bench.reference_parity(far, live, dict(fx2, horizons={"ref": [m + 3, m + 3]}), "fixture.json")
    assert not p["ok"]


def test_fullsize_fixture_lookup(bench):
    """the committed full-size fixture of a workload, or (None, None) at sizes without one; files
    of other shapes (the CUDA-mode cases, with no single method) are passed over, not a KeyError
    (bench.py --size 1.25e8 failed there in round 5)"""
    import types

    a = types.SimpleNamespace(objective="rosenbrock", history=10, line_search="backtracking")
    d, src = bench.fullsize_fixture(a, 10 ** 8)
    assert d is not None and src.endswith("config2_n1e8.json")
    d, src = bench.fullsize_fixture(a, 10 ** 7)
    assert d is not None and src.endswith("config1_n1e7.json")
    assert bench.fullsize_fixture(a, 125_000_000) == (None, None)
    assert bench.fullsize_fixture(a, 50_000_000) == (None, None)


def test_reference_parity_with_an_x0_only_fixture(bench):
    """configs[4]'s fixture holds the reference at x0 only (no per-iteration trace): the line
    compares that state and the canonical states instead of failing (KeyError 'seq', round 5)"""
    import types

    import numpy as np

    a = types.SimpleNamespace(objective="rosenbrock", history=10, line_search="backtracking")
    fx, src = bench.fullsize_fixture(a, 10 ** 9)
    assert fx is not None and "seq" not in fx
    c = fx["canon"]
    f64 = lambda hs: np.array([int(h, 16) for h in hs], dtype=np.uint64).view(np.float64)  # noqa: E731
    traj = {"tr_f": f64(c["f"]), "tr_gnorm": f64(c["gnorm"]), "tr_alpha": f64(c["alpha"] + ["0"]),
            "tr_c1": np.array([int(v) for v in c["c1"]], dtype=np.uint64),
            "tr_c2": np.array([int(v) for v in c["c2"]], dtype=np.uint64)}
    out = bench.reference_parity(traj, None, fx, src)
    assert out["iterations_compared"] == 1 and out["within_tolerance_iterations"]["f"] == 1
    assert out["canonical"]["bit_exact"] is True
