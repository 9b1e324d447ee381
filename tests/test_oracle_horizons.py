"""The canonical order's horizon against the reference is the reference's own conditioning.

tests/golden/horizons.json (tests/golden/make_horizons.py) holds, per golden case, how many
leading iterations keep f and |g| within 1e-10 of the reference when only the order of its sums
changes: the canonical device order, and three equally valid alternatives (pairwise, right to
left, FMA-contracted). The fixture is recomputed here, and the canonical order's horizon must be
at least the alternatives' minimum (K_ref): where the GPU (bit-exact with the canonical order,
tests/test_gpu_parity.py) stops agreeing with the reference after 2 iterations, so does the
reference itself under a different order. The GPU test asserts the same bound on the device run.
"""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_horizons as MH  # noqa: E402
import oracle_lib as O  # noqa: E402

FIXTURE = json.load(open(os.path.join(HERE, "golden", "horizons.json")))


def test_fixture_covers_every_golden():
    assert sorted(FIXTURE) == O.golden_cases()


@pytest.mark.parametrize("name", O.golden_cases())
def test_horizons_recomputed(name):
    assert MH.case_horizons(name) == FIXTURE[name]


@pytest.mark.parametrize("name", O.golden_cases())
def test_canonical_horizon_at_least_the_references_own(name):
    h = FIXTURE[name]
    assert h["canon"][0] >= h["ref"][0] and h["canon"][1] >= h["ref"][1], h
