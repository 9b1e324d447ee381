"""CPU: the oracle's vector-free restatement (orc_lbfgs_vf) against the reference's own
sequential traces — f and |g| within 1e-10 relative over the measured horizons and the same
outcome on the golden cases — so the vector-free order is pinned to the reference the same way
as the canonical order (tests/test_gpu_vector_free.py then holds the GPU to it bit for bit)."""
import numpy as np
import pytest

import oracle_lib as O
from test_gpu_vector_free import HORIZON_VF

FAST = ["qsep_main", "qtri_n1e4_m10_bt", "qtri_n1e4_m20_wolfe", "qtri_n1e5_m20_wolfe", "rosen_n100_m5_bt",
        "rosen_n1_bt", "rosen_n1e4_m5_bt", "rosen_n1e4_m5_btw", "rosen_n1e4_m5_interp", "rosen_n1e4_m5_wolfe",
        "rosen_n1e5_m10_bt", "rosen_n2_m3_bt", "rosen_n3_m1_wolfe", "rosen_n4097_m7_interp"]


@pytest.mark.parametrize("name", FAST)
def test_oracle_vector_free_vs_reference_trace(name):
    meta, g = O.load_golden(name)
    x0 = O.x0_uniform(meta["n"], meta["seed"], meta["lo"], meta["hi"])
    v = O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"], mode=O.CANON,
                vector_free=True)
    Kf, Kg = HORIZON_VF[name]
    if meta["method"] in ("backtracking", "interpolation"):
        gnf = g["grad_nf"].astype(np.int64)
        ref_f, ref_g = g["f_calls"][gnf - 1], g["grad_norm"]
    else:
        s = O.lbfgs(meta["objective"], x0, meta["method"], meta["m"], meta["maxit"], meta["tol"], mode=O.SEQ)
        ref_f, ref_g = s["f"], s["gnorm"]
    rel_f = np.abs(v["f"][:Kf] - ref_f[:Kf]) / np.maximum(np.abs(ref_f[:Kf]), 1e-300)
    rel_g = np.abs(v["gnorm"][:Kg] - ref_g[:Kg]) / np.maximum(np.abs(ref_g[:Kg]), 1e-300)
    assert np.all(rel_f <= 1e-10) and np.all(rel_g <= 1e-10)
    assert v["messages"].strip().splitlines()[-1] == meta["stdout"].strip().splitlines()[-1]
