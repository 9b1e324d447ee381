#!/usr/bin/env python3
"""Per-kernel means of the gap probe's counter passes (tools/gpu_r06.sh gappmc).

usage: python tools/gap_pmc_summary.py out.json <pass_dir> [<pass_dir> ...]

Each pass dir holds one rocprofv3 --pmc run of tools/gap_probe.py; its run_counter_collection.csv
has one row per (dispatch, counter). The summary averages every counter over a kernel's dispatches
and derives per-wave figures for the two-loop pass against the probe kernels:
instructions per wave (VALU, SALU, VMEM), wave cycles per wave, the share of wave cycles spent
waiting (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES) and HBM bytes (FETCH_SIZE doubled for gfx950's wide
streaming reads, MI355X_MICROARCH.md §HBM, + WRITE_SIZE).
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402

KERNELS = ("k_axpy_dot", "k_axpy2_dot", "k_probe_stream", "k_probe_stream2", "k_commit", "k_probe_commit")


def main(out, dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for fn in sorted(glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True)):
            for r in csv.DictReader(open(fn)):
                agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in agg.items():
        if not any(k.startswith(p) for p in KERNELS):
            continue
        v = {c: sum(x) / len(x) for c, x in cs.items()}
        v["dispatches"] = max(len(x) for x in cs.values())
        waves = v.get("SQ_WAVES")
        if waves:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM",
                      "SQ_INSTS_LDS", "SQ_WAVE_CYCLES"):
                if c in v:
                    v[c + "_per_wave"] = v[c] / waves
        if v.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in v:
                    v[c + "_share"] = v[c] / v["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            v["hbm_bytes"] = (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
        res[k] = v
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    keys = sorted({c for v in res.values() for c in v})
    for k in sorted(res):
        print(k)
        for c in keys:
            if c in res[k]:
                print(f"   {c:32s} {res[k][c]:.6g}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
