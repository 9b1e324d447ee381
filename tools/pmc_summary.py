#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/: kernel stats (trace) and PMC byte counters.

usage: python tools/pmc_summary.py <trace_dir> <fetch_dir> <write_dir> <out.json> [n [bench_log ...]]

bench_log: the output of the profiled bench runs; the `build` of their JSON line (the library's
source hash, lbfgs_build_info) is recorded as `_build`, and every log must name the same library.
bench.py's pmc_traffic() only takes traffic from a summary whose `_build` is the loaded library's.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. On gfx950 FETCH_SIZE counts half of the bytes
of wide (16 B/lane) coalesced streaming reads (MI355X_MICROARCH.md §HBM), so the corrected HBM
read bytes are 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for 16-B streaming stores.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def find(d, name):
    """d/name, or the one file of that name below d (rocprofv3 adds host / pid levels)"""
    p = os.path.join(d, name)
    if os.path.exists(p):
        return p
    hits = sorted(glob.glob(os.path.join(d, "**", name), recursive=True))
    if not hits:
        raise FileNotFoundError(p)
    return hits[-1]


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    m = re.match(r"([A-Za-z_0-9]+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


def build_of(logs):
    """the `build` object of the bench JSON line in each log; all must agree"""
    seen = []
    for fn in logs:
        for line in open(fn):
            if line.startswith("{"):
                try:
                    d = json.loads(line)
                except ValueError:
                    continue
                if "build" in d:
                    seen.append((fn, d["build"]))
    libs = {b.get("library") for _, b in seen}
    if len(libs) > 1:
        raise SystemExit(f"profiled runs name different libraries: {seen}")
    return seen[0][1] if seen else None


def main(trace_dir, fetch_dir, write_dir, out, n=None, logs=()):
    res = collections.OrderedDict()
    if logs:
        b = build_of(logs)
        if b is None:
            raise SystemExit(f"no bench JSON line with a build field in {logs}")
        res["_build"] = b
    for r in csv.DictReader(open(find(trace_dir, "run_kernel_stats.csv"))):
        k = short(r["Name"])
        res.setdefault(k, {})
        res[k].update(calls=int(r["Calls"]), avg_us=float(r["AverageNs"]) / 1e3,
                      total_pct=float(r["Percentage"]))
    for tag, d in [("FETCH_SIZE", fetch_dir), ("WRITE_SIZE", write_dir)]:
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(find(d, "run_counter_collection.csv"))):
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            res.setdefault(k, {})[tag + "_KiB"] = sum(v) / len(v)
    for k, v in res.items():
        if k.startswith("_"):
            continue
        if "FETCH_SIZE_KiB" in v and "WRITE_SIZE_KiB" in v:
            rd = 2 * v["FETCH_SIZE_KiB"] * 1024
            wr = v["WRITE_SIZE_KiB"] * 1024
            v["hbm_read_bytes_corrected"] = rd
            v["hbm_write_bytes"] = wr
            v["hbm_bytes_per_launch"] = rd + wr
            if n:
                v["read_vectors"] = rd / (8 * n)
                v["write_vectors"] = wr / (8 * n)
            if "avg_us" in v:
                v["measured_GBps"] = (rd + wr) / (v["avg_us"] * 1e-6) / 1e9
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        if k.startswith("_"):
            print(f"{k}: {v}")
            continue
        print(f"{k:34s} " + " ".join(f"{kk}={vv:.4g}" if isinstance(vv, float) else f"{kk}={vv}"
                                      for kk, vv in v.items()))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], float(sys.argv[5]) if len(sys.argv) > 5 else None,
         sys.argv[6:])
