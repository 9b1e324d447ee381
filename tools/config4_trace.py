#!/usr/bin/env python3
"""Per-rank iteration times from rocprofv3 kernel traces of a sharded bench run (BENCH_RANK_WRAPPER,
tools/gpu_r05b.sh): the time between consecutive commit launches (one per iteration), the steady-state
mean (h = m, the last `tail` iterations of the sharded solve), and the exchange kernels' share of the
sharded solve. A rank that also ran the one-GPU repeat (shard_check) shows it as a second block.

usage: python tools/config4_trace.py <dir with *_kernel_trace.csv[.gz]> [tail]
"""
import csv
import glob
import gzip
import io
import os
import sys


def rows_of(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as fp:
        return sorted(csv.DictReader(io.StringIO(fp.read())), key=lambda r: int(r["Start_Timestamp"]))


def series(its):
    """the whole block's iteration times: mean of each tenth, in order (drift over the solve)"""
    if len(its) < 20:
        return ""
    k = len(its) // 10
    return f"; {len(its)} iterations, mean per tenth (ms): " + " ".join(
        f"{sum(its[i * k:(i + 1) * k]) / k:.1f}" for i in range(10))


def main():
    d = sys.argv[1]
    tail = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    files = sorted(glob.glob(os.path.join(d, "*_kernel_trace.csv*")))
    for f in files:
        rows = rows_of(f)
        commits = [r for r in rows if "k_commit" in r["Kernel_Name"]]
        starts = [int(r["Start_Timestamp"]) for r in commits]
        # blocks of the solve separated by a gap of > 2 s (the one-GPU repeat comes after a barrier)
        blocks, cur = [], [starts[0]] if starts else []
        for a, b in zip(starts, starts[1:]):
            if b - a > 2e9:
                blocks.append(cur)
                cur = []
            cur.append(b)
        if cur:
            blocks.append(cur)
        out = []
        for bi, blk in enumerate(blocks):
            gaps = [(b - a) / 1e6 for a, b in zip(blk, blk[1:])]
            # an iteration whose first step was rejected has a second (re)commit a few ms after the
            # first: iteration times are the gaps between first commits (gaps above 0.3x the block's
            # upper quartile)
            q3 = sorted(gaps)[3 * len(gaps) // 4] if gaps else 0.0
            every = [g for g in gaps if g > 0.3 * q3]
            its = every[-tail:]
            med = sorted(its)[len(its) // 2] if its else 0.0
            lo, hi = blk[0], blk[-1]
            ex = [r for r in rows if "xgmi" in r["Kernel_Name"] and lo <= int(r["Start_Timestamp"]) <= hi]
            ex_ms = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ex) / 1e6
            out.append(f"block {bi}: {len(blk)} commits over {(hi - lo) / 1e6:.1f} ms; last {len(its)} iterations "
                       f"median {med:.1f} ms ({1e3 / med if med else 0:.2f} it/s; "
                       f"{', '.join(f'{g:.1f}' for g in its)}); exchange kernels {len(ex)}, {ex_ms:.1f} ms "
                       f"({100 * ex_ms / max((hi - lo) / 1e6, 1e-9):.1f} %)" + series(every))
        print(os.path.basename(f).split("_")[0], "|", " || ".join(out))


if __name__ == "__main__":
    main()
