#!/usr/bin/env python3
"""configs[4] on one card: does the slow regime follow from the queues the earlier
contexts of a rank created, with no computation on them? Before running bench.py in this process,
creates and closes solver contexts that never compute: PRECTX_SHARDED sharded ones (this rank's
CU-masked stream under LBFGS_CU_PARTITION=1, as the headline's and the vector-free line's) and
PRECTX_ONE one-GPU ones (an unmasked stream, as rank 0's shard check), alternating.

usage (as a rank wrapper):
  PRECTX_SHARDED=2 PRECTX_ONE=1 BENCH_RANK_WRAPPER="python tools/prectx_wrap.py --" \\
      python bench.py --gpus 8 --size 1e9 ...
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

args = sys.argv[1:]
if args and args[0] == "--":
    args = args[1:]
if args and os.path.basename(args[0]).startswith("python"):
    args = args[1:]
rank = int(os.environ.get("RANK", "0"))
world = 8
for i, a in enumerate(args):
    if a == "--gpus" and i + 1 < len(args):
        world = int(args[i + 1])
ns, n1 = int(os.environ.get("PRECTX_SHARDED", "2")), int(os.environ.get("PRECTX_ONE", "1"))
dev = 0 if "BENCH_DEVICE_MOD" in os.environ else rank
made = []
for i in range(max(ns, n1)):
    if i < ns:
        with L.Context(10 ** 7, 10, device=dev, rank=rank, world=world, uid=None):
            made.append("sharded")
    if i < n1:
        with L.Context(10 ** 6, 10, device=dev):
            made.append("one-GPU")
print(f"rank {rank}: created and closed {made} before the bench", file=sys.stderr, flush=True)
sys.argv = args
runpy.run_path(args[0], run_name="__main__")
