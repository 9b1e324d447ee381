#!/usr/bin/env python3
"""Device memory around every solver context of a bench rank (DESIGN.md §5, configs[4] on one
card): runs bench.py in this process with lbfgs_amd.Context's create / init / close wrapped so each
logs hipMemGetInfo's free bytes (device-wide: on one card, every rank's allocations) to stderr.

usage (as a rank wrapper): BENCH_RANK_WRAPPER="python tools/meminfo_wrap.py --" python bench.py ...
"""
import ctypes as C
import os
import runpy
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402

args = sys.argv[1:]
if args and args[0] == "--":
    args = args[1:]
if args and os.path.basename(args[0]).startswith("python"):
    args = args[1:]  # the launcher passes [python, bench.py, ...]
RANK = os.environ.get("RANK", "0")
T0 = time.perf_counter()
HIP = None


def log(tag, n=None):
    global HIP
    if HIP is None:
        HIP = C.CDLL("libamdhip64.so")
    free, total = C.c_size_t(), C.c_size_t()
    HIP.hipMemGetInfo(C.byref(free), C.byref(total))
    print(f"meminfo rank {RANK} t={time.perf_counter() - T0:7.1f}s {tag:<14} n={n} free {free.value / 2**30:7.1f} "
          f"of {total.value / 2**30:.1f} GiB", file=sys.stderr, flush=True)


_init, _close, _solve_init = L.Context.__init__, L.Context.close, L.Context.init


def init(self, n, *a, **k):
    t = time.perf_counter()
    _init(self, n, *a, **k)
    log(f"create {time.perf_counter() - t:.2f}s", n)


def close(self):
    live = getattr(self, "h", None)
    _close(self)
    if live:
        log("close", self.n)


def solve_init(self, *a, **k):
    t = time.perf_counter()
    r = _solve_init(self, *a, **k)
    log(f"init {time.perf_counter() - t:.2f}s", self.n)
    return r


L.Context.__init__, L.Context.close, L.Context.init = init, close, solve_init
sys.argv = args
runpy.run_path(args[0], run_name="__main__")
