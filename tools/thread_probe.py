#!/usr/bin/env python3
"""Which step of bench.py's sequence leaves a host thread spinning beside the solver's own
(in the one-card N = 8 rehearsal every rank runs two threads at 100 % during
configs[4] and the job's 16-CPU quota throttles)? One process, one GPU, n = 1e8, m = 10: a solve
of 20 iterations after each step below, with every thread's CPU ticks over that solve
(/proc/self/task/*/stat) and the thread count.

usage: python tools/thread_probe.py [out.json]
       python tools/thread_probe.py --solves K [out.json]   (only K solves of 30 iterations on one
       context: run under the library's switches to find the host interaction behind the spin)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402


def ticks():
    out = {}
    for t in os.listdir("/proc/self/task"):
        try:
            s = open(f"/proc/self/task/{t}/stat").read()
        except OSError:
            continue
        f = s[s.rindex(")") + 2:].split()
        out[int(t)] = int(f[11]) + int(f[12])
    return out


rows = []


def solve_and_count(ctx, what, steps=20):
    a = ticks()
    t = time.perf_counter()
    ctx.step(steps)
    ctx.sync()
    dt = time.perf_counter() - t
    b = ticks()
    busy = sorted(((b[k] - a.get(k, 0)) / 100.0 / dt for k in b), reverse=True)
    row = dict(after=what, threads=len(b), busy_threads=sum(1 for x in busy if x > 0.5),
               top_cpu=[round(x, 2) for x in busy[:4]], ms_per_it=round(dt / steps * 1e3, 2),
               new_threads=sorted(set(b) - set(a)))
    rows.append(row)
    print(row, flush=True)


n, m = 10 ** 8, 10
x0 = L.x0_uniform(n, 42, -2.0, 2.0)
L.lib()
if len(sys.argv) > 2 and sys.argv[1] == "--solves":
    sw = {k: v for k, v in os.environ.items() if k.startswith("LBFGS_")}
    with L.Context(n, m) as c:
        c.init("rosenbrock", x0, "backtracking", tolerance=1e-5)
        c.step(m)
        for i in range(int(sys.argv[2])):
            solve_and_count(c, f"solve {i} {sw}", 30)
    if len(sys.argv) > 3:
        json.dump(dict(tool="tools/thread_probe.py", switches=sw, rows=rows, build=L.build_info()[0]),
                  open(sys.argv[3], "w"), indent=1)
    sys.exit(0)
c = L.Context(n, m)
c.init("rosenbrock", x0, "backtracking", tolerance=1e-5, trace=True)
c.step(m)
solve_and_count(c, "history fill (traced init)")
c.trace_enable(False)
solve_and_count(c, "trace off")
c.stream_probe(20)
solve_and_count(c, "stream_probe")
c.prof_reset()
c.prof_enable(True)
c.step(5)
c.sync()
for k in L.KERNELS:
    c.prof_get(k)
c.prof_enable(False)
solve_and_count(c, "prof (HIP event pairs)")
c.close()
c = L.Context(n, m)
c.init("rosenbrock", x0, "backtracking", tolerance=1e-5)
c.step(m)
solve_and_count(c, "a new context")
c.close()
c = L.Context(n, m)
c.init("rosenbrock", x0, "backtracking", tolerance=1e-5, vector_free=True)
c.step(m)
solve_and_count(c, "vector-free context")
c.close()
out = dict(tool="tools/thread_probe.py", rows=rows, build=L.build_info()[0])
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
print(json.dumps(out))
