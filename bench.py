#!/usr/bin/env python3
"""Headline benchmark: L-BFGS iterations/s and achieved HBM GB/s on n = 1e8 Rosenbrock, m = 10,
backtracking line search, fp64 (BASELINE.json metric; configs[2] on one GPU, the 1->8 GPU
series sharding the same n across ranks).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

With --gpus N > 1 and no launcher around it (no RANK in the environment) bench.py is its own
launcher: it starts the N rank processes itself (self_launch) before anything touches a GPU.

A step is one L-BFGS iteration of the whole n-vector problem (two-loop recursion, line search,
commit). Before the W warm-up steps, m untimed iterations fill the m-pair history
(`history_fill`), so every timed step uses h = m pairs whatever W is; the line reports the
h range of the timed steps (`h_min`, `h_max`, `steady_state`).
All vectors are resident in HBM before timing starts. One process per GPU; the solver's data
path exchanges group partials through the xGMI peer mailboxes (or RCCL all-gathers) inside
liblbfgs_hip.so; torch.distributed (gloo) is only used for the rendezvous (unique id), barriers,
votes and the max-over-ranks time.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import platform
import shutil
import signal
import socket
import struct
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402  (ctypes only: the library is loaded in main(), not here)
import numpy as np  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    # (not --n / --m: torch.distributed.run would take them as its own abbreviated options)
    p.add_argument("--size", type=float, default=1e8, help="problem size n")
    p.add_argument("--history", type=int, default=10, help="L-BFGS memory m")
    p.add_argument("--objective", default="rosenbrock")
    p.add_argument("--line-search", default="backtracking")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-n", type=float, default=None,
                   help="CPU baseline size (default: the benchmark's n, measured directly)")
    p.add_argument("--cpu-n2", type=float, default=1e7,
                   help="secondary CPU baseline size reported beside it (0: none)")
    p.add_argument("--no-prof", action="store_true", help="no per-kernel HIP events")
    p.add_argument("--unfused", action="store_true",
                   help="one launch per BLAS-1 op (BASELINE configs[1] shape), same iterates")
    p.add_argument("--vector-free", action="store_true",
                   help="Gram-matrix two-loop, one fused pass per iteration (opt-in mode)")
    p.add_argument("--no-persistent", action="store_true",
                   help="skip the persistent-block two-loop line (LBFGS_PERSIST=2) beside the default")
    p.add_argument("--persistent", action="store_true",
                   help="measure the headline itself with the persistent-block two-loop (LBFGS_PERSIST=2)")
    p.add_argument("--no-vector-free", action="store_true",
                   help="skip the vector-free measurement reported beside the default mode")
    p.add_argument("--no-config4", action="store_true",
                   help="8 ranks: skip the n=1e9 measurement (BASELINE configs[4]) after the headline")
    p.add_argument("--exchange", choices=["auto", "xgmi", "rccl"], default="auto",
                   help="sharded runs: reductions through the xGMI peer mailboxes (measured again over "
                        "RCCL when any rank's mailbox self-test fails) or RCCL all-gathers; auto: the "
                        "mailboxes, with an RCCL communicator created and timed only after the "
                        "measurement (bounded by LBFGS_RCCL_TIMEOUT, reported as rccl_leg)")
    p.add_argument("--launch-timeout", type=float, default=float(os.environ.get("BENCH_LAUNCH_TIMEOUT", 3000)),
                   help="--gpus N > 1 without a launcher: seconds before the self-launched ranks are stopped")
    p.add_argument("--no-box-probe", action="store_true", help="skip the in-process HBM stream probe")
    return p.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(argv, world, timeout, script=None):
    """--gpus N > 1 with no launcher around the command (no RANK in the environment): start the N
    rank processes here, as `torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr
    127.0.0.1` would - RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR = 127.0.0.1 and
    a free MASTER_PORT in each child's environment - and wait for them. This process never touches
    a GPU (it has not loaded liblbfgs_hip.so): the ranks are fresh child processes, nothing is
    re-executed. Rank 0's JSON line is this process's only stdout; every other line any rank
    prints on stdout (gloo's connection notes, for one) goes to stderr. As soon as a rank fails, or `timeout` seconds pass, the remaining ranks are
    stopped (their process groups: SIGTERM, then SIGKILL after 15 s) and the exit status is
    non-zero: the failed rank's, or 124 on the time limit. Returns the exit status."""
    script = script or os.path.abspath(__file__)
    port = _free_port()
    procs = []
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                LOCAL_WORLD_SIZE=str(world))
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for the peer mailboxes / RCCL
    if "BENCH_DEVICE_MOD" in base:
        # several ranks on one card (a rehearsal): one unmasked hardware queue per rank, its
        # CU-masked solver queue on top. With the runtime's default each rank holds 3 compute
        # queues and rank 0's one-GPU check adds a 25th on the card, past what its scheduler maps
        # at once: the ranks' passes then run in turns (configs[4] 2.5-5 it/s instead of 8.7;
        # DESIGN.md §5, profiles/r05/config4_queues/). One process per GPU never gets near that.
        # (Set, not defaulted: the runtime's default, 4, is often already in the environment.)
        base["GPU_MAX_HW_QUEUES"] = "1"

    def stop(reason):
        alive = [p for p in procs if p.poll() is None]
        if alive:
            print(f"bench.py launcher: {reason}; stopping {len(alive)} rank(s)", file=sys.stderr, flush=True)
        for p in alive:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        t_end = time.monotonic() + 15
        for p in alive:
            try:
                p.wait(timeout=max(t_end - time.monotonic(), 0.1))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    def on_term(signum, frame):  # the launcher itself is stopped: take the ranks with it
        stop(f"signal {signum}")
        sys.exit(128 + signum)

    def forward(pipe):  # rank 0: JSON lines to stdout, the rest to stderr
        for line in iter(pipe.readline, b""):
            out = sys.stdout if line.startswith(b"{") else sys.stderr
            out.buffer.write(line)
            out.flush()
        pipe.close()

    import threading

    old = signal.signal(signal.SIGTERM, on_term)
    rc = 0
    fwd = None
    # BENCH_RANK_WRAPPER (profiling): a command each rank is started under, e.g. "rocprofv3
    # --kernel-trace --stats -d DIR -o %pid% --": the profiler then starts the rank itself (this
    # launcher stays outside it and never touches a GPU)
    import shlex

    wrap = shlex.split(os.environ.get("BENCH_RANK_WRAPPER", ""))
    try:
        for r in range(world):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
            env.pop("BENCH_RANK_WRAPPER", None)
            procs.append(subprocess.Popen([*wrap, sys.executable, script, *argv], env=env, start_new_session=True,
                                          stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
            if r == 0:
                fwd = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True)
                fwd.start()
        deadline = time.monotonic() + timeout
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                rc = c if c > 0 else 128 - c  # killed by signal s: 128 + s
                stop(f"rank {r} exited with status {c}")
                break
            if all(c == 0 for c in codes):
                break
            if time.monotonic() > deadline:
                rc = 124
                stop(f"time limit of {timeout:.0f} s")
                break
            time.sleep(0.2)
    finally:
        stop("launcher exiting")
        signal.signal(signal.SIGTERM, old)
        if fwd is not None:
            fwd.join(timeout=10)
    return rc


class Dist:
    def __init__(self, world):
        self.world = world
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if world > 1:
            import torch.distributed as dist

            dist.init_process_group("gloo", rank=self.rank, world_size=world)
            self.dist = dist

    def broadcast_bytes(self, b):
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def allreduce(self, v, op="max"):
        if not self.dist:
            return v
        import torch

        t = torch.tensor([v], dtype=torch.float64)
        ops = {"max": self.dist.ReduceOp.MAX, "min": self.dist.ReduceOp.MIN, "sum": self.dist.ReduceOp.SUM}
        self.dist.all_reduce(t, op=ops[op])
        return float(t.item())

    def allgather_bytes(self, b):
        out = [None] * self.world
        self.dist.all_gather_object(out, b)
        return out

    def all_ok(self, ok):
        return self.allreduce(1.0 if ok else 0.0, "min") > 0.5

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


class CpuBaseline:
    """The reference itself (oracle/_ref/ref_lbfgs: the reference's sequential sources compiled
    unmodified, -O2 -ffp-contract=off), one core, Rosenbrock, m, backtracking, x0 ~ U(-2,2) from
    std::mt19937(42), as BASELINE.md §3 prescribes: m + 2 iterations, the steady state is the mean
    of the iterations with h = m pairs. Per-iteration times come from the trace driver's grad()
    timestamps (each grad call also checksums x and takes |g|: 2 extra reads of ~8m + 11 vector
    passes, i.e. the CPU figure is ~2 % pessimistic).

    The runs start as child processes pinned (taskset) to host cores the benchmark process
    leaves alone, before the GPU work, and are collected after it: the GPU timing does not
    wait for them and they share no device or core with it. `pinned` records whether taskset
    worked; an unpinned run is reported as such, never silently."""

    def __init__(self, sizes, m):
        self.runs = []
        ref = os.path.join(ROOT, "oracle", "_ref", "ref_lbfgs")
        if not os.path.exists(ref):
            return
        try:
            cores = sorted(os.sched_getaffinity(0))
        except AttributeError:
            cores = list(range(os.cpu_count() or 1))
        self.tmp = tempfile.TemporaryDirectory()
        for j, n in enumerate(sizes):
            n = int(n)
            pre = os.path.join(self.tmp.name, f"cpu{j}")
            cmd = [ref, "rosenbrock", str(n), str(m), "backtracking", str(m + 2), "1e-5", "42", "-2", "2", pre, "0"]
            core = cores[j % len(cores)] if len(cores) > len(sizes) else None
            pinned = False
            if core is not None and shutil.which("taskset"):
                probe = subprocess.run(["taskset", "-c", str(core), "true"], capture_output=True)
                pinned = probe.returncode == 0
            full = (["taskset", "-c", str(core)] + cmd) if pinned else cmd
            p = subprocess.Popen(full, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            self.runs.append(dict(n=n, m=m, pre=pre, proc=p, core=core if pinned else None, pinned=pinned,
                                  t0=time.perf_counter()))
        # keep the benchmark's own threads off the reference's cores
        used = {r["core"] for r in self.runs if r["core"] is not None}
        rest = [c for c in cores if c not in used]
        if used and rest:
            try:
                os.sched_setaffinity(0, rest)
            except OSError:
                pass

    def collect(self, timeout=900):
        out = []
        for r in self.runs:
            p = r["proc"]
            try:
                p.wait(timeout=max(timeout - (time.perf_counter() - r["t0"]), 1))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
                out.append(dict(n=r["n"], error="timed out"))
                continue
            if p.returncode != 0:
                out.append(dict(n=r["n"], error=f"rc={p.returncode} {p.stderr.read().decode()[-200:]}"))
                continue
            g = np.fromfile(r["pre"] + ".g.bin", dtype=np.uint64).reshape(-1, 5)
            fcalls = np.fromfile(r["pre"] + ".f.bin", dtype=np.float64)
            t = g[:, 3].copy().view(np.float64)
            dt = np.diff(t)  # dt[k] = time of iteration k (grad call k -> k+1)
            steady = dt[r["m"]:]  # iterations with h = m
            # the reference's trajectory: grad call k is made at x_k (lbfgs.cpp:30,171; backtracking
            # calls grad nowhere else), right after f(x_k) (:29,160), the nf-th f call
            nf = g[:, 4].astype(np.int64)
            traj = dict(f=fcalls[nf - 1], gnorm=g[:, 2].copy().view(np.float64), c1=g[:, 0].copy(),
                        c2=g[:, 1].copy())
            out.append(dict(n=r["n"], per_iter_s=float(np.mean(steady)), iters_timed=len(steady),
                            total_s=float(t[-1]), pinned=r["pinned"], core=r["core"], trajectory=traj))
        for r in self.runs:
            if r["proc"].stderr:
                r["proc"].stderr.close()
        if self.runs:
            self.tmp.cleanup()
        return out


def ntag(n):
    """100000000 -> '1e8' (file tags of profiles/)."""
    e = len(str(n)) - 1
    return f"1e{e}" if n == 10 ** e else str(n)


def pmc_traffic(kernel, n, world):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary of this workload
    (profiles/<round>/pmc_bench_n<n>.json, produced by tools/pmc_summary.py from separate FETCH_SIZE
    and WRITE_SIZE passes, gfx950 FETCH_SIZE x2 correction applied), newest round first. Only a
    summary profiled on THIS library counts: its `_build.library` must carry the loaded library's
    source hash (lbfgs_build_info), else it describes other code and is refused.
    Returns (bytes per launch or None, source file or None, why a file was refused or None)."""
    import glob

    if world != 1:
        return None, None, None
    lib_src = L.build_info()[0].split()[0]  # "src=<hash>"
    refused = []
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"pmc_bench_n{ntag(n)}.json")))
    for fn in reversed(files):
        try:
            d = json.load(open(fn))
        except (OSError, ValueError):
            continue
        for k, v in d.items():
            if (k.startswith("k_" + kernel + "<") or k == "k_" + kernel) and "hbm_bytes_per_launch" in v:
                built = (d.get("_build") or {}).get("library", "")
                rel = os.path.relpath(fn, ROOT)
                if built.split(" ")[0] != lib_src:
                    refused.append(f"{rel}: profiled on {built.split(' ')[0] or 'an unrecorded library'}, "
                                   f"the loaded library is {lib_src}")
                    break
                return v["hbm_bytes_per_launch"], rel, None
    return None, None, "; ".join(refused) or None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def measure(a, D, n, x0, dev, rank, world, uid, unfused=False, vector_free=False, box_probe=False,
            defer_rccl=False):
    """W warm-up steps, then EXACTLY K timed steps (barrier + device sync on both sides, no
    instrumentation), then a separate event-instrumented pass for per-kernel durations.

    Every rank returns, or every rank raises LbfgsError: a failure on one rank (a mailbox wait
    that timed out, an allocation) is carried through the same sequence of gloo collectives the
    other ranks make - its compute is skipped, its collectives are not - to a vote that all ranks
    reach after each stage, so no rank is left in a collective its peers never enter. The context
    is closed on every path."""
    ctx, err = None, None
    try:
        ctx = L.Context(n, a.history, device=dev, rank=rank, world=world, uid=uid)
    except L.LbfgsError as e:
        err = e
    if not D.all_ok(err is None):
        if ctx is not None:
            ctx.close()
        raise err or L.LbfgsError("context creation failed on another rank")
    try:
        return _measure(a, D, ctx, x0, rank, world, uid, unfused, vector_free, box_probe, defer_rccl)
    finally:
        ctx.close()


def _measure(a, D, ctx, x0, rank, world, uid, unfused, vector_free, box_probe, defer_rccl=False):
    failed = []  # this rank's first failure (sticky: later compute is skipped, collectives are not)

    def run(fn, *args, **kw):
        if failed:
            return None
        try:
            return fn(*args, **kw)
        except L.LbfgsError as e:
            failed.append(e)
            print(f"rank {rank}: {e}", file=sys.stderr, flush=True)
            return None

    def vote(stage):
        if not D.all_ok(not failed):
            raise failed[0] if failed else L.LbfgsError(f"{stage} failed on another rank")

    if world > 1 and a.exchange in ("xgmi", "auto"):
        # the measurement's exchange path: the peer mailboxes alone (every wait bounded, 60 s); no
        # RCCL communicator exists yet (rccl_leg below creates one after the measurement)
        ok, msg = ctx.connect_peers(D.allgather_bytes, D.all_ok)  # collective, its own vote
        if msg:
            print(f"rank {rank}: {msg}", file=sys.stderr, flush=True)
        if not ok and uid is None:
            raise L.LbfgsError("xGMI peer exchange unavailable and no RCCL communicator")  # on every rank
    backend = ctx.backend + ("+fold" if world > 1 and ctx.backend == "xgmi" and ctx.folded else "")
    # the untimed history fill and warm-up record the trajectory (f, |g|, alpha, x checksums at
    # the top of every iteration) for reference_parity; the timed steps run untraced
    trace = not vector_free
    run(ctx.init, a.objective, x0, a.line_search, tolerance=1e-5, unfused=unfused, vector_free=vector_free,
        trace=trace)
    # history fill (untimed, not counted as warm-up): m iterations store m pairs, so every later
    # step uses h = m whatever --warmup is (B_iter grows with h)
    fill = run(ctx.step, a.history)
    warm = run(ctx.step, a.warmup)
    if trace:
        run(ctx.trace_enable, False)
    run(ctx.sync)
    vote("history fill / warm-up")
    D.barrier()
    run(ctx.sync)
    w0 = run(ctx.wait_stats)
    c0 = time.process_time()
    t0 = time.perf_counter()
    res = run(ctx.step, a.steps)
    run(ctx.sync)
    t_local = time.perf_counter() - t0
    cpu_local = time.process_time() - c0
    w1 = run(ctx.wait_stats)
    D.barrier()
    T = D.allreduce(t_local, "max")
    bytes_all = D.allreduce(res["bytes"] if res else 0.0, "sum")
    vote("timed steps")
    # this box's rate for the passes' 3 R + 1 W access pattern, on the same buffers, right after
    # the timed steps (bench lines from different boxes are compared against it)
    probe = None
    if box_probe and not a.no_box_probe and res["status"] == "running":
        probe = run(ctx.stream_probe, 20)
        mine = probe["gbps"] if probe and probe["gbps"] else 0.0
        gmin, gsum = D.allreduce(mine, "min"), D.allreduce(mine, "sum")
        vote("box probe")
        probe = dict(probe, gbps_min_over_ranks=gmin, gbps_sum_over_ranks=gsum) if probe else None
    # roofline region: the same kind of steps again with a HIP event pair around every launch
    # on the solver stream (per-kernel durations; the events add a few us per launch, which
    # is why they are kept out of the timed region above)
    prof = {}
    if not a.no_prof and res["status"] == "running":
        run(ctx.prof_reset)
        run(ctx.prof_enable, True)
        tp = time.perf_counter()
        run(ctx.step, min(a.steps, 20))
        run(ctx.sync)
        prof_wall_ms = (time.perf_counter() - tp) * 1e3
        run(ctx.prof_enable, False)
        for kname in L.KERNELS:
            p = run(ctx.prof_get, kname)
            if p and p["launches"]:
                prof[kname] = p
        # the GPU's busy share of those iterations: kernel time (exchange launches included) over
        # wall time; the rest is launch gaps, host decisions and waits (the events add a few us)
        kms = sum(p["ms"] for p in prof.values())
        prof["_busy"] = {"kernel_ms": round(kms, 3), "wall_ms": round(prof_wall_ms, 3),
                         "share": round(kms / max(prof_wall_ms, 1e-9), 4)}
        if world > 1:
            # the share of the (instrumented) iterations this rank spent in reduction exchanges,
            # waiting for its peers included; the max over ranks is reported
            ex = prof.get("exchange", {"ms": 0.0, "launches": 0})
            share = D.allreduce(ex["ms"] / max(prof_wall_ms, 1e-9), "max")
            prof["_exchange_share"] = {"share_max_over_ranks": round(share, 4),
                                       "rank0_ms": round(ex["ms"], 3), "rank0_exchanges": ex["launches"],
                                       "rank0_wall_ms": round(prof_wall_ms, 3),
                                       "iterations": min(a.steps, 20)}
        vote("profiled steps")
    # sharded: the cost of one reduction exchange on this machine, per backend available on
    # every rank (collective calls, same sequence everywhere): the two-loop issues ~2h + 3 of
    # them per iteration, each on the critical path
    lat = None
    if world > 1 and not vector_free and not unfused:
        lat = {}
        uid_leg = uid is not None
        if backend.startswith("xgmi") and uid is None and a.exchange == "auto" and not defer_rccl:
            # only now, with the measurement done: an RCCL communicator for the comparison leg
            lat["rccl_leg"] = rccl_leg(D, ctx, rank)
            uid_leg = lat["rccl_leg"]["ok"]
        backends = (["xgmi"] if backend.startswith("xgmi") else []) + (["rccl"] if uid_leg else [])
        exchange_timings(D, ctx, rank, backends, lat, failed)
        vote("exchange latency")
    if trace:
        res["trajectory"] = ctx.trace()
    # this process's host CPU over the timed steps (all its threads) and the time its completion-word
    # waits slept (LBFGS_WAIT)
    res["host"] = ({"cpu_s": round(cpu_local, 4), "cpu_share": round(cpu_local / max(t_local, 1e-9), 4),
                    "slept_share": round((w1["slept_s"] - w0["slept_s"]) / max(t_local, 1e-9), 4),
                    "waits": w1["waits"] - w0["waits"], "wait_mode": "adaptive" if w1["adaptive"] else "spin"}
                   if w0 and w1 else None)
    res["vector_fallbacks"] = run(lambda: ctx.vector_fallbacks)
    res["vector_pool"] = run(lambda: ctx.vector_pool)
    res["history_fill"] = fill["iterations"]
    res["warm_counters"] = {k: warm[k] for k in ("trials_f", "trials_fg", "commits", "passes")} if warm else None
    res["box_probe"] = probe
    done_steps = a.steps if res["status"] == "running" else max(res["iterations"] - a.warmup - fill["iterations"], 1)
    return T, res, prof, bytes_all, done_steps, (backend, lat)


def exchange_timings(D, ctx, rank, backends, lat, failed):
    """200 back-to-back exchanges of 8 and 96 doubles per backend into lat (collective: every rank
    makes the same calls); an RCCL wait is bounded in the library (LBFGS_RCCL_TIMEOUT), a stall
    costs its entry, and a failed RCCL timing on any rank stops every rank's RCCL timings"""
    for b in backends:
        for k in (8, 96):
            us = None
            try:
                us = ctx.exchange_latency(b, k, 200) if not failed else None
            except L.LbfgsError as e:
                if b != "rccl":
                    failed.append(e)
                lat[f"{b}_{k * 8}doubles_error"] = str(e)
                print(f"rank {rank}: {b} exchange timing: {e}", file=sys.stderr, flush=True)
            if b == "rccl" and not D.all_ok(us is not None):
                break  # a rank's RCCL timing failed: no rank enters another RCCL collective
            if us is not None:
                lat[f"{b}_{k * 8}doubles"] = round(us, 2)


def rccl_comparison(a, D, n, dev, rank, world):
    """The RCCL leg last (round 5): after every measurement of the run - the headline, the
    vector-free line, configs[4] - a fresh sharded context (no RCCL id, its vectors untouched)
    takes an RCCL communicator (rccl_leg) and times the RCCL exchanges beside the mailboxes'. On one
    card the init attempt of 8 processes (RCCL refuses two ranks on one device) left a later large
    solve at half speed; nothing measured comes after it now. Returns the entries
    for the headline's exchange_latency_us."""
    out, ctx, err = {}, None, None
    try:
        ctx = L.Context(n, a.history, device=dev, rank=rank, world=world, uid=None)
    except L.LbfgsError as e:
        err = str(e)
    if not D.all_ok(ctx is not None):
        if ctx is not None:
            ctx.close()
        return {"rccl_leg": {"ok": False, "errors": [err or "context creation failed on another rank"]}}
    try:
        out["rccl_leg"] = rccl_leg(D, ctx, rank)
        failed = []
        if out["rccl_leg"]["ok"]:
            exchange_timings(D, ctx, rank, ["rccl"], out, failed)
    finally:
        ctx.close()
    return out


RCCL_ABANDONED = False


def rccl_leg(D, ctx, rank):
    """Sharded, --exchange auto, after the measurement: an RCCL communicator for the comparison
    timing (lbfgs_rccl_attach: non-blocking init, bootstrap and self-test all-gather bounded by
    LBFGS_RCCL_TIMEOUT). A failure or stall on any rank is reported here and costs nothing else:
    the line has been measured on the mailboxes already. BENCH_RCCL_STALL=<rank> makes that rank
    skip the init (a peer that never joins: the other ranks' init must time out)."""
    t0 = time.perf_counter()
    err, mine = None, None
    if rank == 0:
        try:
            mine = L.unique_id()
        except L.LbfgsError as e:
            err = f"unique id: {e}"
    uid = D.broadcast_bytes(mine)  # every rank enters the broadcast (None: no id on rank 0)
    if uid is None and err is None:
        err = "rank 0 produced no RCCL unique id"
    stall = os.environ.get("BENCH_RCCL_STALL")
    if uid is not None:
        if stall is not None and int(stall) == rank:
            err = "BENCH_RCCL_STALL: this rank did not join the RCCL init"
        else:
            try:
                ctx.rccl_attach(uid)
            except L.LbfgsError as e:
                err = str(e)
    if err:
        print(f"rank {rank}: RCCL leg: {err}", file=sys.stderr, flush=True)
        if "abandoned" in err:  # an RCCL thread still waits in its bootstrap: main() ends with os._exit
            global RCCL_ABANDONED
            RCCL_ABANDONED = True
    ok = D.all_ok(err is None)
    errs = [e for e in D.allgather_bytes(err or "") if e]
    return {"ok": ok, "init_s": round(time.perf_counter() - t0, 2),
            "errors": errs[:4] or None,
            "note": "RCCL communicator created after every measurement of the run (non-blocking init, bounded wait)"}


def shard_check(a, D, n, x0, dev, rank, world, res):
    """Sharded runs: rank 0 repeats the measured solve on its GPU alone (world = 1, the same
    fill, warm-up and timed step counts) and compares f and |g| bit for bit with the sharded
    result. The canonical reduction order is a function of n only, so every
    exchange path must reproduce the one-GPU trajectory exactly; this checks it on the node the
    scaling series runs on. The other ranks wait at a barrier."""
    out = None
    if rank == 0:
        try:
            t0 = time.perf_counter()
            with L.Context(n, a.history, device=dev) as c:
                c.init(a.objective, x0, a.line_search, tolerance=1e-5, unfused=a.unfused,
                       vector_free=a.vector_free)
                c.step(a.history)
                c.step(a.warmup)
                r1 = c.step(a.steps)
            bits = lambda v: struct.pack("<d", v).hex()  # noqa: E731
            same = bits(r1["f"]) == bits(res["f"]) and bits(r1["gnorm"]) == bits(res["gnorm"])
            out = {"one_gpu_f": r1["f"], "one_gpu_gnorm": r1["gnorm"], "iterations": r1["iterations"],
                   "bit_identical": bool(same and r1["iterations"] == res["iterations"]),
                   "seconds": round(time.perf_counter() - t0, 2)}
        except L.LbfgsError as e:
            out = {"error": str(e)}
    D.barrier()
    return out


def config4(a, D, dev, rank, world):
    """BASELINE configs[4]: Rosenbrock n = 1e9, m = 10, sharded over 8 GPUs, default mode, the
    xGMI peer exchange (no RCCL communicator: a rank that fails early cannot strand the others in
    a collective init). Every rank generates the full x0 (std::mt19937(42), as everywhere) and
    uploads its slice. Like the headline, m untimed iterations fill the history before the
    warm-up, so every timed step has h = m. Each step that can fail is followed by a gloo vote,
    so all ranks skip together. Then rank 0 repeats the solve on its GPU alone (n = 1e9 is 240 GB
    resident, which fits one MI355X) and compares f, |g| and the iteration count bit for bit
    (`shard_check`, as for the n = 1e8 line)."""
    n9 = 10 ** 9
    t0 = time.perf_counter()
    try:
        x0 = L.x0_uniform(n9, 42, -2.0, 2.0)
    except MemoryError:
        x0 = None
    if not D.all_ok(x0 is not None):
        return {"skipped": "x0 allocation failed on a rank"}
    gen_s = time.perf_counter() - t0
    ctx, err = None, None
    try:
        ctx = L.Context(n9, a.history, device=dev, rank=rank, world=world, uid=None)
    except L.LbfgsError as e:
        err = str(e)
    if not D.all_ok(ctx is not None):
        if ctx:
            ctx.close()
        return {"skipped": f"context creation failed on a rank ({err})"}
    ok, msg = ctx.connect_peers(D.allgather_bytes, D.all_ok)
    if not ok:
        ctx.close()
        return {"skipped": f"xGMI peer exchange unavailable ({msg})"}
    folded = ctx.folded
    res, T, err, fill = None, None, None, None
    try:
        ctx.init(a.objective, x0, a.line_search, tolerance=1e-5)
        fill = ctx.step(a.history)
        ctx.step(a.warmup)
        ctx.sync()
    except L.LbfgsError as e:
        err = str(e)
    if D.all_ok(err is None):
        D.barrier()
        t1 = time.perf_counter()
        try:
            res = ctx.step(a.steps)
            ctx.sync()
        except L.LbfgsError as e:
            err = str(e)
        t_local = time.perf_counter() - t1
        D.barrier()
        T = D.allreduce(t_local, "max")
        bytes_all = D.allreduce(res["bytes"] if res else 0.0, "sum")
    ok = D.all_ok(err is None and res is not None)
    ctx.close()  # every rank frees its shard before rank 0's one-GPU check
    if not ok:
        return {"skipped": f"solve failed on a rank ({err})"}
    D.barrier()
    if rank != 0:
        del x0
    check = shard_check(a, D, n9, x0 if rank == 0 else None, dev, rank, world, res)
    fill_n = fill["iterations"] if fill else 0
    steps = a.steps if res["status"] == "running" else max(res["iterations"] - a.warmup - fill_n, 1)
    return {"workload": f"{a.objective} n=1e9 m={a.history} {a.line_search}, sharded over {world} GPUs "
                        "(BASELINE configs[4])",
            "value": round(steps / T, 4), "unit": "iters/s", "steps": steps, "warmup": a.warmup,
            "history_fill": fill_n, "h_min": res.get("h_min", -1), "h_max": res.get("h_max", -1),
            "steady_state": res.get("h_min", -1) == a.history,
            "ms_per_step": round(T / steps * 1e3, 4), "achieved_hbm_gbps": round(bytes_all / T / 1e9, 1),
            "exchange": "xgmi+fold" if folded else "xgmi", "x0_generation_s": round(gen_s, 1),
            "solver": {"status": res["status"], "f": res["f"], "gnorm": res["gnorm"]},
            "shard_check": check}


FULLSIZE = os.path.join(ROOT, "tests", "golden", "fullsize")
PARITY_TOL = 1e-10  # BASELINE.json north star: within 1e-10 relative on fp64


def fullsize_fixture(a, n):
    """The committed full-size fixture of this workload (tests/golden/make_fullsize.py: the
    reference's own trace and the canonical-order oracle's, generated where the reference
    lives), or (None, None). Data only: nothing under oracle/ is loaded here."""
    import glob

    for fn in sorted(glob.glob(os.path.join(FULLSIZE, "*.json"))):
        try:
            d = json.load(open(fn))
        except (OSError, ValueError):
            continue
        # (fixtures of other shapes, e.g. the CUDA-mode cases file, have no single method)
        keys = ("objective", "n", "m", "method", "seed", "lo", "hi")
        if tuple(d.get(k) for k in keys) == (a.objective, n, a.history, a.line_search, 42, -2.0, 2.0):
            return d, os.path.relpath(fn, ROOT)
    return None, None


def reference_parity(traj, live, fixture, fsrc):
    """The measured run's own trajectory (the traced history fill and warm-up: f, |g|, alpha and
    the x checksums at the top of every iteration) against
      * the reference: the live run of the CPU baseline on this host (N = 1), else the
        fixture's trace of the reference itself; f and |g| within 1e-10 relative
        (lbfgs.cpp:72-199 on benchmark.cpp:58-81), and the first k where that fails;
      * the canonical-order oracle (the fixture): bit for bit."""
    if traj is None or (live is None and fixture is None):
        return None
    gf, gg = np.asarray(traj["tr_f"]), np.asarray(traj["tr_gnorm"])
    out = {"tolerance": PARITY_TOL, "gpu_iterations_traced": int(len(gf))}
    u64 = lambda xs: np.array([int(v) for v in xs], dtype=np.uint64)  # noqa: E731
    f64 = lambda hs: np.array([int(h, 16) for h in hs], dtype=np.uint64).view(np.float64)  # noqa: E731
    if live is not None:
        rf, rg, rc1, rc2 = live["f"], live["gnorm"], live["c1"], live["c2"]
        out["reference"] = "live: oracle/_ref/ref_lbfgs (the reference's sources) on this host, the CPU baseline run"
        if fixture is not None:  # the box's build of the reference against the committed trace of it
            fr = fixture["reference"]
            k = min(len(fr["grad_norm"]), len(rg))
            out["live_reference_matches_fixture"] = bool(
                np.array_equal(f64(fr["grad_norm"])[:k].view(np.uint64), rg[:k].view(np.uint64))
                and np.array_equal(u64(fr["grad_c1"])[:k], rc1[:k]))
    elif "seq" in fixture:
        s = fixture["seq"]
        rf, rg, rc1, rc2 = f64(s["f"]), f64(s["gnorm"]), u64(s["c1"]), u64(s["c2"])
        out["reference"] = f"fixture: {fsrc} (the reference's own trace, tests/golden/make_fullsize.py)"
    else:  # the reference at x0 only (configs[4]'s fixture: maxit 0, f and grad at x0)
        r = fixture["reference"]
        rf, rg = f64(r["f_calls"][:1]), f64(r["grad_norm"][:1])
        rc1, rc2 = u64(r["grad_c1"][:1]), u64(r["grad_c2"][:1])
        out["reference"] = f"fixture: {fsrc} (the reference's f and grad at x0, tests/golden/make_fullsize.py)"
    k = min(len(gf), len(rf))
    rel_f = np.abs(gf[:k] - rf[:k]) / np.maximum(np.abs(rf[:k]), 1e-300)
    rel_g = np.abs(gg[:k] - rg[:k]) / np.maximum(np.abs(rg[:k]), 1e-300)
    bad_f, bad_g = np.nonzero(rel_f > PARITY_TOL)[0], np.nonzero(rel_g > PARITY_TOL)[0]
    hf = int(bad_f[0]) if len(bad_f) else int(k)  # leading iterations within tolerance
    hg = int(bad_g[0]) if len(bad_g) else int(k)
    same_x = np.nonzero((np.asarray(traj["tr_c1"])[:k] != rc1[:k]) | (np.asarray(traj["tr_c2"])[:k] != rc2[:k]))[0]
    out.update(iterations_compared=int(k), max_rel_f=float(rel_f.max()) if k else None,
               max_rel_gnorm=float(rel_g.max()) if k else None,
               first_divergent_k=min(hf, hg) if min(hf, hg) < k else None,
               within_tolerance_iterations={"f": hf, "gnorm": hg},
               x_bit_identical_iterations=int(same_x[0]) if len(same_x) else int(k))
    # The bar: no parallel summation order can match the reference's left-to-right sums
    # indefinitely; the fixture records how many leading iterations the
    # reference itself keeps within 1e-10 under another equally valid order (K_ref). The run
    # passes when its own horizon reaches K_ref (capped at the iterations compared); without a
    # fixture every compared iteration must be within tolerance.
    kref = (fixture or {}).get("horizons", {}).get("ref")
    if kref:
        need_f, need_g = min(int(kref[0]), k), min(int(kref[1]), k)
        out["reference_self_horizon"] = {"f": int(kref[0]), "gnorm": int(kref[1])}
    else:
        need_f = need_g = k
    ok = k > 0 and hf >= need_f and hg >= need_g
    if fixture is not None:
        c = fixture["canon"]
        kc = min(len(gf), len(c["f"]))
        ta = np.asarray(traj["tr_alpha"])[:kc - 1]  # the canonical trace's last entry has no step
        exact = bool(np.array_equal(gf[:kc].view(np.uint64), f64(c["f"])[:kc].view(np.uint64))
                     and np.array_equal(gg[:kc].view(np.uint64), f64(c["gnorm"])[:kc].view(np.uint64))
                     and np.array_equal(ta.view(np.uint64), f64(c["alpha"])[:kc - 1].view(np.uint64))
                     and np.array_equal(np.asarray(traj["tr_c1"])[:kc], u64(c["c1"])[:kc])
                     and np.array_equal(np.asarray(traj["tr_c2"])[:kc], u64(c["c2"])[:kc]))
        out["canonical"] = {"fixture": fsrc, "iterations_compared": int(kc), "bit_exact": exact}
        ok = ok and exact
    out["ok"] = bool(ok)
    return out


def survey_bytes(res, n, a, steps, T):
    """SURVEY.md 8(d)'s algorithmic bytes per iteration, B_iter = 8 n (8h + 2 T_f + 3 T_g + 9), over
    the timed steps: h = the pairs in use (m in the steady state), T_f / T_g the line-search
    evaluations per iteration that read x and d (f only / f and g.d), counted per pass: the first
    trial, which the commit pass takes (T_g for the Wolfe searches, T_f otherwise), plus the extra
    trial passes the solver counted over the timed steps (a batched pass evaluating up to 4 halving
    steps in one read of x and d counts once). Beside it the line keeps the solver's own count
    (bytes_per_step: 8n per vector pass actually issued)."""
    w = res.get("warm_counters")
    if not w or steps < 1 or res.get("h_min", -1) != res.get("h_max", -2):
        return {}
    wolfe = a.line_search in ("wolfe", "backtracking_wolfe")
    tf = (res["trials_f"] - w["trials_f"]) / steps + (0 if wolfe else 1)
    tg = (res["trials_fg"] - w["trials_fg"]) / steps + (1 if wolfe else 0)
    h = res["h_max"]
    b = 8.0 * n * (8 * h + 2 * tf + 3 * tg + 9)
    return {"bytes_per_step_survey": b, "achieved_hbm_gbps_survey": round(b * steps / T / 1e9, 1),
            "survey_bytes_terms": {"formula": "8n(8h + 2T_f + 3T_g + 9), SURVEY.md 8(d)", "h": h,
                                   "T_f": round(tf, 4), "T_g": round(tg, 4)}}


def box_fields(probe, value, achieved_gbps, world):
    """This box's HBM rate for the two-loop passes' access pattern (lbfgs_stream_probe: 20 launches
    of a 3 R + 1 W stream over the solver's own q, y, s in the passes' geometry and cache policy,
    right after the timed steps, every rank at once) and the line's value against it, so lines
    from different boxes compare by the code rather than by the box. The box rate
    of a sharded line is the sum of its ranks' concurrent probes: the aggregate of N GPUs, or the
    one card's rate when the ranks share it (a rehearsal)."""
    if not probe or not probe.get("gbps"):
        return {"box_copy_tbps": None}
    gb = probe.get("gbps_sum_over_ranks") or probe["gbps"]
    return {"box_copy_tbps": round(gb / 1e3, 4),
            "value_per_box_tbps": round(value / (gb / 1e3), 4),
            "hbm_frac_of_box": round(achieved_gbps / gb, 4),
            "box_probe": {"kernel": "k_probe_stream (3 R + 1 W, k_axpy_dot's loads and store, no stage 2; "
                                    "another history pair every launch, as the passes; the written vector "
                                    "holds random data, a copy of y_0: zeros stream ~3 % faster)",
                          "avg_launch_us": round(probe["avg_launch_us"], 2), "launches": 20,
                          "bytes_per_launch": probe["bytes_per_launch"],
                          "rank0_gbps": round(probe["gbps"], 1),
                          "slowest_rank_gbps": round(probe.get("gbps_min_over_ranks") or probe["gbps"], 1),
                          "over": f"sum of {world} ranks' concurrent probes" if world > 1 else "one GPU"}}


def roofline(prof, n, world):
    prof = {k: v for k, v in (prof or {}).items() if not k.startswith("_")}
    streaming = [k for k in prof if prof[k]["bytes"] > 0]  # not the stage-2 / exchange launches
    if not streaming:
        return None
    dom = max(streaming, key=lambda k: prof[k]["ms"])
    p = prof[dom]
    avg_s = p["ms"] / p["launches"] / 1e3
    per_launch = p["bytes"] / p["launches"]  # this rank's algorithmic bytes per launch
    achieved = per_launch / avg_s / 1e9
    traffic, tsrc, trefused = pmc_traffic(dom, n, world)
    tot = sum(q["ms"] for q in prof.values())
    # every streaming kernel's own rate (algorithmic bytes / event-timed duration), for A/B lines
    rates = {k: {"avg_launch_us": round(prof[k]["ms"] / prof[k]["launches"] * 1e3, 2),
                 "gbps": round(prof[k]["bytes"] / (prof[k]["ms"] / 1e3) / 1e9, 1)}
             for k in streaming if prof[k]["launches"] and prof[k]["ms"] > 0}
    return dict(bound="hbm", kernel=dom, achieved=round(achieved, 1), peak=HBM_PEAK_GBPS, unit="GB/s",
                frac=round(achieved / HBM_PEAK_GBPS, 4), traffic=traffic, traffic_unit="bytes/launch",
                traffic_source=tsrc, traffic_refused=trefused, bytes_per_launch=per_launch, avg_launch_us=round(avg_s * 1e6, 2),
                launches=p["launches"], kernel_share={k: round(v["ms"] / tot, 4) for k, v in prof.items()},
                kernel_rates=rates)


def vectors_info(res):
    """how the timed context's vectors were allocated (LBFGS_VEC_ALLOC)"""
    vp = res.get("vector_pool")
    mode, pooled, held = vp if isinstance(vp, (tuple, list)) else (None, None, None)
    what = {"pool": "physically contiguous vectors (hipDeviceMallocContiguous) from a process-wide pool that "
                    "never returns them to the driver (64 MiB .. 2 GiB vectors; others plain hipMalloc)",
            "plain": "plain hipMalloc per vector",
            "contiguous": "physically contiguous per vector, freed with hipFree (A/B only)"}.get(mode)
    return {"mode": mode, "allocation": what, "pooled_vectors": pooled, "pool_gib": round(held, 2) if held else held,
            "contiguous_fallbacks": res.get("vector_fallbacks")}


def main():
    a = parse()
    if a.gpus > 1 and "RANK" not in os.environ:
        # no launcher around the command: bench.py starts the ranks itself, before any HIP call
        sys.exit(self_launch(sys.argv[1:], a.gpus, a.launch_timeout))
    # load liblbfgs_hip.so (and through it /opt/rocm's HIP runtime and RCCL) before torch can load
    # its bundled copies: libraries with the same soname are then shared, not duplicated
    L.lib()
    if a.persistent:  # read by every context this process creates (lbk_create)
        os.environ["LBFGS_PERSIST"] = "2"
    n = int(a.size)
    D = Dist(a.gpus)
    world, rank = a.gpus, D.rank
    # sharded: no RCCL communicator before the measurement (the mailboxes carry it; --exchange rccl
    # or a mailbox failure creates one, non-blocking with a bounded wait, inside the library).
    # BENCH_DEVICE_MOD (several ranks on one GPU) cannot measure over RCCL: RCCL refuses two ranks
    # on one device (its comparison leg then reports that refusal)
    rehearsal = "BENCH_DEVICE_MOD" in os.environ
    need_uid = world > 1 and a.exchange == "rccl"
    uid = D.broadcast_bytes(L.unique_id() if (need_uid and rank == 0) else None) if need_uid else None

    # the reference on host cores, started first and collected after the GPU work (rank 0, N=1)
    cpu_runs = None
    if world == 1 and rank == 0 and not a.no_cpu_baseline:
        sizes = [int(a.cpu_n) if a.cpu_n else n] + ([int(a.cpu_n2)] if a.cpu_n2 else [])
        cpu_runs = CpuBaseline(sizes, a.history)

    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    # BENCH_DEVICE_MOD=k maps rank -> device local_rank % k (rehearsing several ranks on fewer GPUs)
    # a launcher that exposes one device per process (HIP_VISIBLE_DEVICES) leaves local_rank >= count
    ndev = max(L.device_count(), 1)
    dev = D.local_rank % int(os.environ["BENCH_DEVICE_MOD"]) if "BENCH_DEVICE_MOD" in os.environ else D.local_rank
    if dev >= ndev:
        dev = dev % ndev
    fallback = None
    try:
        T, res, prof, bytes_all, done_steps, (backend, xlat) = measure(a, D, n, x0, dev, rank, world, uid,
                                                      unfused=a.unfused, vector_free=a.vector_free, box_probe=True,
                                                      defer_rccl=True)
    except L.LbfgsError as e:
        # a mailbox failure across GPUs: measure() raises on every rank together (its votes), so
        # every rank lands here and the line is measured again over RCCL rather than lost, and
        # says why
        if not (world > 1 and uid is None and a.exchange in ("xgmi", "auto") and not rehearsal):
            raise
        fallback = f"xgmi: {e}"
        print(f"rank {rank}: {fallback}; measuring again over RCCL", file=sys.stderr, flush=True)
        import copy

        a = copy.copy(a)
        a.exchange = "rccl"
        uid = D.broadcast_bytes(L.unique_id() if rank == 0 else None)
        need_uid = True
        T, res, prof, bytes_all, done_steps, (backend, xlat) = measure(a, D, n, x0, dev, rank, world, uid,
                                                      unfused=a.unfused, vector_free=a.vector_free, box_probe=True)
    check = shard_check(a, D, n, x0, dev, rank, world, res) if world > 1 else None
    # the opt-in vector-free mode alongside the default (outside the bit-parity contract with
    # the reference's operation order); sharded runs over RCCL need a fresh id
    vf = None
    if not (a.unfused or a.vector_free or a.no_vector_free) and a.history <= 20:
        # a failure here is deterministic across ranks (same arguments everywhere) and must not
        # cost the headline line above
        try:
            uid2 = D.broadcast_bytes(L.unique_id() if rank == 0 else None) if need_uid else None
            Tv, rv, pv, bv, dv, _ = measure(a, D, n, x0, dev, rank, world, uid2, vector_free=True)
            vf = dict(value=round(dv / Tv, 4), ms_per_step=round(Tv / dv * 1e3, 4), steps=dv,
                      achieved_hbm_gbps=round(bv / Tv / 1e9, 1), roofline=roofline(pv, n, world),
                      solver={"status": rv["status"], "f": rv["f"], "gnorm": rv["gnorm"],
                              "trials_f": rv["trials_f"], "commits": rv["commits"], "passes": rv["passes"]},
                      parity=("bit-exact vs the oracle's restatement (ORC_CANON_VF); f and |g| within "
                              "1e-10 of the reference over the same horizons as the default mode "
                              "(tests/test_gpu_vector_free.py)"))
        except L.LbfgsError as e:
            vf = {"error": str(e)}
    # BASELINE configs[2] names the "fused persistent-block two-loop": the same steps with the
    # two-loop's 2h - 1 passes in one resident launch per iteration (k_persist_twoloop,
    # LBFGS_PERSIST=2; one GPU), beside the launch sequence on the same box, with its trajectory
    # checked bit for bit against the default run's
    pers = None
    if world == 1 and not (a.unfused or a.vector_free or a.no_persistent or a.persistent):
        prev = os.environ.get("LBFGS_PERSIST")
        os.environ["LBFGS_PERSIST"] = "2"
        try:
            Tp, rp, pp, bp, dp, _ = measure(a, D, n, x0, dev, rank, world, None)
            same = None
            if res.get("trajectory") is not None and rp.get("trajectory") is not None:
                ta, tb = res["trajectory"], rp["trajectory"]
                k = min(len(ta["tr_f"]), len(tb["tr_f"]))
                same = bool(k > 0 and all(np.array_equal(ta[key][:k].view(np.uint64), tb[key][:k].view(np.uint64))
                                          for key in ("tr_f", "tr_gnorm", "tr_c1", "tr_c2")))
            pers = dict(value=round(dp / Tp, 4), ms_per_step=round(Tp / dp * 1e3, 4), steps=dp,
                        vs_default=round((dp / Tp) / (done_steps / T), 4),
                        achieved_hbm_gbps=round(bp / Tp / 1e9, 1), roofline=roofline(pp, n, world),
                        kernel="k_persist_twoloop (LBFGS_PERSIST=2): the 2h - 1 two-loop passes in one launch",
                        launches_persistent=(pp.get("small_iter") or {}).get("launches"),
                        trajectory_bit_identical_to_default=same,
                        solver={"status": rp["status"], "f": rp["f"], "gnorm": rp["gnorm"], "passes": rp["passes"]})
        except L.LbfgsError as e:
            pers = {"error": str(e)}
        finally:
            if prev is None:
                os.environ.pop("LBFGS_PERSIST", None)
            else:
                os.environ["LBFGS_PERSIST"] = prev
    del x0
    c4 = None
    if world == 8 and n == 10 ** 8 and not (a.unfused or a.vector_free or a.no_config4):
        c4 = config4(a, D, dev, rank, world)
    # the RCCL comparison leg after everything measured (rccl_comparison)
    if xlat is not None and fallback is None and backend.startswith("xgmi") and uid is None and a.exchange == "auto":
        xlat.update(rccl_comparison(a, D, n, dev, rank, world))

    out = None
    if rank == 0:
        value = done_steps / T
        roof = roofline(prof, n, world)
        cpu, cbs = None, None
        if cpu_runs is not None:
            cbs = cpu_runs.collect()
            main_cb = cbs[0] if cbs else None
            if main_cb and "per_iter_s" in main_cb:
                scale = n / main_cb["n"]
                cpu = dict(value=round(1.0 / (main_cb["per_iter_s"] * scale), 6), unit="iters/s", cores=1,
                           kind="reference", pinned=main_cb["pinned"],
                           sample=(f"reference sequential LBFGS (oracle/_ref, its sources compiled -O2 "
                                   f"-ffp-contract=off), Rosenbrock n={main_cb['n']:.0e} m={a.history} "
                                   f"backtracking, {a.history + 2} iterations, mean of the "
                                   f"{main_cb['iters_timed']} with h=m = {main_cb['per_iter_s']:.3f} s/iter"
                                   + (f" (scaled x{scale:g} linearly in n to n={n:.0e})" if scale != 1 else
                                      " (measured directly at the benchmark's n)")
                                   + f"; {'pinned to core ' + str(main_cb['core']) if main_cb['pinned'] else 'NOT pinned'}"
                                   f", 1 thread, of {os.cpu_count()} cores ({cpu_model()})"),
                           per_iter_s=main_cb["per_iter_s"], total_s=round(main_cb["total_s"], 2),
                           secondary=[dict(n=c["n"], per_iter_s=c.get("per_iter_s"), pinned=c.get("pinned"),
                                           error=c.get("error")) for c in cbs[1:]])
            elif cbs:
                cpu = {"error": cbs[0].get("error", "no result")}
        live = None
        if cpu_runs is not None and cbs and "trajectory" in cbs[0] and cbs[0]["n"] == n and \
                a.objective == "rosenbrock" and a.line_search == "backtracking":
            live = cbs[0]["trajectory"]
        fixture, fsrc = fullsize_fixture(a, n)
        parity = reference_parity(res.get("trajectory"), live, fixture, fsrc)
        h_min, h_max = res.get("h_min", -1), res.get("h_max", -1)
        out = {
            "metric": f"L-BFGS iters/sec (n={ntag(n)} {a.objective.capitalize()}, m={a.history}, fp64)",
            "value": round(value, 4),
            "unit": "iters/s",
            "n_gpus": world,
            "steps": done_steps,
            "warmup": a.warmup,
            "history_fill": res["history_fill"],
            "h_min": h_min,
            "h_max": h_max,
            "steady_state": h_min == a.history,
            "ms_per_step": round(T / done_steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: x0 ~ U(-2,2) from std::mt19937(42), as the reference's main.cpp",
            "config": {"workload": (f"{a.objective} n={n:.0e} m={a.history} {a.line_search}, "
                                    f"{'sharded over ' + str(world) + ' GPUs' if world > 1 else 'one GPU'}"
                                    + (", unfused per-vector kernels" if a.unfused else
                                       ", vector-free (Gram-matrix) mode" if a.vector_free else
                                       ", persistent-block fused two-loop" if a.persistent else ", fused passes")
                                    + (" (BASELINE configs[2])" if n == 10 ** 8 else "")),
                       "kernels": ("unfused" if a.unfused else "vector_free" if a.vector_free else
                                   "persistent" if a.persistent else "fused"),
                       "n": n, "m": a.history, "line_search": a.line_search,
                       "parallelism": f"shard{world}" if world > 1 else "single",
                       "exchange": backend},
            "achieved_hbm_gbps": round(bytes_all / T / 1e9, 1),
            "bytes_per_step": bytes_all / max(done_steps, 1),
            "bytes_per_step_note": "the solver's own count: 8n per vector read or written by the passes it issued",
            **survey_bytes(res, n, a, done_steps, T),
            "roofline": roof,
            **box_fields(res.get("box_probe"), value, bytes_all / T / 1e9, world),
            "exchange_latency_us": xlat,
            "exchange_share": prof.get("_exchange_share"),
            "exchange_fallback": fallback,
            "kernel_busy": prof.get("_busy"),
            "host": res.get("host"),
            "vectors": vectors_info(res),
            "cpu_baseline": cpu,
            "reference_parity": parity,
            "solver": {"status": res["status"], "f": res["f"], "gnorm": res["gnorm"],
                       "trials_f": res["trials_f"], "commits": res["commits"],
                       "passes": res["passes"]},
            "shard_check": check,
            "vector_free": vf,
            "persistent": pers,
            "config4_n1e9": c4,
            "build": dict(zip(("library", "tree_sources", "current"), L.build_info())),
        }
        print(json.dumps(out), flush=True)
    D.close()
    if RCCL_ABANDONED:
        # an abandoned RCCL bootstrap thread could hold the interpreter's teardown: every context is
        # closed and the line printed, so the process ends here
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


if __name__ == "__main__":
    main()
