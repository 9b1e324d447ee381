"""bench.py's sharded line survives an RCCL problem, on the CPU: two gloo
ranks run bench.measure() over a stub Context that records every call. The measurement runs on
the peer mailboxes with no RCCL communicator; the communicator is created only afterwards
(rccl_leg), and a failed or stalled init there is reported in the line instead of losing it:
no rank enters an RCCL exchange unless every rank's init succeeded. As main() runs it (`_late`),
the leg comes after every measurement of the run, on a context of its own (rccl_comparison)."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class StubContext:
    """lbfgs_amd.Context's surface as measure() uses it; records the call order"""

    log = []
    attach_error = None  # rank-local: the message rccl_attach raises (a failed / timed-out init)

    def __init__(self, n, m=10, device=0, rank=0, world=1, uid=None, group=None):
        self.rank, self.uid, self.attached, self.k = rank, uid, False, 0
        StubContext.log.append(("create", uid is not None))

    def connect_peers(self, allgather, agree):
        allgather(b"h" * 64)
        StubContext.log.append(("connect_peers",))
        return agree(True), None

    backend = "xgmi"
    folded = True

    def init(self, *a, **kw):
        StubContext.log.append(("init",))

    def step(self, k):
        StubContext.log.append(("step", k))
        self.k += k
        return dict(iterations=self.k, status="running", f=1.0, gnorm=1.0, trials_f=0, trials_fg=0,
                    commits=self.k, passes=83 * self.k, bytes=8.0e8 * 83 * k, h_min=10, h_max=10)

    def trace_enable(self, on):
        pass

    def sync(self):
        pass

    def stream_probe(self, launches):
        return dict(avg_launch_us=500.0, bytes_per_launch=3.2e9, gbps=6400.0)

    def wait_stats(self):
        return dict(slept_s=0.0, waits=0, adaptive=True)

    vector_fallbacks = 0
    vector_pool = ("pool", 0, 0.0)

    def prof_reset(self):
        pass

    def prof_enable(self, on):
        pass

    def prof_get(self, kind):
        return dict(ms=0.0, launches=0, bytes=0.0)

    def rccl_attach(self, uid):
        import lbfgs_amd as L

        StubContext.log.append(("rccl_attach",))
        if StubContext.attach_error:
            raise L.LbfgsError(StubContext.attach_error)
        self.attached = True

    def exchange_latency(self, backend, k, iters):
        StubContext.log.append(("exchange_latency", backend))
        if backend == "rccl" and not self.attached:
            raise AssertionError("RCCL exchange without a communicator on this rank")
        return 3.0

    def trace(self):
        return {}

    def close(self):
        StubContext.log.append(("close",))


def _worker(rank, world, port, mode_arg, q):
    mode = mode_arg
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    os.environ.pop("BENCH_RCCL_STALL", None)
    mode = mode.replace("_late", "") if mode.endswith("_late") else mode
    if mode == "stall":
        os.environ["BENCH_RCCL_STALL"] = "0"  # rank 0 never joins; rank 1's bounded init times out
        if rank == 1:
            StubContext.attach_error = "ncclCommInitRankConfig: no progress in 60 s (RCCL communicator aborted)"
    elif mode == "fail" and rank == 1:
        StubContext.attach_error = "ncclCommInitRankConfig: invalid usage (RCCL communicator aborted)"
    sys.path.insert(0, ROOT)
    import bench

    bench.L.Context = StubContext
    bench.L.unique_id = lambda: bytes(128)
    a = bench.parse(["--gpus", str(world), "--steps", "5", "--warmup", "2"])
    D = bench.Dist(world)
    late = mode_arg.endswith("_late")
    T, res, prof, bytes_all, steps, (backend, lat) = bench.measure(a, D, 10 ** 8, None, 0, rank, world, None,
                                                                   defer_rccl=late)
    if late:  # main()'s order: the leg after every measurement, on a context of its own
        StubContext.log.append(("measurements done",))
        lat.update(bench.rccl_comparison(a, D, 10 ** 8, 0, rank, world))
    D.close()
    q.put((rank, StubContext.log, backend, lat, steps))


def _run(mode, world=2):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return out


@pytest.mark.parametrize("mode", ["ok", "fail", "stall", "ok_late", "fail_late", "stall_late"])
def test_rccl_created_after_the_measurement(mode):
    out = _run(mode)
    late = mode.endswith("_late")
    mode = mode.replace("_late", "")
    for rank, log, backend, lat, steps in out:
        assert backend == "xgmi+fold" and steps == 5
        assert log[0] == ("create", False)  # the measurement's context has no RCCL id
        timed = log.index(("step", 5))
        joined = ("rccl_attach",) in log
        assert joined == (mode != "stall" or rank != 0)
        if joined:
            assert log.index(("rccl_attach",)) > timed  # the communicator only after the timed steps
        if late:  # ... and, as main() runs it, only after every measurement, on its own context
            done = log.index(("measurements done",))
            assert log[done + 1] == ("create", False)
            assert all(e != ("rccl_attach",) for e in log[:done])
            assert log[-1] == ("close",)
        rccl_timings = [e for e in log if e == ("exchange_latency", "rccl")]
        leg = lat["rccl_leg"]
        if mode == "ok":
            assert leg["ok"] and leg["errors"] is None and len(rccl_timings) == 2
            assert "rccl_64doubles" in lat
        else:
            # any rank's failure or stall: reported, no rank enters an RCCL exchange, the line stands
            assert not leg["ok"] and len(leg["errors"]) >= 1 and rccl_timings == []
            assert "xgmi_64doubles" in lat and "rccl_64doubles" not in lat
        if mode == "stall":
            assert any("BENCH_RCCL_STALL" in e for e in leg["errors"])
            assert any("no progress" in e for e in leg["errors"])
