"""CPU tests of the multi-rank path that need no GPU: the shard plan (contiguous slices that
partition [0, n) along canonical segment/group boundaries, so the reduction order is the same
for 1, 2, 4 and 8 ranks) and bench.py's torch.distributed (gloo) bootstrap with 2 processes."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402
import oracle_lib as O  # noqa: E402


@pytest.mark.parametrize("n", [4_000_003, 10_000_000, 100_000_000, 1_000_000_000, 123_456_789])
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_shard_plan_partitions_along_groups(n, world):
    Lseg, nseg = O.geometry(n)
    prev = 0
    for r in range(world):
        lo, nl = L.shard_range(n, r, world)
        assert lo == prev and nl > 0
        assert lo % Lseg == 0  # a shard starts on a canonical segment boundary...
        g_lo = r * (8 // world)
        assert lo == min(g_lo * 1024 * Lseg, n)  # ...and on its first group's boundary
        prev = lo + nl
    assert prev == n


def test_shard_plan_rejects_empty_ranks():
    with pytest.raises(L.LbfgsError):
        L.shard_range(10_000, 1, 2)
    with pytest.raises(L.LbfgsError):
        L.shard_range(10**8, 0, 3)  # world must divide 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench

    D = bench.Dist(world)
    uid = D.broadcast_bytes(bytes(range(128)) if rank == 0 else None)
    D.barrier()
    tmax = D.allreduce(1.0 + rank, "max")
    tsum = D.allreduce(2.0 * (rank + 1), "sum")
    # the xGMI peer bootstrap's host channel: handle all-gather and the all-ranks-ok vote
    hs = D.allgather_bytes(bytes([rank]) * 64)
    vote_all = D.all_ok(True)
    vote_one_fails = D.all_ok(rank != 1)
    D.close()
    q.put((rank, uid == bytes(range(128)), tmax, tsum, hs == [bytes([0]) * 64, bytes([1]) * 64], vote_all,
           vote_one_fails))


def test_bench_distributed_bootstrap_gloo_world2():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert [r[1] for r in res] == [True, True]
    assert all(r[2] == 2.0 for r in res)  # max over ranks (bench's timing rule)
    assert all(r[3] == 6.0 for r in res)  # sum over ranks (bench's byte count)
    assert all(r[4] for r in res)  # peer handles gathered in rank order
    assert all(r[5] and not r[6] for r in res)  # one failing rank vetoes the peer exchange everywhere


STUB = '''
import json, os, sys
sys.path.insert(0, {root!r})
import bench

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
mode = sys.argv[1]
if mode == "fail" and rank == 1:
    sys.exit(3)  # before the barrier: rank 0 would wait there forever
D = bench.Dist(world)
D.barrier()
tmax = D.allreduce(float(rank), "max")
if rank == 0:
    print(json.dumps({{"world": world, "tmax": tmax, "local_rank": os.environ["LOCAL_RANK"],
                      "master": os.environ["MASTER_ADDR"], "argv": sys.argv[1:],
                      "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}}), flush=True)
D.close()
'''


def _launch(tmp_path, world, mode, timeout=120.0, extra_env=None):
    import subprocess

    stub = tmp_path / "stub_rank.py"
    stub.write_text(STUB.format(root=ROOT))
    drop = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "GPU_MAX_HW_QUEUES", "BENCH_DEVICE_MOD")
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(extra_env or {})
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"sys.exit(bench.self_launch([{mode!r}], {world}, {timeout}, script={str(stub)!r}))")
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=180)


@pytest.mark.parametrize("world", [2, 4])
def test_bench_self_launch_starts_ranks(tmp_path, world):
    """bench.py --gpus N > 1 with no launcher: self_launch starts N rank processes with the
    torch.distributed env (127.0.0.1, a free port), they rendezvous over gloo, and rank 0's one
    JSON line is the launcher's only stdout (the driver's N > 1 command shape, no wrapper)."""
    import json

    p = _launch(tmp_path, world, "ok")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d == {"world": world, "tmax": float(world - 1), "local_rank": "0", "master": "127.0.0.1", "argv": ["ok"],
                 "hw_queues": None}


def test_bench_self_launch_rehearsal_holds_ranks_to_one_unmasked_queue(tmp_path):
    """several ranks on one card (BENCH_DEVICE_MOD): each rank gets GPU_MAX_HW_QUEUES=1, so the
    card holds 2 compute queues per rank instead of 3 and stays under what its scheduler maps at
    once (DESIGN.md §5, configs[4] on one card) - also over the runtime's default of 4 already in
    the environment, as on the GPU boxes"""
    import json

    for extra in ({"BENCH_DEVICE_MOD": "1"}, {"BENCH_DEVICE_MOD": "1", "GPU_MAX_HW_QUEUES": "4"}):
        p = _launch(tmp_path, 2, "ok", extra_env=extra)
        assert p.returncode == 0, p.stderr[-2000:]
        assert json.loads(p.stdout.strip().splitlines()[-1])["hw_queues"] == "1"
    p = _launch(tmp_path, 2, "ok", extra_env={"GPU_MAX_HW_QUEUES": "4"})  # one rank per GPU: untouched
    assert json.loads(p.stdout.strip().splitlines()[-1])["hw_queues"] == "4"


def test_bench_self_launch_stops_on_a_failed_rank(tmp_path):
    """a rank that fails ends the launch at once with its status; the rank left waiting in a
    collective for it is stopped, not left hanging until the time limit"""
    import time

    t0 = time.time()
    p = _launch(tmp_path, 2, "fail", timeout=150.0)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert time.time() - t0 < 90 and "rank 1 exited with status 3" in p.stderr


def test_bench_self_launch_time_limit(tmp_path):
    """past the launch time limit every rank is stopped and the status is 124"""
    p = _launch(tmp_path, 2, "fail", timeout=3.0)  # rank 1 fails too, but the limit may come first
    assert p.returncode in (3, 124)
    stub = tmp_path / "sleeper.py"
    stub.write_text("import time; time.sleep(600)\n")
    import subprocess

    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"sys.exit(bench.self_launch([], 2, 2.0, script={str(stub)!r}))")
    q = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert q.returncode == 124 and "time limit" in q.stderr


def test_bench_main_self_launches_without_rank(monkeypatch):
    """main() takes the launcher branch before loading the library when --gpus > 1 and RANK is
    unset, and passes its own argv through"""
    sys.path.insert(0, ROOT)
    import bench

    calls = []
    monkeypatch.delenv("RANK", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3", "--launch-timeout", "77"])
    monkeypatch.setattr(bench, "self_launch", lambda argv, world, timeout: calls.append((argv, world, timeout)) or 0)
    monkeypatch.setattr(bench.L, "lib", lambda: pytest.fail("library loaded before the launch"))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and calls == [(["--gpus", "2", "--steps", "3", "--launch-timeout", "77"], 2, 77.0)]
