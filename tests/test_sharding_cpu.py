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
