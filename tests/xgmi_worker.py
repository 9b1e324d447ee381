"""One rank of a multi-process sharded solve whose exchanges go through the xGMI peer mailboxes
(cuda-lbfgs_amd/csrc/lbfgs_xgmi.hip) — no RCCL communicator at all. Started by
tests/test_gpu_xgmi.py, one process per rank, every rank on the same GPU (the box has one):
the mailboxes are then IPC-mapped between processes on one device, which runs the same kernel,
wire format and bootstrap as the cross-GPU case.

Bootstrap through files in a shared directory (each rank writes its handle, waits for all;
then the same for the connect verdict), so no torch import is needed.

    python xgmi_worker.py DIR RANK WORLD N M OBJ LS ITERS MODE

LBFGS_CU_PARTITION=1 in the environment confines each rank's solver stream to its own CUs (the
forward-progress situation of distinct GPUs; the folded exchanges then run ungated).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-lbfgs_amd"))
import lbfgs_amd as L  # noqa: E402


def wait_all(paths, timeout=120.0):
    t0 = time.time()
    while not all(os.path.exists(p) for p in paths):
        if time.time() - t0 > timeout:
            raise TimeoutError(f"peers missing: {[p for p in paths if not os.path.exists(p)]}")
        time.sleep(0.01)


def publish(path, data):
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)


def main():
    d, rank, world, n, m, obj, ls, iters, mode = sys.argv[1:10]
    rank, world, n, m, iters = int(rank), int(world), int(n), int(m), int(iters)
    x0 = L.x0_uniform(n, 42, -2.0, 2.0)
    ctx = L.Context(n, m, device=0, rank=rank, world=world, uid=None)

    def allgather(b):
        publish(os.path.join(d, f"h{rank}"), b)
        paths = [os.path.join(d, f"h{r}") for r in range(world)]
        wait_all(paths)
        return [open(p, "rb").read() for p in paths]

    def agree(ok):
        publish(os.path.join(d, f"ok{rank}"), b"1" if ok else b"0")
        paths = [os.path.join(d, f"ok{r}") for r in range(world)]
        wait_all(paths)
        return all(open(p, "rb").read() == b"1" for p in paths)

    if mode == "silent":  # a peer that publishes its handle and never exchanges (timeout test)
        allgather(ctx.peer_handle())
        agree(False)
        ctx.close()
        return
    ok, msg = ctx.connect_peers(allgather, agree)
    if not ok:
        print(f"rank {rank}: peer connect failed: {msg}", flush=True)
        sys.exit(3)
    assert ctx.backend == "xgmi", ctx.backend
    folded = ctx.folded
    if mode == "stall":  # connected, then never exchanges while a peer solves (timeout test)
        time.sleep(float(os.environ.get("XGMI_STALL_S", "20")))
        ctx.close()
        return
    if mode == "expect_fail":  # the peer stalls: the solve must fail, once, within its timeout
        t0 = time.time()
        try:
            ctx.minimize(obj, x0, ls, iters, trace=True)
        except L.LbfgsError as e:
            print(f"rank {rank}: failed after {time.time() - t0:.1f} s: {e}", flush=True)
            ctx.close()
            sys.exit(4)
        print(f"rank {rank}: no failure", flush=True)
        sys.exit(0)
    if mode == "latency":  # lbfgs_exchange_latency through the mailboxes (collective)
        us8 = ctx.exchange_latency("xgmi", 8, 50)
        us96 = ctx.exchange_latency("xgmi", 96, 50)
        np.savez(os.path.join(d, f"out{rank}.npz"), us8=us8, us96=us96)
        ctx.close()
        print(f"rank {rank}: {us8:.2f} / {us96:.2f} us per exchange", flush=True)
        return
    if mode == "steps":  # configs[4] sizes: init + step as bench.py's config4() (no full-size x back)
        t0 = time.time()
        ctx.init(obj, x0, ls, tolerance=1e-5, trace=True)
        del x0
        r = ctx.step(iters)
        ctx.sync()
        tr = ctx.trace()
        np.savez(os.path.join(d, f"out{rank}.npz"), status=r["status"], iterations=r["iterations"], f=r["f"],
                 gnorm=r["gnorm"], h_max=r["h_max"], folded=folded, cu_part=ctx.cu_partition,
                 seconds=time.time() - t0, **tr)
        ctx.close()
        print(f"rank {rank}: {r['status']} after {r['iterations']} iterations, f={r['f']!r}", flush=True)
        return
    r = ctx.minimize(obj, x0, ls, iters, trace=True, vector_free=(mode == "vf"))
    lo, nl = ctx.elem_lo, ctx.n_loc
    np.savez(os.path.join(d, f"out{rank}.npz"), tr_f=r["tr_f"], tr_gnorm=r["tr_gnorm"], tr_alpha=r["tr_alpha"],
             tr_c1=r["tr_c1"], tr_c2=r["tr_c2"], x=r["x"][lo:lo + nl], lo=lo, status=r["status"],
             messages=r["messages"], folded=folded, cu_part=ctx.cu_partition)
    ctx.close()
    print(f"rank {rank}: {r['status']} after {r['iterations']} iterations, f={r['f']!r}", flush=True)


if __name__ == "__main__":
    main()
