"""Python binding of liblbfgs_hip.so (include/lbfgs_hip.h) — the MI355X L-BFGS solver.

The shared library is the product: HIP kernels for gfx950 plus the C host driver. This module
is a thin ctypes layer for tests and benchmarks; it never computes anything itself and raises
if the library is missing (there is no CPU fallback).

    import lbfgs_amd as L
    with L.Context(n=10**8, m=10) as ctx:
        res = ctx.minimize("rosenbrock", x0, "backtracking", max_iterations=100)
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LBFGS_LIB") or os.path.join(HERE, "liblbfgs_hip.so")  # LBFGS_LIB: A/B builds

OBJECTIVES = {"rosenbrock": 0, "quad_tridiag": 1, "quad_sep": 2, "host": 3, "dense": 4}
LINE_SEARCHES = {"backtracking": 0, "interpolation": 1, "wolfe": 2, "backtracking_wolfe": 3}
STATUS = {0: "converged", 1: "max_iter", 2: "ls_failed", 3: "running"}
FLAG_VERBOSE, FLAG_QUIET, FLAG_TRACE, FLAG_UNFUSED, FLAG_VECTOR_FREE = 1, 2, 4, 8, 16
FLAG_REFERENCE_CALLS = 32
FLAG_CUDA_COMPAT = 64
FLAG_CUDA_VARIANT = 128  # LBFGS_CUDA's semantics (parallel-implementation/L-BFGS.cu), include/lbfgs_hip.h
KERNELS = ["dot", "axpy_dot", "mid", "axpy2_dot", "last", "negdot", "eval", "trial_f",
           "trial_fg", "commit", "point", "checksum", "update", "vf_commit", "vf_dir", "small_iter",
           "group_reduce", "exchange"]


class LbfgsError(RuntimeError):
    pass


class Constants(C.Structure):
    _fields_ = [("c1", C.c_double), ("c2", C.c_double), ("initial_step", C.c_double),
                ("backtracking_alpha", C.c_double), ("backtracking_tol", C.c_double),
                ("wolfe_interp_min", C.c_double), ("wolfe_interp_max", C.c_double)]


class Result(C.Structure):
    _fields_ = [("iterations", C.c_int), ("status", C.c_int), ("f", C.c_double),
                ("gnorm", C.c_double), ("trials_f", C.c_int64), ("trials_fg", C.c_int64),
                ("commits", C.c_int64), ("passes", C.c_int64), ("bytes", C.c_double),
                ("seconds", C.c_double), ("h_min", C.c_int), ("h_max", C.c_int),
                ("f_calls", C.c_int64), ("grad_calls", C.c_int64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["status"] = STATUS.get(self.status, self.status)
        return d


HOST_F = C.CFUNCTYPE(C.c_double, C.POINTER(C.c_double), C.c_int64, C.c_void_p)
HOST_G = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double), C.c_void_p)


class HostFn(C.Structure):
    _fields_ = [("f", HOST_F), ("grad", HOST_G), ("user", C.c_void_p)]


_lib = None


def lib():
    """Load liblbfgs_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LbfgsError(f"{LIB_PATH} not built: run `make -C cuda-lbfgs_amd` "
                         "(or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
    vp = C.c_void_p
    L.lbfgs_ctx_create.argtypes = [C.POINTER(vp), C.c_int64, C.c_int, C.c_int]
    L.lbfgs_ctx_create_sharded.argtypes = [C.POINTER(vp), C.c_int64, C.c_int, C.c_int, C.c_int,
                                           C.c_int, C.c_char_p]
    L.lbfgs_unique_id.argtypes = [C.c_char_p]
    L.lbfgs_device_count.argtypes = []
    L.lbfgs_host_group_create.argtypes = [C.POINTER(vp), C.c_int]
    L.lbfgs_host_group_destroy.argtypes = [vp]
    L.lbfgs_host_group_destroy.restype = None
    L.lbfgs_ctx_create_emulated.argtypes = [C.POINTER(vp), C.c_int64, C.c_int, C.c_int, C.c_int, vp]
    L.lbfgs_ctx_destroy.argtypes = [vp]
    L.lbfgs_ctx_destroy.restype = None
    L.lbfgs_last_error.argtypes = [vp]
    L.lbfgs_last_error.restype = C.c_char_p
    L.lbfgs_local_range.argtypes = [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.lbfgs_shard_range.argtypes = [C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_int64),
                                    C.POINTER(C.c_int64)]
    L.lbfgs_constants_default.argtypes = [C.POINTER(Constants)]
    L.lbfgs_constants_default.restype = None
    L.lbfgs_constants_cuda.argtypes = [C.POINTER(Constants)]
    L.lbfgs_constants_cuda.restype = None
    L.lbfgs_minimize.argtypes = [vp, C.c_int, C.POINTER(HostFn), C.c_int, C.POINTER(Constants),
                                 dp, dp, C.c_int, C.c_double, C.c_uint, C.POINTER(Result)]
    L.lbfgs_solver_init.argtypes = [vp, C.c_int, C.POINTER(HostFn), C.c_int,
                                    C.POINTER(Constants), dp, C.c_double, C.c_uint]
    L.lbfgs_solver_step.argtypes = [vp, C.c_int, C.POINTER(Result)]
    L.lbfgs_get_x.argtypes = [vp, dp]
    L.lbfgs_sync.argtypes = [vp]
    L.lbfgs_messages.argtypes = [vp, C.c_char_p, C.c_int]
    L.lbfgs_trace_len.argtypes = [vp]
    L.lbfgs_trace_enable.argtypes = [vp, C.c_int]
    L.lbfgs_trace_get.argtypes = [vp, dp, dp, dp, np.ctypeslib.ndpointer(dtype=np.uint64),
                                  np.ctypeslib.ndpointer(dtype=np.uint64), C.c_int]
    L.lbfgs_dev_dot.argtypes = [vp, dp, dp, C.POINTER(C.c_double)]
    L.lbfgs_dev_norm.argtypes = [vp, dp, C.POINTER(C.c_double)]
    L.lbfgs_dev_objective.argtypes = [vp, C.c_int, dp, C.POINTER(C.c_double), vp]
    L.lbfgs_dev_trial.argtypes = [vp, C.c_int, dp, dp, C.c_double, C.POINTER(C.c_double), vp,
                                  C.POINTER(C.c_double)]
    L.lbfgs_dev_twoloop.argtypes = [vp, dp, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int,
                                    dp, C.POINTER(C.c_double)]
    L.lbfgs_peer_handle.argtypes = [vp, C.c_char_p]
    L.lbfgs_peer_connect.argtypes = [vp, C.c_char_p]
    L.lbfgs_peer_enable.argtypes = [vp, C.c_int]
    L.lbfgs_rccl_attach.argtypes = [vp, C.c_char_p]
    L.lbfgs_exchange_backend.argtypes = [vp]
    L.lbfgs_exchange_fold.argtypes = [vp]
    L.lbfgs_exchange_latency.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
    L.lbfgs_spec_stats.argtypes = [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.lbfgs_search_stats.argtypes = [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.lbfgs_cu_partition.argtypes = [vp]
    L.lbfgs_coop_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.lbfgs_wait_stats.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.POINTER(C.c_int)]
    L.lbfgs_vector_fallbacks.argtypes = [vp]
    L.lbfgs_vector_pool.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_double)]
    L.lbfgs_stream_probe.argtypes = [vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.lbfgs_stream_probe_variant.argtypes = [vp, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.lbfgs_stream_probe_vectors.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
    L.lbfgs_vector_address.argtypes = [vp, C.c_int, C.POINTER(C.c_uint64)]
    L.lbfgs_prof_enable.argtypes = [vp, C.c_int]
    L.lbfgs_prof_enable.restype = None
    L.lbfgs_prof_reset.argtypes = [vp]
    L.lbfgs_prof_reset.restype = None
    L.lbfgs_prof_get.argtypes = [vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                 C.POINTER(C.c_double)]
    _lib = L
    return L


EXPORTED_SYMBOLS = [
    "lbfgs_constants_default", "lbfgs_constants_cuda", "lbfgs_ctx_create",
    "lbfgs_ctx_create_sharded", "lbfgs_unique_id", "lbfgs_host_group_create",
    "lbfgs_host_group_destroy", "lbfgs_ctx_create_emulated", "lbfgs_ctx_destroy", "lbfgs_last_error",
    "lbfgs_local_range", "lbfgs_shard_range", "lbfgs_minimize", "lbfgs_solver_init", "lbfgs_solver_step",
    "lbfgs_get_x", "lbfgs_sync", "lbfgs_messages", "lbfgs_trace_len", "lbfgs_trace_get",
    "lbfgs_trace_enable",
    "lbfgs_dev_dot", "lbfgs_dev_norm", "lbfgs_dev_objective", "lbfgs_dev_trial",
    "lbfgs_dev_twoloop", "lbfgs_dev_elementwise", "lbfgs_line_search", "lbfgs_prof_enable",
    "lbfgs_prof_reset", "lbfgs_prof_get", "lbfgs_peer_handle", "lbfgs_peer_connect", "lbfgs_peer_enable", "lbfgs_rccl_attach",
    "lbfgs_exchange_backend", "lbfgs_exchange_fold", "lbfgs_exchange_latency", "lbfgs_device_count", "lbfgs_set_dense_quadratic", "lbfgs_build_info",
    "lbfgs_spec_stats", "lbfgs_cu_partition", "lbfgs_stream_probe", "lbfgs_stream_probe_variant", "lbfgs_stream_probe_vectors", "lbfgs_vector_address", "lbfgs_coop_info", "lbfgs_wait_stats", "lbfgs_vector_fallbacks", "lbfgs_vector_pool", "lbfgs_search_stats",
]
PEER_HANDLE_BYTES = 64
BACKENDS = {0: "single", 1: "rccl", 2: "xgmi", 3: "host-group"}


def constants(profile="config"):
    k = Constants()
    (lib().lbfgs_constants_cuda if profile == "cuda" else lib().lbfgs_constants_default)(C.byref(k))
    return k


def shard_range(n, rank, world):
    """(elem_lo, n_loc) of `rank` when n is sharded over `world` ranks (no device needed)."""
    lo, nl = C.c_int64(), C.c_int64()
    rc = lib().lbfgs_shard_range(int(n), int(rank), int(world), C.byref(lo), C.byref(nl))
    if rc != 0:
        raise LbfgsError(f"cannot shard n={n} over {world} ranks")
    return lo.value, nl.value


def build_info():
    """(the library's embedded build string, the source hash of this tree, match?): a library
    built from other sources than the ones beside it is stale."""
    lib().lbfgs_build_info.restype = C.c_char_p
    info = lib().lbfgs_build_info().decode()
    return info, source_hash(), info.startswith("src=" + source_hash() + " ")


def source_hash():
    """sha256 over the library's sources, in cuda-lbfgs_amd/Makefile's SRC_HASH order."""
    import glob
    import hashlib

    here = os.path.dirname(os.path.abspath(__file__))
    rel = []
    for pat in ("csrc/*.hip", "csrc/*.h", "csrc/*.c", "csrc/*.cpp", "../include/*.h"):
        rel += glob.glob(pat, root_dir=here)
    h = hashlib.sha256()
    for r in sorted(set(rel)):
        with open(os.path.join(here, r), "rb") as fp:
            h.update(fp.read())
    return h.hexdigest()[:16]


def device_count():
    return int(lib().lbfgs_device_count())


def unique_id():
    buf = C.create_string_buffer(128)
    rc = lib().lbfgs_unique_id(buf)
    if rc != 0:
        raise LbfgsError(f"lbfgs_unique_id failed ({rc})")
    return buf.raw


def x0_uniform(n, seed=42, lo=-2.0, hi=2.0):
    """x0 exactly as std::mt19937(seed) + std::uniform_real_distribution<double>(lo, hi)
    (libstdc++: generate_canonical<double,53> from two 32-bit draws), main.cpp:36-43."""
    rs = np.random.RandomState(seed)  # MT19937 with init_genrand(seed) == std::mt19937(seed)
    out = np.empty(n, dtype=np.float64)
    chunk = 1 << 22
    for s in range(0, n, chunk):
        k = min(chunk, n - s)
        raw = rs.randint(0, 1 << 32, size=2 * k, dtype=np.uint64).reshape(k, 2).astype(np.float64)
        u = (raw[:, 0] + raw[:, 1] * 4294967296.0) / 18446744073709551616.0
        u[u >= 1.0] = np.nextafter(1.0, 0.0)
        out[s:s + k] = u * (hi - lo) + lo
    return out


class HostGroup:
    """Exchange group for emulated ranks (threads of one process, e.g. on one GPU)."""

    def __init__(self, world):
        h = C.c_void_p()
        rc = lib().lbfgs_host_group_create(C.byref(h), int(world))
        if rc != 0:
            raise LbfgsError(f"lbfgs_host_group_create failed ({rc})")
        self.h, self.world = h, int(world)

    def close(self):
        if getattr(self, "h", None):
            lib().lbfgs_host_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """A persistent solver context: device vectors for n (or this rank's shard of n) and the
    m-pair history ring stay resident across calls."""

    def __init__(self, n, m=10, device=0, rank=0, world=1, uid=None, group=None):
        self.n, self.m = int(n), int(m)
        h = C.c_void_p()
        if group is not None:
            rc = lib().lbfgs_ctx_create_emulated(C.byref(h), self.n, self.m, device, rank, group.h)
        elif world == 1 and uid is None:
            rc = lib().lbfgs_ctx_create(C.byref(h), self.n, self.m, device)
        else:
            rc = lib().lbfgs_ctx_create_sharded(C.byref(h), self.n, self.m, device, rank, world, uid)
        if rc != 0:
            raise LbfgsError(f"lbfgs_ctx_create failed ({rc})")
        self.h = h
        lo, nl = C.c_int64(), C.c_int64()
        lib().lbfgs_local_range(self.h, C.byref(lo), C.byref(nl))
        self.elem_lo, self.n_loc = lo.value, nl.value
        self._cb = None

    def close(self):
        if getattr(self, "h", None):
            lib().lbfgs_ctx_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def spec_stats(self):
        """(adopted, dropped): speculative next-iteration launches the host took / discarded
        since solver init (small n, cooperative iteration; LBFGS_SPEC=0: none)."""
        a, d = C.c_int64(), C.c_int64()
        lib().lbfgs_spec_stats(self.h, C.byref(a), C.byref(d))
        return a.value, d.value

    def search_stats(self):
        """(launches, commits): line searches continued on the device since solver init, and the
        commits those launches took at the step they found (small n; LBFGS_DEV_SEARCH=0: none)."""
        a, d = C.c_int64(), C.c_int64()
        lib().lbfgs_search_stats(self.h, C.byref(a), C.byref(d))
        return a.value, d.value

    def set_dense_quadratic(self, A, b):
        """Upload A (n x n, symmetric) and b for the "dense" objective f = x'Ax + b'x."""
        A = np.ascontiguousarray(A, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        assert A.shape == (self.n, self.n) and b.shape == (self.n,)
        rc = lib().lbfgs_set_dense_quadratic(self.h, A.ctypes.data_as(C.c_void_p), b.ctypes.data_as(C.c_void_p))
        if rc != 0:
            self._err("lbfgs_set_dense_quadratic", rc)

    # ---- sharded runs: xGMI peer exchange ----
    def peer_handle(self):
        buf = C.create_string_buffer(PEER_HANDLE_BYTES)
        rc = lib().lbfgs_peer_handle(self.h, buf)
        if rc != 0:
            self._err("lbfgs_peer_handle", rc)
        return buf.raw

    def connect_peers(self, allgather, agree):
        """Switch this sharded context's exchanges to the xGMI peer mailboxes.
        allgather(bytes) -> list of every rank's bytes (rank order); agree(ok: bool) -> True iff
        every rank passed (e.g. torch.distributed gloo all_gather_object / all_reduce MIN).
        Returns (enabled, this rank's connect error or None); when a rank fails, no rank enables
        and the context keeps its RCCL communicator (if it has one)."""
        msg = None
        try:
            mine = self.peer_handle()
        except LbfgsError as e:  # no mailbox on this rank: every rank still joins the collectives
            mine, msg = b"", str(e)
        handles = allgather(mine)
        if all(len(h) == PEER_HANDLE_BYTES for h in handles):
            rc = lib().lbfgs_peer_connect(self.h, b"".join(handles))
            if rc != 0:
                m = lib().lbfgs_last_error(self.h)
                msg = f"lbfgs_peer_connect failed ({rc}): {m.decode() if m else ''}"
        else:
            rc = -1
            msg = msg or "a peer has no mailbox"
        ok = agree(rc == 0)
        if ok:
            rc2 = lib().lbfgs_peer_enable(self.h, 1)
            if rc2 != 0:
                self._err("lbfgs_peer_enable", rc2)
        return ok, msg

    def peer_enable(self, on=True):
        """Route this context's exchanges through the peer mailboxes (after connect_peers) or
        back to its RCCL communicator. Every rank must make the same choice."""
        rc = lib().lbfgs_peer_enable(self.h, 1 if on else 0)
        if rc != 0:
            self._err("lbfgs_peer_enable", rc)

    def rccl_attach(self, uid):
        """Give this sharded context (created without an RCCL id) a communicator: collective over
        every rank, bounded by LBFGS_RCCL_TIMEOUT (60 s); raises LbfgsError on a failed or stalled
        init, leaving the context on its mailboxes."""
        rc = lib().lbfgs_rccl_attach(self.h, uid)
        if rc != 0:
            self._err("lbfgs_rccl_attach", rc)

    def exchange_latency(self, backend, components=8, iters=200):
        """Collective: microseconds per exchange through 'rccl' or 'xgmi' (every rank calls)."""
        us = C.c_double()
        rc = lib().lbfgs_exchange_latency(self.h, {"rccl": 1, "xgmi": 2}[backend], int(components), int(iters),
                                          C.byref(us))
        if rc != 0:
            self._err("lbfgs_exchange_latency", rc)
        return us.value

    @property
    def backend(self):
        return BACKENDS.get(lib().lbfgs_exchange_backend(self.h), "unknown")

    def coop_info(self):
        """dict(coop_max, search_max, fallbacks): the cooperative forms' grid caps (segments) and
        the device line searches redone on the host loop after a grid-barrier time-out"""
        a, b, f = C.c_int(), C.c_int(), C.c_int()
        lib().lbfgs_coop_info(self.h, C.byref(a), C.byref(b), C.byref(f))
        return dict(coop_max=a.value, search_max=b.value, fallbacks=f.value)

    def stream_probe_vectors(self, q, y, s, launches=20):
        """the probe's stream over three of the context's vectors by allocation index
        (lbfgs_stream_probe_vectors): mean microseconds per launch"""
        us = C.c_double()
        rc = lib().lbfgs_stream_probe_vectors(self.h, int(q), int(y), int(s), int(launches), C.byref(us))
        if rc != 0:
            self._err("lbfgs_stream_probe_vectors", rc)
        return us.value

    def vector_address(self, k):
        a = C.c_uint64()
        if lib().lbfgs_vector_address(self.h, int(k), C.byref(a)) != 0:
            return None
        return a.value

    @property
    def vector_pool(self):
        """(mode, vectors of this context taken from / added to the contiguous pool, GiB the process's
        pool owns); mode 'pool' (default), 'plain' or 'contiguous' (lbfgs_vector_pool)"""
        n, gb = C.c_int(), C.c_double()
        mode = int(lib().lbfgs_vector_pool(self.h, C.byref(n), C.byref(gb)))
        return {0: "pool", 1: "plain", 2: "contiguous"}.get(mode, mode), n.value, gb.value

    @property
    def vector_fallbacks(self):
        """vectors that asked for a physically contiguous allocation (LBFGS_VEC_ALLOC=contiguous) and got a plain one"""
        return int(lib().lbfgs_vector_fallbacks(self.h))

    def wait_stats(self):
        """host waits on completion words: dict(slept_s, waits, adaptive) (lbfgs_wait_stats)"""
        s, w, a = C.c_double(), C.c_uint64(), C.c_int()
        lib().lbfgs_wait_stats(self.h, C.byref(s), C.byref(w), C.byref(a))
        return dict(slept_s=s.value, waits=w.value, adaptive=bool(a.value))

    @property
    def cu_partition(self):
        """CUs this rank's solver stream is confined to (LBFGS_CU_PARTITION=1), 0 if not"""
        return int(lib().lbfgs_cu_partition(self.h))

    def stream_probe(self, launches=20, variant=0):
        """This box's rate for the two-loop passes' 3 R + 1 W access pattern over the context's own
        buffers (lbfgs_stream_probe; after init): dict(avg_launch_us, bytes_per_launch, gbps).
        variant > 0: the pass's machinery added piece by piece (lbfgs_stream_probe_variant)."""
        us, b = C.c_double(), C.c_double()
        rc = lib().lbfgs_stream_probe_variant(self.h, int(variant), int(launches), C.byref(us), C.byref(b))
        if rc != 0:
            self._err("lbfgs_stream_probe", rc)
        return dict(avg_launch_us=us.value, bytes_per_launch=b.value,
                    gbps=b.value / (us.value * 1e-6) / 1e9 if us.value > 0 else None)

    @property
    def folded(self):
        """the two-loop's mailbox exchanges ride inside the passes (lbfgs_exchange_fold)"""
        return lib().lbfgs_exchange_fold(self.h) == 1

    def _err(self, what, rc):
        msg = lib().lbfgs_last_error(self.h)
        raise LbfgsError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def _host_fn(self, f, grad):
        def cf(xp, n, user):
            return float(f(np.ctypeslib.as_array(xp, shape=(n,)).copy()))

        def cg(xp, n, gp, user):
            g = np.asarray(grad(np.ctypeslib.as_array(xp, shape=(n,)).copy()), dtype=np.float64)
            np.ctypeslib.as_array(gp, shape=(n,))[:] = g

        self._cb = (HOST_F(cf), HOST_G(cg))
        return HostFn(self._cb[0], self._cb[1], None)

    def minimize(self, objective, x0, line_search="backtracking", max_iterations=1000, m=None,
                 tolerance=1e-5, verbose=False, quiet=True, trace=False, consts=None,
                 f=None, grad=None, unfused=False, vector_free=False, reference_calls=False, out=None,
                 cuda_compat=False, cuda_variant=False):
        """out: a caller-owned float64 buffer of n for the result (else a new array; a fresh
        array's pages are first touched by the result's copy, which costs as much as the copy)"""
        assert m is None or m == self.m
        x0 = np.ascontiguousarray(x0, dtype=np.float64)
        assert x0.shape == (self.n,)
        if out is not None:
            assert out.dtype == np.float64 and out.shape == (self.n,) and out.flags["C_CONTIGUOUS"]
        x = out if out is not None else np.zeros(self.n)
        res = Result()
        flags = (FLAG_VERBOSE if verbose else 0) | (FLAG_QUIET if quiet else 0) | \
                (FLAG_TRACE if trace else 0) | (FLAG_UNFUSED if unfused else 0) | \
                (FLAG_VECTOR_FREE if vector_free else 0) | (FLAG_REFERENCE_CALLS if reference_calls else 0) | \
                (FLAG_CUDA_COMPAT if cuda_compat else 0) | (FLAG_CUDA_VARIANT if cuda_variant else 0)
        cb = self._host_fn(f, grad) if objective == "host" else None
        # the CUDA path reads parallel-implementation/constants.h (C2 = 0.7), not config.h
        k = consts if consts is not None else constants("cuda" if cuda_compat else "config")
        rc = lib().lbfgs_minimize(self.h, OBJECTIVES[objective], C.byref(cb) if cb else None,
                                  LINE_SEARCHES[line_search], C.byref(k), x0, x,
                                  int(max_iterations), float(tolerance), flags, C.byref(res))
        if rc < 0:
            self._err("lbfgs_minimize", rc)
        out = res.as_dict()
        out["x"] = x
        out["messages"] = self.messages()
        if trace:
            out.update(self.trace())
        return out

    def init(self, objective, x0, line_search="backtracking", tolerance=1e-5, quiet=True,
             trace=False, consts=None, unfused=False, vector_free=False):
        x0 = np.ascontiguousarray(x0, dtype=np.float64)
        flags = (FLAG_QUIET if quiet else 0) | (FLAG_TRACE if trace else 0) | \
            (FLAG_UNFUSED if unfused else 0) | (FLAG_VECTOR_FREE if vector_free else 0)
        k = consts if consts is not None else constants()
        rc = lib().lbfgs_solver_init(self.h, OBJECTIVES[objective], None,
                                     LINE_SEARCHES[line_search], C.byref(k), x0, float(tolerance),
                                     flags)
        if rc != 0:
            self._err("lbfgs_solver_init", rc)

    def step(self, steps):
        res = Result()
        rc = lib().lbfgs_solver_step(self.h, int(steps), C.byref(res))
        if rc < 0:
            self._err("lbfgs_solver_step", rc)
        return res.as_dict()

    def sync(self):
        rc = lib().lbfgs_sync(self.h)
        if rc != 0:
            self._err("lbfgs_sync", rc)

    def get_x(self):
        x = np.zeros(self.n)
        rc = lib().lbfgs_get_x(self.h, x)
        if rc != 0:
            self._err("lbfgs_get_x", rc)
        return x

    def messages(self):
        buf = C.create_string_buffer(1 << 20)
        lib().lbfgs_messages(self.h, buf, len(buf))
        return buf.value.decode()

    def trace_enable(self, on=True):
        """Record (or stop recording) the per-iteration trace between step() calls."""
        rc = lib().lbfgs_trace_enable(self.h, 1 if on else 0)
        if rc != 0:
            self._err("lbfgs_trace_enable", rc)

    def trace(self):
        n = lib().lbfgs_trace_len(self.h)
        f, g, a = np.empty(max(n, 1)), np.empty(max(n, 1)), np.empty(max(n, 1))
        c1, c2 = np.empty(max(n, 1), np.uint64), np.empty(max(n, 1), np.uint64)
        lib().lbfgs_trace_get(self.h, f, g, a, c1, c2, n)
        return dict(tr_f=f[:n], tr_gnorm=g[:n], tr_alpha=a[:n], tr_c1=c1[:n], tr_c2=c2[:n])

    # ---- primitives ----
    def dot(self, a, b):
        out = C.c_double()
        rc = lib().lbfgs_dev_dot(self.h, np.ascontiguousarray(a, np.float64),
                                 np.ascontiguousarray(b, np.float64), C.byref(out))
        if rc != 0:
            self._err("lbfgs_dev_dot", rc)
        return out.value

    def objective(self, objective, x, with_grad=True):
        f = C.c_double()
        g = np.zeros(self.n) if with_grad else None
        rc = lib().lbfgs_dev_objective(self.h, OBJECTIVES[objective],
                                       np.ascontiguousarray(x, np.float64), C.byref(f),
                                       g.ctypes.data_as(C.c_void_p) if with_grad else None)
        if rc != 0:
            self._err("lbfgs_dev_objective", rc)
        return f.value, g

    def trial(self, objective, x, d, alpha, with_grad=True):
        f, dphi = C.c_double(), C.c_double()
        g = np.zeros(self.n) if with_grad else None
        rc = lib().lbfgs_dev_trial(self.h, OBJECTIVES[objective],
                                   np.ascontiguousarray(x, np.float64),
                                   np.ascontiguousarray(d, np.float64), float(alpha), C.byref(f),
                                   g.ctypes.data_as(C.c_void_p) if with_grad else None,
                                   C.byref(dphi))
        if rc != 0:
            self._err("lbfgs_dev_trial", rc)
        return f.value, g, dphi.value

    def line_search(self, objective, line_search, x, d, g, consts=None):
        """lbfgs_line_search: the reference's free line-search functions (line_search.cpp) at x along
        d with gradient g, device objective; returns the step"""
        a = C.c_double()
        k = consts if consts is not None else constants()
        dp = lambda v: np.ascontiguousarray(v, np.float64).ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        xs, ds, gs = (np.ascontiguousarray(v, np.float64) for v in (x, d, g))
        rc = lib().lbfgs_line_search(self.h, OBJECTIVES[objective], None, LINE_SEARCHES[line_search], C.byref(k),
                                     dp(xs), dp(ds), dp(gs), C.byref(a))
        if rc != 0:
            self._err("lbfgs_line_search", rc)
        return a.value

    def twoloop(self, g, S, Y):
        h = len(S)
        S = [np.ascontiguousarray(s, np.float64) for s in S]
        Y = [np.ascontiguousarray(y, np.float64) for y in Y]
        sp = (C.c_void_p * h)(*[s.ctypes.data for s in S])
        yp = (C.c_void_p * h)(*[y.ctypes.data for y in Y])
        d = np.zeros(self.n)
        gd = C.c_double()
        rc = lib().lbfgs_dev_twoloop(self.h, np.ascontiguousarray(g, np.float64), sp, yp, h, d,
                                     C.byref(gd))
        if rc != 0:
            self._err("lbfgs_dev_twoloop", rc)
        return d, gd.value

    # ---- profiling ----
    def prof_enable(self, on=True):
        lib().lbfgs_prof_enable(self.h, int(on))

    def prof_reset(self):
        lib().lbfgs_prof_reset(self.h)

    def prof_get(self, kind):
        ms, n, b = C.c_double(), C.c_int64(), C.c_double()
        rc = lib().lbfgs_prof_get(self.h, KERNELS.index(kind), C.byref(ms), C.byref(n), C.byref(b))
        if rc != 0:
            self._err("lbfgs_prof_get", rc)
        return dict(ms=ms.value, launches=n.value, bytes=b.value)
