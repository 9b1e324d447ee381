"""ctypes binding of oracle/_build/liboracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the checker (a plain-C restatement of the reference, pinned against the
reference's own traces in tests/golden/). Product code must never import this module.
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# ORACLE_LIB: an instrumented build of the same source (tests/test_sanitize.py, ASan + UBSan)
ORACLE_SO = os.environ.get("ORACLE_LIB") or os.path.join(ORACLE_DIR, "_build", "liboracle.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

OBJ = {"rosenbrock": 0, "quad_tridiag": 1, "quad_sep": 2, "host": 3, "dense": 4}
LS = {"backtracking": 0, "interpolation": 1, "wolfe": 2, "backtracking_wolfe": 3}
SEQ, CANON = 0, 1
PAIR, REV, FMA = 3, 4, 5  # alternative summation orders (horizon yardsticks)
STATUS = {0: "converged", 1: "max_iter", 2: "ls_failed"}

# sequential-implementation/config.h:5-17
CONFIG_H = dict(c1=1e-4, c2=0.9, initial_step=1.0, backtracking_alpha=0.5,
                backtracking_tol=1e-8, wolfe_interp_min=1e-10)


class Opts(C.Structure):
    _fields_ = [("obj", C.c_int), ("ls", C.c_int), ("mode", C.c_int), ("verbose", C.c_int),
                ("n", C.c_int64), ("m", C.c_int), ("maxit", C.c_int), ("tol", C.c_double),
                ("c1", C.c_double), ("c2", C.c_double), ("initial_step", C.c_double),
                ("backtracking_alpha", C.c_double), ("backtracking_tol", C.c_double),
                ("wolfe_interp_min", C.c_double),
                ("host_f", C.c_void_p), ("host_g", C.c_void_p), ("host_user", C.c_void_p),
                ("vf", C.c_int), ("cuda", C.c_int)]


HOST_F = C.CFUNCTYPE(C.c_double, C.POINTER(C.c_double), C.c_int64, C.c_void_p)
HOST_G = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double), C.c_void_p)


def host_callbacks(f, grad):
    """ctypes callbacks for ORC_OBJ_HOST (keep the returned tuple alive during the run)."""
    def cf(xp, n, user):
        return float(f(np.ctypeslib.as_array(xp, shape=(n,)).copy()))

    def cg(xp, n, gp, user):
        np.ctypeslib.as_array(gp, shape=(n,))[:] = np.asarray(
            grad(np.ctypeslib.as_array(xp, shape=(n,)).copy()), dtype=np.float64)

    return HOST_F(cf), HOST_G(cg)


class Result(C.Structure):
    _fields_ = [("iters", C.c_int), ("status", C.c_int), ("ntrace", C.c_int),
                ("nf", C.c_int64), ("ng", C.c_int64), ("skips", C.c_int64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", ORACLE_DIR, "oracle"], check=True,
                           capture_output=True)
        L = C.CDLL(ORACLE_SO)
        dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
        up = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
        ip = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
        L.orc_x0_uniform.argtypes = [dp, C.c_int64, C.c_uint32, C.c_double, C.c_double]
        L.orc_dot.argtypes = [dp, dp, C.c_int64, C.c_int]
        L.orc_dot.restype = C.c_double
        L.orc_sum.argtypes = [dp, C.c_int64, C.c_int64, C.c_int]
        L.orc_sum.restype = C.c_double
        L.orc_canon_dot_groups.argtypes = [dp, dp, C.c_int64, dp]
        L.orc_canon_geometry.argtypes = [C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.orc_f.argtypes = [C.c_int, dp, C.c_int64, C.c_int]
        L.orc_f.restype = C.c_double
        L.orc_grad.argtypes = [C.c_int, dp, C.c_int64, dp]
        L.orc_checksum.argtypes = [dp, C.c_int64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.orc_lbfgs.argtypes = [C.POINTER(Opts), dp, dp, dp, dp, dp, up, up, ip, C.c_int,
                                dp, C.c_int64, C.POINTER(C.c_int64),
                                up, C.c_int64, C.POINTER(C.c_int64),
                                C.c_char_p, C.c_int, C.POINTER(Result)]
        L.orc_lbfgs.restype = C.c_int
        _lib = L
    return _lib


def x0_uniform(n, seed, lo, hi):
    x = np.empty(n, dtype=np.float64)
    lib().orc_x0_uniform(x, n, seed, lo, hi)
    return x


def dot(a, b, mode=CANON):
    return lib().orc_dot(np.ascontiguousarray(a, np.float64), np.ascontiguousarray(b, np.float64),
                         len(a), mode)


def canon_groups(a, b):
    q = np.zeros(8)
    lib().orc_canon_dot_groups(np.ascontiguousarray(a, np.float64),
                               np.ascontiguousarray(b, np.float64), len(a), q)
    return q


def geometry(n):
    L, ns = C.c_int64(), C.c_int64()
    lib().orc_canon_geometry(n, C.byref(L), C.byref(ns))
    return L.value, ns.value


def vf_factor(n):
    """canonical segments per vector-free commit segment (orc_vf_factor)"""
    lib().orc_vf_factor.argtypes = [C.c_int64]
    return lib().orc_vf_factor(n)


def f(obj, x, mode=CANON):
    return lib().orc_f(OBJ[obj], np.ascontiguousarray(x, np.float64), len(x), mode)


def grad(obj, x):
    g = np.empty(len(x))
    lib().orc_grad(OBJ[obj], np.ascontiguousarray(x, np.float64), len(x), g)
    return g


def checksum(x):
    a, b = C.c_uint64(), C.c_uint64()
    lib().orc_checksum(np.ascontiguousarray(x, np.float64), len(x), C.byref(a), C.byref(b))
    return a.value, b.value


def np_checksum(x):
    u = np.ascontiguousarray(x, np.float64).view(np.uint64)
    idx = np.arange(1, len(u) + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int(u.sum(dtype=np.uint64)), int((u * idx).sum(dtype=np.uint64))


def lbfgs(obj, x0, ls, m, maxit, tol, mode=CANON, consts=None, log_calls=False, verbose=False,
          f=None, grad=None, vector_free=False, cuda=False):
    """Run the oracle; returns a dict with x, trace arrays, call logs and messages.
    obj="host" takes the objective from the Python callables f(x) and grad(x)."""
    x0 = np.ascontiguousarray(x0, np.float64)
    n = len(x0)
    k = dict(CONFIG_H)
    if consts:
        k.update(consts)
    o = Opts(obj=OBJ[obj], ls=LS[ls], mode=mode, verbose=int(verbose), n=n, m=m, maxit=maxit,
             tol=tol, vf=int(vector_free), cuda=int(cuda), **k)
    cbs = None
    if obj == "host":
        cbs = host_callbacks(f, grad)
        o.host_f = C.cast(cbs[0], C.c_void_p)
        o.host_g = C.cast(cbs[1], C.c_void_p)
    cap = maxit + 2
    x = np.empty(n)
    trf, trg, tra = np.empty(cap), np.empty(cap), np.empty(cap)
    tc1, tc2 = np.empty(cap, np.uint64), np.empty(cap, np.uint64)
    tnf = np.empty(cap, np.int64)
    fcap = (60 * maxit + 100) if log_calls else 0
    flog = np.empty(max(fcap, 1))
    gcap = 3 * (30 * maxit + 10) if log_calls else 0
    glog = np.empty(max(gcap, 1), np.uint64)
    fn, gn = C.c_int64(0), C.c_int64(0)
    msg = C.create_string_buffer(1 << 20)
    res = Result()
    rc = lib().orc_lbfgs(C.byref(o), x0, x, trf, trg, tra, tc1, tc2, tnf, cap, flog, fcap,
                         C.byref(fn), glog, gcap, C.byref(gn), msg, len(msg), C.byref(res))
    assert rc == 0
    nt = res.ntrace
    return dict(x=x, f=trf[:nt].copy(), gnorm=trg[:nt].copy(), alpha=tra[:nt].copy(),
                c1=tc1[:nt].copy(), c2=tc2[:nt].copy(), nf=tnf[:nt].copy(),
                iters=res.iters, status=STATUS[res.status], nf_total=res.nf, ng_total=res.ng, skips=res.skips,
                flog=flog[:fn.value].copy(), glog=glog[:gn.value].reshape(-1, 3).copy(),
                messages=msg.value.decode())


# parallel-implementation/constants.h:5-17 (the CUDA path's constants: C2 = 0.7)
CONSTANTS_H = dict(CONFIG_H, c2=0.7)


def cuda_line_search(ls, x, d, g, mode=SEQ, obj="rosenbrock"):
    """One line search of parallel-implementation/line_search.cpp restated (orc_cuda_line_search),
    constants.h constants: (alpha, f-call values, grad-call log rows (c1, c2, |g| bits))."""
    L = lib()
    L.orc_cuda_line_search.argtypes = [C.POINTER(Opts), np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS"),
                                       np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS"),
                                       np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS"),
                                       C.POINTER(C.c_double),
                                       np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS"), C.c_int64,
                                       C.POINTER(C.c_int64),
                                       np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS"), C.c_int64,
                                       C.POINTER(C.c_int64)]
    x, d, g = (np.ascontiguousarray(v, np.float64) for v in (x, d, g))
    o = Opts(obj=OBJ[obj], ls=LS[ls], mode=mode, verbose=0, n=len(x), m=1, maxit=1, tol=0.0, vf=0, cuda=1,
             **CONSTANTS_H)
    flog, glog = np.empty(256), np.empty(3 * 64, np.uint64)
    a, fn, gn = C.c_double(), C.c_int64(), C.c_int64()
    assert L.orc_cuda_line_search(C.byref(o), x, d, g, C.byref(a), flog, len(flog), C.byref(fn), glog, len(glog),
                                  C.byref(gn)) == 0
    return a.value, flog[:fn.value].copy(), glog[:gn.value].reshape(-1, 3).copy()


_dense_refs = []


def dense_set(A, b):
    """Data of the "dense" objective (x'Ax + b'x); the arrays are kept alive here."""
    A = np.ascontiguousarray(A, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    _dense_refs[:] = [A, b]
    lib().orc_dense_set(A.ctypes.data_as(C.c_void_p), b.ctypes.data_as(C.c_void_p))


def load_golden(name):
    with open(os.path.join(GOLDEN, name + ".json")) as fp:
        meta = json.load(fp)
    arr = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return meta, {k: arr[k] for k in arr.files}


def golden_cases():
    return sorted(f[:-5] for f in os.listdir(GOLDEN)
                  if f.endswith(".json") and not f.startswith(("kat_", "stress_")) and f not in ("horizons.json", "cuda_ls.json"))


def stress_cases():
    """Guard-path goldens: the reference run on our stress objectives (oracle/ref_driver.cpp)."""
    return sorted(f[:-5] for f in os.listdir(GOLDEN) if f.startswith("stress_") and f.endswith(".json"))


def _seqsum(t):
    # left-to-right, from 0.0, as the reference's `for (...) sum += term`
    return float(np.cumsum(t)[-1]) if len(t) else 0.0


def stress_objective(name):
    """(f, grad) of a stress objective, operand for operand as oracle/ref_driver.cpp writes it."""
    if name == "stress_tiny_sq":
        return (lambda x: _seqsum(x * x)), (lambda x: 2.0 * x)
    if name == "stress_scaled_sq":
        return (lambda x: _seqsum(1e100 * x * x)), (lambda x: 2.0 * 1e100 * x)
    if name == "stress_quartic_well":
        return ((lambda x: _seqsum(-0.2 * x * x + 0.0016 * x * x * x * x)),
                (lambda x: 2.0 * -0.2 * x + 4.0 * 0.0016 * x * x * x))
    raise KeyError(name)


def twoloop(g, S, Y, mode=CANON):
    L = lib()
    L.orc_twoloop.argtypes = [np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS"),
                              C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int, C.c_int64,
                              C.c_int, np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")]
    L.orc_twoloop.restype = C.c_double
    S = [np.ascontiguousarray(s, np.float64) for s in S]
    Y = [np.ascontiguousarray(y, np.float64) for y in Y]
    sp = (C.c_void_p * len(S))(*[s.ctypes.data for s in S])
    yp = (C.c_void_p * len(Y))(*[y.ctypes.data for y in Y])
    d = np.empty(len(g))
    gd = L.orc_twoloop(np.ascontiguousarray(g, np.float64), sp, yp, len(S), len(g), mode, d)
    return d, gd
