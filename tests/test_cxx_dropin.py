"""The C++ drop-in layer (include/lbfgs.h, benchmark.h, line_search.h, vector_utils.h,
config.h): a reference-style caller compiles against our headers (CPU) and, on the GPU, gives
the canonical-order results of the oracle."""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cuda-lbfgs_amd")
SRC = os.path.join(ROOT, "tests", "cxx", "dropin_main.cpp")
CXX_DIR = os.path.join(ROOT, "tests", "cxx")
REF_MAIN_SRC = "/root/reference/sequential-implementation/main.cpp"
REF_MAIN_EXE = os.path.join(CXX_DIR, "_build", "ref_main")


def _build(tmp):
    lib = os.path.join(PKG, "liblbfgs_hip.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)
    exe = os.path.join(tmp, "dropin_main")
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), SRC, "-o", exe, lib,
                    "-Wl,-rpath," + PKG], check=True, capture_output=True, text=True)
    return exe


def test_reference_style_caller_compiles(tmp_path):
    assert os.path.exists(_build(str(tmp_path)))


def _parse(out):
    d = {}
    for line in out.splitlines():
        if line.startswith("KEY "):
            parts = line.split(" ", 2)
            d[parts[1]] = parts[2]
    return d


def _fx(s):
    return float.fromhex(s)


def _ck(s):
    a, b = s.split()
    return int(a), int(b)


@pytest.mark.gpu
def test_cxx_dropin_on_gpu(tmp_path):
    exe = _build(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    k = _parse(r.stdout)
    n = 2000
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    o = O.lbfgs("rosenbrock", x0, "backtracking", 5, 30, 1e-5, mode=O.CANON)
    assert _ck(k["x_device"]) == O.checksum(o["x"])
    assert _fx(k["xh_minus_x_max"]) <= 1e-8  # host callbacks (sequential f) vs device f
    oq = O.lbfgs("quad_tridiag", x0, "wolfe", 20, 1000, 1e-5, mode=O.CANON)
    assert _ck(k["x_qtri"]) == O.checksum(oq["x"])
    assert _fx(k["dot"]) == O.dot(x0, x0, O.CANON)
    assert _fx(k["norm"]) == np.sqrt(O.dot(x0, x0, O.CANON))
    assert _ck(k["add"]) == O.checksum(x0 + x0)
    assert _ck(k["scal"]) == O.checksum(0.37 * x0)
    assert _ck(k["neg"]) == O.checksum(-x0)
    assert k["size_error"] == "Vectors must be of same size"
    # standalone line searches == the first step the oracle takes from x0 (d = -g)
    for ls in ["backtracking", "interpolation", "wolfe", "backtracking_wolfe"]:
        ol = O.lbfgs("rosenbrock", x0, ls, 5, 1, 1e-5, mode=O.CANON)
        assert _fx(k["ls_" + ls]) == ol["alpha"][0], ls
    assert k["bad_method"] == "Unknown line search method: bogus"
    oc = O.lbfgs("rosenbrock", x0, "wolfe", 5, 20, 1e-5, mode=O.CANON, consts=dict(c2=0.7))
    assert _ck(k["x_cuda"]) == O.checksum(oc["x"])
    ob = O.lbfgs("rosenbrock", x0, "backtracking", 5, 20, 1e-5, mode=O.CANON, consts=dict(c2=0.7))
    assert _ck(k["x_cuda_bt"]) == O.checksum(ob["x"])
    assert _fx(k["C2"]) == 0.9
    assert "Maximum iterations reached" in r.stdout and "Converged!" in r.stdout
    # dense quadratic functors -> the device dense objective (LBFGS_OBJ_DENSE_QUAD), converged
    assert k["dense_objective"] == "4"
    assert _fx(k["dense_gnorm"]) < 1e-6


@pytest.mark.gpu
def test_cxx_dropin_vector_free_mode(tmp_path):
    """LBFGS_MODE=vector_free: the unchanged reference-style caller runs the vector-free mode for
    its device objectives (bit-exact with the oracle's restatement) and the default mode for its
    host-callback objective."""
    exe = _build(str(tmp_path))
    env = dict(os.environ, LBFGS_MODE="vector_free")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    k = _parse(r.stdout)
    x0 = O.x0_uniform(2000, 42, -2.0, 2.0)
    o = O.lbfgs("rosenbrock", x0, "backtracking", 5, 30, 1e-5, mode=O.CANON, vector_free=True)
    assert _ck(k["x_device"]) == O.checksum(o["x"])
    oq = O.lbfgs("quad_tridiag", x0, "wolfe", 20, 1000, 1e-5, mode=O.CANON, vector_free=True)
    assert _ck(k["x_qtri"]) == O.checksum(oq["x"])


def test_reference_main_compiles_unchanged():
    """The reference's own entry point (sequential-implementation/main.cpp, which calls
    benchmark() of benchmark.h:19-26 on its own quadratic) compiles UNCHANGED against include/
    and links liblbfgs_hip.so (tests/cxx/Makefile `ref`; only the reference's matrices.h data
    header is taken from its directory). Built here, run on the GPU box below."""
    if not os.path.exists(REF_MAIN_SRC):
        if os.path.exists(REF_MAIN_EXE):
            return  # GPU box: the binary built in the source container travels with the tree
        pytest.skip("/root/reference absent and tests/cxx/_build/ref_main not built")
    r = subprocess.run(["make", "-C", CXX_DIR, "ref"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.exists(REF_MAIN_EXE)


@pytest.mark.parametrize("link", [[], ["-fno-pic", "-no-pie"]], ids=["pie", "no-pie"])
def test_caller_defined_objective_is_not_replaced(tmp_path, link):
    """identify() only maps THIS library's rosenbrock / quadratic / generate_quadratic_* to device
    kernels (protected symbols). A caller's own function of the same name (main.cpp:7-21 defines
    quadratic) stays the caller's and runs as a host callback. Without a GPU the solve throws after
    the objective has been classified; with one it runs (n = 50). A non-PIE caller takes the
    library's rosenbrock through a canonical PLT entry of its own (a different address from the
    library's protected one), which identify() recognises by the undefined symbol behind it."""
    src = tmp_path / "own.cpp"
    src.write_text(r'''
#include <cstdio>
#include <stdexcept>
#include <benchmark.h>
double quadratic(const vector<double>& X) { double s = 0; for (double x : X) s += (x - 2) * (x - 2); return s; }
vector<double> quadratic_grad(const vector<double>& X) {
    vector<double> g(X.size()); for (size_t i = 0; i < X.size(); ++i) g[i] = 2.0 * (X[i] - 2); return g; }
int main() {
    vector<double> x0(50, 0.5);
    int ids[2];
    try { LBFGS(rosenbrock, rosenbrock_grad, x0, "backtracking", 3, 3, 1e-5, false); } catch (const std::runtime_error&) {}
    ids[0] = lbfgs_amd::last_objective();
    try { LBFGS(quadratic, quadratic_grad, x0, "backtracking", 3, 3, 1e-5, false); } catch (const std::runtime_error&) {}
    ids[1] = lbfgs_amd::last_objective();
    std::printf("IDS %d %d\n", ids[0], ids[1]);
    return 0;
}
''')
    exe = tmp_path / "own"
    subprocess.run(["g++", "-std=c++17", "-O2", *link, "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe), "-L", PKG, "-l:liblbfgs_hip.so", "-Wl,-rpath," + PKG], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("IDS ")][0]
    assert line.split()[1:] == ["0", "3"]  # device Rosenbrock; the caller's quadratic on the host


def _quad_seq(x):  # main.cpp:7-13, left to right
    s = 0.0
    for v in x.tolist():
        s += (v - 1) * (v - 1)
    return s


@pytest.mark.gpu
def test_reference_main_on_gpu():
    """The reference's unchanged main.cpp (BASELINE configs' main: separable quadratic, n = 1e4,
    x0 ~ U(-1000, 1000) from mt19937(42), m = 10, tol 1e-8, through benchmark()) on the GPU.
    Its "Optimum value" line equals the canonical-order oracle's f at its final x (the same
    host-callback run), and like the reference's own (3.44e-23, tests/golden/qsep_main) it is
    zero to within 1e-20 of f(x0) ~ 3.3e9; it converges as the reference does."""
    if not os.path.exists(REF_MAIN_EXE):
        pytest.skip("tests/cxx/_build/ref_main not built (needs /root/reference where it is built)")
    r = subprocess.run([REF_MAIN_EXE], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    meta, g = O.load_golden("qsep_main")
    assert "Converged!" in lines and meta["stdout"] == "Converged!\n"
    assert "Function: Quadratic Function" in lines
    opt = [ln for ln in lines if ln.startswith("Optimum value: ")]
    assert len(opt) == 1
    v = float(opt[0].split(": ", 1)[1])
    x0 = O.x0_uniform(10000, 42, -1000.0, 1000.0)
    o = O.lbfgs("host", x0, "backtracking", 10, 15000, 1e-8, mode=O.CANON, f=_quad_seq,
                grad=lambda x: 2.0 * (x - 1))
    assert opt[0] == "Optimum value: " + ("%g" % _quad_seq(o["x"]))
    assert abs(v) <= 1e-20 and abs(_quad_seq(g["ret_x"])) <= 1e-20
    assert sum(ln.startswith("Elapsed time: ") for ln in lines) == 2  # benchmark() + main.cpp:55
    assert lines.count("---------------------------------------------") == 1


# ---- the CUDA path's callers (parallel-implementation/*.cu main()) ----------------------------
CUDA_DIR = "/root/reference/parallel-implementation"
# .cu file -> (executable suffix, line search the variant implies, n, method passed as a string)
CUDA_MAINS = {
    "L-BFGS.cu": ("LBFGS", "wolfe", 5),                              # L-BFGS.cu:384-409
    "L-BFGS-Backtracking.cu": ("Backtracking", "backtracking", 50000),  # :429-457
    "L-BFGS-Interpolation.cu": ("Interpolation", "interpolation", 50000),  # :444-472
    "L-BFGS-Wolfe.cu": ("Wolfe", "wolfe", 50000),                     # :456-484
    "L-BFGS-Backtracking_Wolfe.cu": ("Backtracking_Wolfe", "backtracking_wolfe", 50000),  # :504-532
}


def _cuda_exe(tag):
    return os.path.join(CXX_DIR, "_build", "cuda_main_" + tag)


def test_cuda_path_mains_compile_unchanged():
    """Each parallel-implementation .cu file's own main() builds unchanged against include/
    (functions.h, constants.h, line_search.h, vector_utils.h, lbfgs.h) and links
    liblbfgs_hip.so (tests/cxx/Makefile `cuda`: the prelude replaces the file's CUDA/cuBLAS
    includes and its LBFGS_CUDA definition; the main() text is piped from the reference)."""
    exes = [_cuda_exe(v[0]) for v in CUDA_MAINS.values()]
    if not os.path.isdir(CUDA_DIR):
        if all(os.path.exists(e) for e in exes):
            return
        pytest.skip("/root/reference absent and tests/cxx/_build/cuda_main_* not built")
    r = subprocess.run(["make", "-C", CXX_DIR, "cuda"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert all(os.path.exists(e) for e in exes)
    # no copy of the reference's text is left in the tree (the recipe pipes it to the compiler)
    assert not [f for f in os.listdir(os.path.join(CXX_DIR, "_build")) if f.endswith(".cpp")]


_VARIANT_CALLER = r'''
#include <cstdio>
#include <stdexcept>
#include <functions.h>
#include <benchmark.h>  // both objective headers in one unit (same declarations)
int main() {
    vector<double> x0(8, 0.5);
    try { LBFGS_CUDA(rosenbrock, rosenbrock_grad, x0, 10, 5, 1e-1); }
    catch (const std::invalid_argument& e) { std::printf("INVALID %s\n", e.what()); }
    catch (const std::runtime_error& e) { std::printf("RUNTIME\n"); }
    return 0;
}
'''


@pytest.mark.parametrize("how", ["macro", "env"])
def test_cuda_variant_selection_unknown_name(tmp_path, how):
    """The string-less LBFGS_CUDA names its line search through -DLBFGS_CUDA_VARIANT (compile time)
    or LBFGS_CUDA_VARIANT (environment); an unknown name throws std::invalid_argument with the
    reference's message (lbfgs.cpp:69, L-BFGS.cu:151) before any device work (runs on CPU)."""
    src = tmp_path / "v.cpp"
    src.write_text(_VARIANT_CALLER)
    exe = tmp_path / "v"
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o",
           str(exe), "-L", PKG, "-l:liblbfgs_hip.so", "-Wl,-rpath," + PKG]
    if how == "macro":
        cmd.insert(3, '-DLBFGS_CUDA_VARIANT="bogus"')
    subprocess.run(cmd, check=True, capture_output=True)
    env = dict(os.environ, LBFGS_CUDA_VARIANT="bogus") if how == "env" else None
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stderr
    assert "INVALID Unknown line search method: bogus" in r.stdout


def _rosen_seq(x):  # functions.cpp:26-36, left to right
    s = 0.0
    v = x.tolist()
    for i in range(len(v) - 1):
        s += 100 * (v[i + 1] - v[i] * v[i]) ** 2 + (1 - v[i]) ** 2
    return s


@pytest.mark.gpu
@pytest.mark.parametrize("cu", list(CUDA_MAINS))
def test_cuda_path_main_on_gpu(cu):
    """The unchanged main() of each CUDA-path file on the GPU: the variant's line search with the
    CUDA path's constants (constants.h, C2 = 0.7). Its printed solution (cout, 6 significant
    digits) and "Optimum value" equal the C ABI's run of the same problem (rosenbrock, m = 10,
    tol 1e-1, x0 ~ U(-2,2) from mt19937(42)); at n = 5 (L-BFGS.cu) also the canonical oracle's."""
    tag, ls, n = CUDA_MAINS[cu]
    exe = _cuda_exe(tag)
    if not os.path.exists(exe):
        pytest.skip("tests/cxx/_build/cuda_main_* not built (needs /root/reference where it is built)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    sol = [ln for ln in lines if ln.startswith("Found solution: ")]
    opt = [ln for ln in lines if ln.startswith("Optimum value: ")]
    assert len(sol) == 1 and len(opt) == 1
    x0 = O.x0_uniform(n, 42, -2.0, 2.0)
    first = [ln for ln in lines if ln.startswith("First x: ")][0]
    assert first.split()[2:5] == ["%g" % v for v in x0[:3]]
    import sys

    if PKG not in sys.path:
        sys.path.insert(0, PKG)
    import lbfgs_amd as LA

    with LA.Context(n, 10, device=0) as ctx:
        res = ctx.minimize("rosenbrock", x0, ls, 50000, tolerance=1e-1, consts=LA.constants("cuda"))
    x = res["x"]
    assert sol[0].split()[2:] == ["%g" % v for v in x]
    assert opt[0] == "Optimum value: %g" % _rosen_seq(x)
    if n == 5:
        o = O.lbfgs("rosenbrock", x0, ls, 10, 50000, 1e-1, mode=O.CANON, consts=dict(c2=0.7))
        assert np.array_equal(x.view(np.uint64), o["x"].view(np.uint64))


_PROGRESS_CALLER = r'''
#include <functions.h>
#include <random>
int main() {
    std::mt19937 gen(42);
    std::uniform_real_distribution<> dis(-2, 2);
    std::vector<double> x0(1000);
    for (double& v : x0) v = dis(gen);
    std::vector<double> x = LBFGS_CUDA(rosenbrock, rosenbrock_grad, x0, "backtracking", 40, 5, 1e-5);
    cout << "END " << x.size() << endl;
    return 0;
}
'''


@pytest.mark.gpu
def test_cuda_progress_lines(tmp_path):
    """LBFGS_CUDA_PROGRESS=1: LBFGS_CUDA prints the CUDA path's progress lines (L-BFGS.cu:115,
    307, 350-351: "Starting", then per iteration "alpha", "Iteration k: norm_g", "Optimum value")
    from the device trace, equal to the C ABI trace of the same solve; without it, none."""
    src = tmp_path / "p.cpp"
    src.write_text(_PROGRESS_CALLER)
    exe = tmp_path / "p"
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe), "-L", PKG, "-l:liblbfgs_hip.so", "-Wl,-rpath," + PKG], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, LBFGS_CUDA_PROGRESS="1"))
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    import sys

    if PKG not in sys.path:
        sys.path.insert(0, PKG)
    import lbfgs_amd as LA

    x0 = O.x0_uniform(1000, 42, -2.0, 2.0)
    with LA.Context(1000, 5, device=0) as ctx:
        t = ctx.minimize("rosenbrock", x0, "backtracking", 40, tolerance=1e-5, trace=True,
                         consts=LA.constants("cuda"))
    want = ["Starting"]
    for k in range(len(t["tr_f"]) - 1):
        want += ["alpha: %g" % t["tr_alpha"][k], "Iteration %d: norm_g = %g" % (k, t["tr_gnorm"][k + 1]),
                 "Optimum value: %g" % t["tr_f"][k + 1]]
    assert lines[:-1] == want and lines[-1] == "END 1000"
    assert len(want) == 1 + 3 * 40
    r0 = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r0.returncode == 0 and "Starting" not in r0.stdout and "alpha: " not in r0.stdout


@pytest.mark.gpu
def test_cuda_compat_env(tmp_path):
    """LBFGS_CUDA_COMPAT=1: LBFGS_CUDA runs L-BFGS.cu's own semantics (LBFGS_FLAG_CUDA_COMPAT) and
    prints its stdout as the library goes; it equals the C ABI's cuda_compat run of the same solve,
    which tests/test_gpu_cuda_compat.py pins to the oracle's restatement of the CUDA path"""
    src = tmp_path / "p.cpp"
    src.write_text(_PROGRESS_CALLER)
    exe = tmp_path / "p"
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe), "-L", PKG, "-l:liblbfgs_hip.so", "-Wl,-rpath," + PKG], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, LBFGS_CUDA_COMPAT="1"))
    assert r.returncode == 0, r.stderr
    import sys

    if PKG not in sys.path:
        sys.path.insert(0, PKG)
    import lbfgs_amd as LA

    x0 = O.x0_uniform(1000, 42, -2.0, 2.0)
    with LA.Context(1000, 5, device=0) as ctx:
        t = ctx.minimize("rosenbrock", x0, "backtracking", 40, tolerance=1e-5, cuda_compat=True,
                         consts=LA.constants("cuda"))
    lines = r.stdout.splitlines()
    assert lines[0] == "Starting" and lines[-1] == "END 1000"
    assert lines[:-1] == t["messages"].splitlines()


_STRINGLESS_CALLER = r'''
#include <functions.h>
#include <random>
int main() {
    std::mt19937 gen(42);
    std::uniform_real_distribution<> dis(-2, 2);
    std::vector<double> x0(1000);
    for (double& v : x0) v = dis(gen);
    std::vector<double> x = LBFGS_CUDA(rosenbrock, rosenbrock_grad, x0, 40, 5, 1e-5);
    cout << "END " << x.size() << endl;
    return 0;
}
'''


@pytest.mark.gpu
@pytest.mark.parametrize("how,variant", [("define", "wolfe"), ("env", "wolfe"), ("env", "backtracking"),
                                         ("env", "interpolation"), ("define", "backtracking_wolfe")])
def test_cuda_compat_variant_stringless(tmp_path, how, variant):
    """LBFGS_CUDA_COMPAT=1 with the string-less LBFGS_CUDA: the variant file's own loop and search
    (LBFGS_FLAG_CUDA_VARIANT), whether the variant is named by -DLBFGS_CUDA_VARIANT or by
    LBFGS_CUDA_VARIANT; its stdout equals the C ABI's run of the same solve"""
    src = tmp_path / "v.cpp"
    src.write_text(_STRINGLESS_CALLER)
    exe = tmp_path / "v"
    cmd = ["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe), "-L", PKG,
           "-l:liblbfgs_hip.so", "-Wl,-rpath," + PKG]
    env = dict(os.environ, LBFGS_CUDA_COMPAT="1")
    if how == "define":
        cmd.insert(3, f'-DLBFGS_CUDA_VARIANT="{variant}"')
    else:
        env["LBFGS_CUDA_VARIANT"] = variant
    subprocess.run(cmd, check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    import sys

    if PKG not in sys.path:
        sys.path.insert(0, PKG)
    import lbfgs_amd as LA

    x0 = O.x0_uniform(1000, 42, -2.0, 2.0)
    with LA.Context(1000, 5, device=0) as ctx:
        t = ctx.minimize("rosenbrock", x0, variant, 40, tolerance=1e-5, cuda_compat=True, cuda_variant=True,
                         consts=LA.constants("cuda"))
    lines = r.stdout.splitlines()
    assert lines[-1] == "END 1000" and lines[:-1] == t["messages"].splitlines()


_EMPTY_CALLER = r'''
#include <cstdio>
#include <stdexcept>
#include <benchmark.h>
#include <lbfgs.h>
int main() {
    std::vector<double> x0;
    try { LBFGS(rosenbrock, rosenbrock_grad, x0, "backtracking"); }
    catch (const std::invalid_argument& e) { std::printf("INVALID %s\n", e.what()); }
    try { LBFGS_CUDA(rosenbrock, rosenbrock_grad, x0, "wolfe", 10, 5, 1e-5); }
    catch (const std::invalid_argument& e) { std::printf("INVALID %s\n", e.what()); }
    return 0;
}
'''


def test_empty_x0_throws(tmp_path):
    """An empty x0 throws std::invalid_argument before any device work (runs on CPU); the
    reference reads out of bounds there (benchmark.cpp:61, size_t wrap)"""
    src = tmp_path / "e.cpp"
    src.write_text(_EMPTY_CALLER)
    exe = tmp_path / "e"
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe), "-L", PKG,
                    "-l:liblbfgs_hip.so", "-Wl,-rpath," + PKG], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ["INVALID x0 must not be empty"] * 2
