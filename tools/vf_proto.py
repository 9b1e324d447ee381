#!/usr/bin/env python3
"""Numerical prototype of the vector-free (Gram-matrix) two-loop against the standard two-loop
on the benchmark objectives (numpy, float64). Prints per-iteration relative differences in f and
iterations to convergence. Not product code: the design check for LBFGS_FLAG_VECTOR_FREE."""
import sys

import numpy as np

sys.path.insert(0, "tests")
import oracle_lib as O  # noqa: E402


def rosen(x):
    t1 = x[1:] - x[:-1] ** 2
    t2 = 1 - x[:-1]
    return float(np.sum(100 * t1 * t1 + t2 * t2))


def rosen_g(x):
    g = np.zeros_like(x)
    t1 = x[1:] - x[:-1] ** 2
    g[:-1] += -400 * x[:-1] * t1 - 2 * (1 - x[:-1])
    g[1:] += 200 * t1
    return g


def standard(x, f, gf, m, maxit, tol):
    g = gf(x); fx = f(x); S, Y = [], []
    fs = []
    for k in range(maxit):
        fs.append(fx)
        if np.linalg.norm(g) < tol:
            break
        q = g.copy(); al = []
        for s, y in zip(reversed(S), reversed(Y)):
            a = (s @ q) / (s @ y); al.append(a); q -= a * y
        if S:
            q *= (S[-1] @ Y[-1]) / (Y[-1] @ Y[-1])
        for (s, y), a in zip(zip(S, Y), reversed(al)):
            b = (y @ q) / (s @ y); q += s * (a - b)
        d = -q
        gd = g @ d
        alpha = 1.0
        while fx - f(x + alpha * d) < 1e-4 * alpha * gd:
            alpha *= 0.5
            if alpha < 1e-8:
                break
        xn = x + alpha * d; gn = gf(xn)
        s, y = xn - x, gn - g
        if s @ y > 0:
            S.append(s); Y.append(y)
            if len(S) > m:
                S.pop(0); Y.pop(0)
        x, g, fx = xn, gn, f(xn)
    return np.array(fs), x


def vector_free(x, f, gf, m, maxit, tol, derive_s=True):
    """basis b = [s_0..s_{h-1}, y_0..y_{h-1}, g]; Gram B; only Gram rows of y_new, g_new
    (and s_new.y_new) are 'direct' dots; s_new rows derived as alpha * c^T B_old."""
    g = gf(x); fx = f(x)
    S, Y = [], []
    B = np.array([[g @ g]])
    fs = []
    for k in range(maxit):
        fs.append(fx)
        h = len(S)
        if np.sqrt(B[-1, -1]) < tol:
            break
        nb = 2 * h + 1
        delta = np.zeros(nb); delta[-1] = 1.0
        al = np.zeros(h)
        if h:
            for i in range(h - 1, -1, -1):
                rho = 1.0 / B[i, h + i]
                al[i] = rho * (B[i] @ delta)
                delta[h + i] -= al[i]
            delta *= B[h - 1, 2 * h - 1] / B[2 * h - 1, 2 * h - 1]
            for i in range(h):
                rho = 1.0 / B[i, h + i]
                beta = rho * (B[h + i] @ delta)
                delta[i] += al[i] - beta
        c = -delta
        basis = S + Y + [g]
        d = sum(ci * bi for ci, bi in zip(c, basis))
        gd = c @ B[-1]                   # g.d from the Gram row of g
        alpha = 1.0
        while fx - f(x + alpha * d) < 1e-4 * alpha * gd:
            alpha *= 0.5
            if alpha < 1e-8:
                break
        xn = x + alpha * d; gn = gf(xn)
        s, y = xn - x, gn - g
        # direct dots (the commit pass)
        yb = np.array([y @ b for b in basis[:-1]]); gb = np.array([gn @ b for b in basis[:-1]])
        ggo = gn @ g; gg = gn @ gn; yy = y @ y; yg = y @ gn; sy = s @ y
        # derived: s_new . v = alpha * c . B[:, v]
        sB = alpha * (c @ B)               # s_new . old basis (incl. g_old)
        sg = alpha * (c[:-1] @ gb + c[-1] * ggo)
        ss = alpha * alpha * (c @ B @ c)
        if not derive_s:
            sB = np.array([s @ b for b in basis]); sg = s @ gn; ss = s @ s
        keep = list(range(h))
        if sy > 0:
            if h == m:
                keep = keep[1:]
            Sn = [S[i] for i in keep] + [s]; Yn = [Y[i] for i in keep] + [y]
        else:
            Sn, Yn = S, Y
        h2 = len(Sn)
        B2 = np.zeros((2 * h2 + 1, 2 * h2 + 1))
        # indices into the old basis of the kept vectors
        if sy > 0:
            old_s = keep; old_y = [h + i for i in keep]
        else:
            old_s = list(range(h)); old_y = [h + i for i in range(h)]
        olds = old_s + old_y
        newpos_old = [j for j in range(len(keep) if sy > 0 else h)] + \
                     [h2 + j for j in range(len(keep) if sy > 0 else h)]
        for a, oa in zip(newpos_old, olds):
            for b_, ob in zip(newpos_old, olds):
                B2[a, b_] = B[oa, ob]
            B2[a, -1] = B2[-1, a] = gb[oa]
        B2[-1, -1] = gg
        if sy > 0:
            si, yi = h2 - 1, 2 * h2 - 1
            for a, oa in zip(newpos_old, olds):
                B2[si, a] = B2[a, si] = sB[oa]
                B2[yi, a] = B2[a, yi] = yb[oa]
            B2[si, si] = ss; B2[yi, yi] = yy; B2[si, yi] = B2[yi, si] = sy
            B2[si, -1] = B2[-1, si] = sg; B2[yi, -1] = B2[-1, yi] = yg
        S, Y, B, g, x, fx = Sn, Yn, B2, gn, xn, f(xn)
    return np.array(fs), x


def main():
    for n, m in [(10000, 5), (1000, 10), (100000, 10)]:
        x0 = O.x0_uniform(n, 42, -2.0, 2.0)
        fa, xa = standard(x0.copy(), rosen, rosen_g, m, 20000, 1e-5)
        fb, xb = vector_free(x0.copy(), rosen, rosen_g, m, 20000, 1e-5)
        fc, xc = vector_free(x0.copy(), rosen, rosen_g, m, 20000, 1e-5, derive_s=False)
        k = min(len(fa), len(fb))
        rel = np.abs(fa[:k] - fb[:k]) / np.abs(fa[:k])
        hz = int(np.argmax(rel > 1e-10)) if np.any(rel > 1e-10) else k
        print(f"n={n} m={m}: standard {len(fa)-1} its f={fa[-1]:.3e}; vector-free(derived) {len(fb)-1} its "
              f"f={fb[-1]:.3e}; vector-free(direct) {len(fc)-1} its; 1e-10 horizon {hz}", flush=True)


if __name__ == "__main__":
    main()
