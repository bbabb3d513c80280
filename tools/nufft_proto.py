#!/usr/bin/env python3
"""Design prototype (numpy, not product): the reciprocal Ewald sum of RCK:513-556 evaluated
by ES-kernel spreading + pruned DFT + interpolation (a type-1/type-2 NUFFT pair), compared
with the exact half-space sum.  Used to choose the kernel width w and the grid size.

  python tools/nufft_proto.py [n_waters] [w ...]
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "openmm-chargeflux_amd")]
from openmmcoul import testsystems as ts  # noqa: E402

KE = 138.935456
SIGMAS = [float(s) for s in os.environ.get("SIGMAS", "2.0,1.5").split(",")]


def es_kernel(t, w, beta):
    """exp(beta (sqrt(1-(2t/w)^2) - 1)) on |t| < w/2, t in grid units."""
    z = 2.0 * t / w
    out = np.zeros_like(t)
    m = np.abs(z) < 1
    out[m] = np.exp(beta * (np.sqrt(1 - z[m] ** 2) - 1))
    return out


def es_kernel_d(t, w, beta):
    z = 2.0 * t / w
    out = np.zeros_like(t)
    m = np.abs(z) < 1
    s = np.sqrt(1 - z[m] ** 2)
    out[m] = np.exp(beta * (s - 1)) * beta * (-z[m] / s) * (2.0 / w)
    return out


def es_hat(xi, w, beta, nq=200):
    """phi_hat(xi) = int phi(t) e^{2 pi i xi t} dt (real, even), Gauss-Legendre."""
    x, wt = np.polynomial.legendre.leggauss(nq)
    t = x * w / 2
    wt = wt * w / 2
    return (wt[None, :] * es_kernel(t, w, beta)[None, :] * np.cos(2 * np.pi * np.outer(xi, t))).sum(1)


def exact_recip(pos, q, L, alpha, kmax):
    """Full-box form of the reference half-space sum: E = 1/2 sum_{n!=0} c a |S|^2."""
    V = L[0] * L[1] * L[2]
    c = 4 * np.pi * KE / V
    u = pos / L
    n1 = [np.arange(-k + 1, k) for k in kmax]
    ex = [np.exp(2j * np.pi * np.outer(u[:, d], n1[d])) for d in range(3)]
    S = np.einsum("j,ja,jb,jc->abc", q, ex[0], ex[1], ex[2])
    kx, ky, kz = np.meshgrid(*(2 * np.pi * n1[d] / L[d] for d in range(3)), indexing="ij")
    k2 = kx**2 + ky**2 + kz**2
    k2[kmax[0] - 1, kmax[1] - 1, kmax[2] - 1] = 1.0
    a = np.exp(-k2 / (4 * alpha**2)) / k2
    a[kmax[0] - 1, kmax[1] - 1, kmax[2] - 1] = 0.0
    E = 0.5 * c * (a * np.abs(S) ** 2).sum()
    f = c * a * np.conj(S)
    phi = np.einsum("abc,ja,jb,jc->j", f, ex[0], ex[1], ex[2]).real
    gx = np.einsum("abc,ja,jb,jc->j", f * 1j * kx, ex[0], ex[1], ex[2]).real
    gy = np.einsum("abc,ja,jb,jc->j", f * 1j * ky, ex[0], ex[1], ex[2]).real
    gz = np.einsum("abc,ja,jb,jc->j", f * 1j * kz, ex[0], ex[1], ex[2]).real
    F = -q[:, None] * np.stack([gx, gy, gz], 1)
    return E, phi, F


def nufft_recip(pos, q, L, alpha, kmax, w, ng, beta=None):
    if beta is None:
        sigma = min(ng[d] / (2 * kmax[d] - 1) for d in range(3))
        beta = 0.97 * np.pi * (1 - 1 / (2 * sigma)) * w
    V = L[0] * L[1] * L[2]
    c = 4 * np.pi * KE / V
    u = (pos / L) % 1.0
    N = len(q)
    # per-dim kernel values: first grid index g0 = ceil(s - w/2), taps g0..g0+w-1
    taps, vals, dvals = [], [], []
    for d in range(3):
        s = u[:, d] * ng[d]
        g0 = np.ceil(s - w / 2).astype(int)
        g = g0[:, None] + np.arange(w)[None, :]
        t = g - s[:, None]
        taps.append(g % ng[d])
        vals.append(es_kernel(t, w, beta))
        dvals.append(-es_kernel_d(t, w, beta) * ng[d] / L[d])   # d/dx of phi(g - ng x/L)
    b = np.zeros(ng)
    for j in range(N):
        blk = q[j] * np.einsum("a,b,c->abc", vals[0][j], vals[1][j], vals[2][j])
        b[np.ix_(taps[0][j], taps[1][j], taps[2][j])] += blk
    n1 = [np.arange(-k + 1, k) for k in kmax]
    dft = [np.exp(2j * np.pi * np.outer(n1[d], np.arange(ng[d])) / ng[d]) for d in range(3)]
    B = np.einsum("xyz,ax,by,cz->abc", b, dft[0], dft[1], dft[2])
    ph = [es_hat(n1[d] / ng[d], w, beta) for d in range(3)]
    deconv = np.einsum("a,b,c->abc", 1 / ph[0], 1 / ph[1], 1 / ph[2])
    S = B * deconv
    kx, ky, kz = np.meshgrid(*(2 * np.pi * n1[d] / L[d] for d in range(3)), indexing="ij")
    k2 = kx**2 + ky**2 + kz**2
    ctr = (kmax[0] - 1, kmax[1] - 1, kmax[2] - 1)
    k2[ctr] = 1.0
    a = np.exp(-k2 / (4 * alpha**2)) / k2
    a[ctr] = 0.0
    E = 0.5 * c * (a * np.abs(S) ** 2).sum()
    f = c * a * np.conj(S) * deconv
    G = np.einsum("abc,ax,by,cz->xyz", f, dft[0], dft[1], dft[2]).real
    phi = np.zeros(N)
    grad = np.zeros((N, 3))
    for j in range(N):
        sub = G[np.ix_(taps[0][j], taps[1][j], taps[2][j])]
        phi[j] = np.einsum("abc,a,b,c->", sub, vals[0][j], vals[1][j], vals[2][j])
        grad[j, 0] = np.einsum("abc,a,b,c->", sub, dvals[0][j], vals[1][j], vals[2][j])
        grad[j, 1] = np.einsum("abc,a,b,c->", sub, vals[0][j], dvals[1][j], vals[2][j])
        grad[j, 2] = np.einsum("abc,a,b,c->", sub, vals[0][j], vals[1][j], dvals[2][j])
    F = -q[:, None] * grad
    return E, phi, F


def kmax_for(L, alpha, tol):
    """RCK:403-420 (getEwaldParamValue): smallest k meeting tol, rounded up to odd."""
    k = 1
    while 0.05 * math.sqrt(L * alpha) * k * math.exp(-(math.pi * k / (L * alpha)) ** 2) > tol:
        k += 1
    return k if k % 2 == 1 else k + 1


def main():
    nw = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    ws = [int(x) for x in sys.argv[2:]] or [8, 10, 12, 14]
    system, force, pos, box = ts.water_box(nw, cutoff=1.0, ewald_tol=1e-3 if nw <= 1000 else 1e-4)
    L = np.array([box[0][0], box[1][1], box[2][2]])
    q = np.array([force.getParticleParameters(i)[0] for i in range(len(pos))])
    alpha = math.sqrt(-math.log(2 * (1e-3 if nw <= 1000 else 1e-4))) / 1.0
    kmax = [kmax_for(L[d], alpha, 1e-3 if nw <= 1000 else 1e-4) for d in range(3)]
    E0, phi0, F0 = exact_recip(pos, q, L, alpha, kmax)
    print(f"N={len(q)} kmax={kmax} E_rec={E0:.10f} |F|max={np.abs(F0).max():.3f} |phi|max={np.abs(phi0).max():.3f}")
    for w in ws:
        for sig in SIGMAS:
            ng = [int(math.ceil(sig * (2 * k - 1) / 2) * 2) for k in kmax]
            E1, phi1, F1 = nufft_recip(pos, q, L, alpha, kmax, w, ng)
            print(f"w={w:2d} ng={ng[0]} dE={abs(E1-E0):.2e} (rel {abs(E1-E0)/abs(E0):.1e}) "
                  f"dphi={np.abs(phi1-phi0).max():.2e} dF={np.abs(F1-F0).max():.2e}")


if __name__ == "__main__":
    main()
