"""Host prototype behind the cluster-pair half list (cf_kernels_cluster.hip).

Answers, on the C3 box (96 000 atoms) or a drifted 12 000-atom box, the questions that fixed the
design before any kernel was written:
  * how many (i, j) atom slots the cluster pairs within rc + skin cover per pair within rc
    (cluster size 4 or 8, within-cell order: atom index, Morton, serpentine z-columns);
  * the phase-B efficiency of the per-i-atom queues (4 i atoms x 16 lanes, ring of 64);
  * the entries per i-cluster under the two cluster-level half rules (cluster index vs x key)
    as the atoms drift away from the lattice the synthetic boxes start on.

    python tools/cluster_proto.py efficiency      # C3: slots per pair, queue efficiency
    python tools/cluster_proto.py counts          # 4000 shuffled waters drifting: entries per i-cluster
"""
import sys

import numpy as np
from scipy.spatial import cKDTree

sys.path.insert(0, "openmm-chargeflux_amd")
from openmmcoul import testsystems as ts  # noqa: E402


def cell_order(x, L, rl, order, zc=4):
    """Sorted atom order and cell bounds as k_cell_hist / k_cell_order build them."""
    N = len(x)
    nc = int(np.floor(L / rl))
    cs = L / nc
    w = x - L * np.floor(x / L)
    c3 = np.minimum((w / cs).astype(int), nc - 1)
    key = (c3[:, 0] * nc + c3[:, 1]) * nc + c3[:, 2]
    loc = np.clip(w / cs - c3, 0, 0.999999)
    if order == "index":
        sk = np.zeros(N)
    elif order == "zcol":   # serpentine z-columns (k_cell_order)
        ca, cb = np.floor(loc[:, 0] * zc), np.floor(loc[:, 1] * zc)
        cb = np.where(ca % 2 == 1, zc - 1 - cb, cb)
        col = ca * zc + cb
        sk = col + np.where(col % 2 == 1, 0.999999 - loc[:, 2], loc[:, 2])
    else:   # Morton code of 4 x 4 x 4 sub-cells
        s3 = np.minimum((loc * 4).astype(int), 3)
        sk = np.zeros(N)
        for b in range(2):
            for d in range(3):
                sk += ((s3[:, d] >> b) & 1) << (3 * b + d)
    o = np.lexsort((np.arange(N), sk, key))
    cnt = np.bincount(key, minlength=nc ** 3)
    return nc, w, o, np.r_[0, np.cumsum(cnt)]


def clusters(w, o, cstart, M):
    out = []
    for c in range(len(cstart) - 1):
        for f in range(cstart[c], cstart[c + 1], M):
            out.append(o[f:min(f + M, cstart[c + 1])])
    return out


def cluster_list(x, L, rc, skin, M, order, rule="xkey"):
    """Per i-cluster list of j-clusters (half rule over the 18-cell window, as k_cl_build)."""
    rl = rc + skin
    nc, w, o, cstart = cell_order(x, L, rl, order)
    cl = clusters(w, o, cstart, M)
    cell_of = np.repeat(np.arange(nc ** 3), [(cstart[c + 1] - cstart[c] + M - 1) // M for c in range(nc ** 3)])
    lo = np.array([w[c].min(0) for c in cl])
    hi = np.array([w[c].max(0) for c in cl])
    cen, half = (lo + hi) / 2, (hi - lo) / 2
    t = cKDTree(cen, boxsize=L)
    pr = t.query_pairs(rl + 2 * np.linalg.norm(half, axis=1).max(), output_type="ndarray")
    d = cen[pr[:, 1]] - cen[pr[:, 0]]
    d -= L * np.round(d / L)
    gap = np.maximum(np.abs(d) - half[pr[:, 0]] - half[pr[:, 1]], 0)
    pr = pr[(gap ** 2).sum(1) <= rl * rl]
    a, b = pr[:, 0], pr[:, 1]
    cx = cell_of // (nc * nc)
    dx = (cx[b] - cx[a]) % nc
    if rule == "index":
        own_a = (dx == 1) | ((dx == 0) & (b > a))
    else:
        xa, xb = cen[a, 0], cen[b, 0]
        own_a = (dx == 1) | ((dx == 0) & ((xb > xa) | ((xb == xa) & (b > a))))
    ii, jj = np.where(own_a, a, b), np.where(own_a, b, a)
    lists = [[] for _ in cl]
    for p, q in zip(ii, jj):
        lists[p].append(q)
    for p in range(len(cl)):
        lists[p].append(p)
    return cl, lists


def queue_efficiency(x, L, rc, cl, lists, sample=1500, cap=64, NI=4, LPI=16, JPS=4):
    rng = np.random.default_rng(0)
    steps, pairs, stepa = 0, 0, 0
    for ci in rng.choice(len(cl), min(sample, len(cl)), replace=False):
        I = cl[ci]
        hits = []
        js = lists[ci]
        for s in range(0, len(js), JPS):
            h = np.zeros(NI, int)
            for cj in js[s:s + JPS]:
                J = cl[cj]
                d = x[I][:, None, :] - x[J][None, :, :]
                d -= L * np.round(d / L)
                ok = (d ** 2).sum(-1) <= rc * rc
                if cj == ci:
                    ok &= np.triu(np.ones((len(I), len(J)), bool), 1)
                h[:len(I)] += ok.sum(1)
            hits.append(h)
        stepa += len(hits)
        q = np.zeros(NI, int)
        for h in hits:
            q += h
            pairs += h.sum()
            while (q >= LPI).all():
                q -= LPI
                steps += 1
            while (q > cap - LPI).any():
                q = np.maximum(q - LPI, 0)
                steps += 1
        while q.any():
            q = np.maximum(q - LPI, 0)
            steps += 1
    return pairs / (64 * steps), pairs / stepa


def efficiency():
    _, _, pos, box = ts.make("C3")
    L = box[0, 0]
    x = pos % L
    npairs = (cKDTree(x, boxsize=L).count_neighbors(cKDTree(x, boxsize=L), 1.0) - len(x)) / 2
    for M, order in ((4, "index"), (4, "morton"), (4, "zcol"), (8, "zcol")):
        cl, lists = cluster_list(x, L, 1.0, 0.15, M, order)
        slots = sum(len(v) for v in lists) * M * M
        msg = f"M={M} {order:6s}: cluster pairs {sum(len(v) for v in lists)}  slots/pair {slots / npairs:.2f}"
        if M == 4:
            eff, per = queue_efficiency(x, L, 1.0, cl, lists)
            msg += f"  phase-B efficiency {eff:.3f}  hits per phase-A step {per:.1f}"
        print(msg)


def counts():
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4)
    perm = np.random.default_rng(2).permutation(4000)
    x = pos.reshape(4000, 3, 3)[perm].reshape(-1, 3)
    L = box[0, 0]
    rng = np.random.default_rng(7)
    for step in range(int(sys.argv[2]) if len(sys.argv) > 2 else 4):
        for rule in ("xkey",) if step > 3 else ("index", "xkey"):
            _, lists = cluster_list(x, L, 1.0, 0.15, 4, "zcol", rule)
            n = np.array([len(v) for v in lists])
            print(f"step {step} rule {rule:5s}: entries per i-cluster mean {n.mean():.1f}  "
                  f"p99 {np.percentile(n, 99):.0f}  max {n.max()}")
        x = x + np.array([0.03, 0.015, 0.0075]) + rng.normal(scale=0.003, size=x.shape)


if __name__ == "__main__":
    {"efficiency": efficiency, "counts": counts}[sys.argv[1] if len(sys.argv) > 1 else "efficiency"]()
