// cf_kernels_core.hip — charge flux, cell list, direct space, exclusions, chain rule,
// energy assembly.  Hand-written HIP for gfx950 (wave64).  All per-atom sums are
// gathers in a fixed order (no atomics), so results are bitwise reproducible.
//
// Reference semantics: platforms/reference/src/ReferenceCoulKernels.cpp (RCK).
#include <algorithm>
#include <type_traits>

#include "cf_pair.h"

namespace cf {


// ---------------------------------------------------------------------------------
// 1. flux terms: one lane per term writes its charge deltas (slots) and its dq/dx
//    block in the reference's entry order.  Bonds RCK:42-80, angles RCK:81-162,
//    waters RCK:163-227.
// ---------------------------------------------------------------------------------
// first dq/dx double of term t: bonds (12 doubles each), then angles (27), then waters (27) --
// the terms of a block write one contiguous range
__device__ __forceinline__ long dqdx_start(int t, int nb, int na) {
    const int b = min(t, nb), an = max(0, min(t, nb + na) - nb), w = max(0, t - nb - na);
    return 3L * (4L * b + 9L * an + 9L * w);
}

__global__ void __launch_bounds__(256) k_flux_terms(int nterms, int nb, int na, const int4* __restrict__ tidx,
                                                    const double* __restrict__ tpar, const double* __restrict__ pos,
                                                    double3 L, double3 T, int pbc, double* __restrict__ dq_slot,
                                                    double* __restrict__ dqdx) {
    // the block's dq/dx blocks are staged in LDS and written out as one coalesced run (each
    // lane's 12 or 27 doubles written straight to memory spread every store instruction over
    // ~100 cache lines)
    __shared__ double st[256 * 27];
    const int t0 = blockIdx.x * blockDim.x;
    const int t = t0 + threadIdx.x;
    const long base = dqdx_start(t0, nb, na);
    if (t < nterms) {
        int4 ti = tidx[t];
        const double* p = tpar + 5 * t;
        double* o = st + (dqdx_start(t, nb, na) - base);
        if (ti.x == 0) {  // bond p1-p2
            double3 d = delta_r(ld3(pos, ti.y), ld3(pos, ti.z), L, pbc, T);
            double r = sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
            double k = p[0], dq = k * (r - p[1]);
            dq_slot[2 * t] = dq;
            dq_slot[2 * t + 1] = -dq;
            double c = k / r;
            double v[3] = {c * d.x, c * d.y, c * d.z};
#pragma unroll
            for (int j = 0; j < 3; j++) { o[j] = -v[j]; o[3 + j] = v[j]; o[6 + j] = v[j]; o[9 + j] = -v[j]; }
        } else if (ti.x == 1) {  // angle p1-p2-p3, p2 central
            int a = t - nb;
            double3 x1 = ld3(pos, ti.y), x2 = ld3(pos, ti.z), x3 = ld3(pos, ti.w);
            double3 d21 = delta_r(x2, x1, L, pbc, T), d23 = delta_r(x2, x3, L, pbc, T), d13 = delta_r(x1, x3, L, pbc, T);
            double r21_2 = d21.x * d21.x + d21.y * d21.y + d21.z * d21.z;
            double r23_2 = d23.x * d23.x + d23.y * d23.y + d23.z * d23.z;
            double r13_2 = d13.x * d13.x + d13.y * d13.y + d13.z * d13.z;
            double r21 = sqrt(r21_2), r23 = sqrt(r23_2);
            double cost = (r23_2 + r21_2 - r13_2) / 2 / r21 / r23;
            double k = p[0];
            double dq = k * (acos(cost) - p[1]);
            int s = 2 * nb + 3 * a;
            dq_slot[s] = dq; dq_slot[s + 1] = -2 * dq; dq_slot[s + 2] = dq;
            double inv_s = 1 / sqrt(1 - cost * cost);
            double c1 = k * (1.0 / r21 / r23) * inv_s;
            double c21 = k * cost * inv_s / r21_2;
            double c23 = k * cost * inv_s / r23_2;
            double a21[3] = {d21.x, d21.y, d21.z}, a23[3] = {d23.x, d23.y, d23.z};
#pragma unroll
            for (int j = 0; j < 3; j++) {
                double v1 = -c1 * a23[j] + c21 * a21[j];
                double v3 = -c1 * a21[j] + c23 * a23[j];
                double v2 = -v1 - v3;
                o[j] = v1; o[3 + j] = v2; o[6 + j] = v3;
                o[9 + j] = -2 * v1; o[12 + j] = -2 * v2; o[15 + j] = -2 * v3;
                o[18 + j] = v1; o[21 + j] = v2; o[24 + j] = v3;
            }
        } else {  // water O,H1,H2
            int w = t - nb - na;
            double3 x1 = ld3(pos, ti.y), x2 = ld3(pos, ti.z), x3 = ld3(pos, ti.w);
            double3 d12 = delta_r(x1, x2, L, pbc, T), d13 = delta_r(x1, x3, L, pbc, T), d23 = delta_r(x2, x3, L, pbc, T);
            double r12 = sqrt(d12.x * d12.x + d12.y * d12.y + d12.z * d12.z);
            double r13 = sqrt(d13.x * d13.x + d13.y * d13.y + d13.z * d13.z);
            double r23 = sqrt(d23.x * d23.x + d23.y * d23.y + d23.z * d23.z);
            double k1 = p[0], k2 = p[1], kub = p[2], b0 = p[3], ub0 = p[4];
            double dq2 = k1 * (r12 - b0) + k2 * (r13 - b0) + kub * (r23 - ub0);
            double dq3 = k1 * (r13 - b0) + k2 * (r12 - b0) + kub * (r23 - ub0);
            int s = 2 * nb + 3 * na + 3 * w;
            dq_slot[s] = -dq2 - dq3; dq_slot[s + 1] = dq2; dq_slot[s + 2] = dq3;
            double e12[3] = {d12.x, d12.y, d12.z}, e13[3] = {d13.x, d13.y, d13.z}, e23[3] = {d23.x, d23.y, d23.z};
#pragma unroll
            for (int j = 0; j < 3; j++) {
                double n12 = e12[j] / r12, n13 = e13[j] / r13, n23 = e23[j] / r23;
                double a12k1 = k1 * n12, a12k2 = k2 * n12, a13k1 = k1 * n13, a13k2 = k2 * n13, ub = kub * n23;
                o[0 + j] = a12k1 + a12k2 + a13k1 + a13k2;
                o[3 + j] = -a12k1 - a12k2 + 2 * ub;
                o[6 + j] = -a13k2 - a13k1 - 2 * ub;
                o[9 + j] = -a12k1 - a13k2;
                o[12 + j] = a12k1 - ub;
                o[15 + j] = a13k2 + ub;
                o[18 + j] = -a12k2 - a13k1;
                o[21 + j] = a12k2 - ub;
                o[24 + j] = a13k1 + ub;
            }
        }
    }
    __syncthreads();
    const int len = (int)(dqdx_start(min(t0 + (int)blockDim.x, nterms), nb, na) - base);
    for (int e = threadIdx.x; e < len; e += blockDim.x) dqdx[base + e] = st[e];
}
__global__ void __launch_bounds__(256) k_atoms_prep(int n, const double* __restrict__ q0,
                                                    const int* __restrict__ qs, const int* __restrict__ qslot,
                                                    const double* __restrict__ dq_slot, int pbc, double alpha, double ke,
                                                    double* __restrict__ q, double* __restrict__ dedq_self,
                                                    double* __restrict__ e_atom, const double* __restrict__ pos,
                                                    const double* __restrict__ pos_ref, double lim2,
                                                    int* __restrict__ skin_flag) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (skin_flag) {
        bool moved = false;
        if (i < n) {
            double3 x = ld3(pos, i), r = ld3(pos_ref, i);
            double dx = x.x - r.x, dy = x.y - r.y, dz = x.z - r.z;
            moved = !(dx * dx + dy * dy + dz * dz <= lim2);  // NaN counts as moved
        }
        if (__ballot(moved) && (threadIdx.x & 63) == 0) atomicOr(skin_flag, 1);
    }
    if (i >= n) return;
    double qi = q0[i];
    for (int s = qs[i]; s < qs[i + 1]; s++) qi += dq_slot[qslot[s]];
    q[i] = qi;
    if (pbc) {
        const double c = ke * alpha / sqrt(kPi);
        dedq_self[i] = -2 * c * qi;
        e_atom[3 * i] = -c * qi * qi;
    } else {
        dedq_self[i] = 0;
        e_atom[3 * i] = 0;
    }
}

// ---------------------------------------------------------------------------------
// 3. cell list (replaces OpenMM computeNeighborListVoxelHash, RCK:559): wrap, bin, sort
//    by cell (atom index within a cell: the order of a stable sort), cell bounds, sorted
//    wrapped (x,y,z,q) and LJ.  A deterministic counting sort whose kernels all return at
//    once when the device rebuild flag is clear, so a kept list costs only launches:
//      clear counts -> keys + histogram -> scan (bounds) -> scatter -> order within cells
//      -> [owned compaction] -> commit (or refresh of the kept list's coordinates)
// ---------------------------------------------------------------------------------

// keys + histogram (wave-aggregated atomics: provisional ranks), then the block that
// finishes last turns the counts into cell bounds (no separate scan launch).  Multi-rank
// (own_cnt != null): also the owned atoms per cell and their scan, the first list row of each
// cell, from which k_cell_order writes the owned rows in cell-sorted order.
__global__ void __launch_bounds__(256) k_cell_hist(int n, const int* __restrict__ flag, const double* __restrict__ pos,
                                                   double3 L, double3 T, int3 nc, int* __restrict__ key, int* __restrict__ rank,
                                                   int* __restrict__ cnt, int* __restrict__ ticket,
                                                   int* __restrict__ cstart, int* __restrict__ cend, int lo, int hi,
                                                   int* __restrict__ own_cnt, int* __restrict__ own_start,
                                                   int* __restrict__ err) {
    __shared__ int sh[256];
    if (!*flag) return;   // uniform over the grid
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < n;
    int k = 0;
    if (valid) {
        // cells in fractional coordinates of the lattice-wrapped position (a sheared box's cells
        // are parallelepipeds; nc per direction from the perpendicular widths, cf_api.hip set_cells)
        const double3 x = ld3(pos, i);
        const double3 wp = wrap_by(x, floor3(fractional(x, L, T)), L, T);
        const double3 f = fractional(wp, L, T);
        const double fs[3] = {f.x, f.y, f.z};
        int ncs[3] = {nc.x, nc.y, nc.z};
        int c[3];
#pragma unroll
        for (int d = 0; d < 3; d++) {
            int ci = (int)(fs[d] * ncs[d]);
            c[d] = ci < 0 ? 0 : (ci >= ncs[d] ? ncs[d] - 1 : ci);
        }
        k = (c[0] * nc.y + c[1]) * nc.z + c[2];
        key[i] = k;
    }
    const int r = wave_agg_inc(cnt, k, valid);   // provisional slot; k_cell_order fixes the order
    if (valid) rank[i] = r;
    if (own_cnt) (void)wave_agg_inc(own_cnt, k, valid && i >= lo && i < hi);
    if (!last_block_done(ticket)) return;
    const int ncell = nc.x * nc.y * nc.z;
    const int total = block_counts_to_bounds<256>(ncell, cnt, cstart, cend, false, sh);
    // guard: the counts add up to the atoms (k_cell_scatter re-zeroes them after each build); bounds
    // that do not are replaced by empty cells, so no kernel after this one indexes past N (the
    // scan's total, block-uniform: no read-back of cend[ncell - 1])
    if (total != n) {
        __syncthreads();   // every thread's bounds stores before they are overwritten
        for (int c = threadIdx.x; c < ncell; c += blockDim.x) { cstart[c] = 0; cend[c] = 0; }
        if (threadIdx.x == 0) atomicOr(err, kGuardCellBounds);
    }
    if (own_cnt) {
        __syncthreads();
        block_counts_to_bounds<256>(nc.x * nc.y * nc.z, own_cnt, own_start, nullptr, true, sh);
    }
}

// also re-zeroes the per-cell counts (consumed by k_cell_hist's bounds) for the next build, so no
// separate zeroing launch precedes k_cell_hist
__global__ void __launch_bounds__(256) k_cell_scatter(int n, const int* __restrict__ flag, const int* __restrict__ key,
                                                      const int* __restrict__ rank, const int* __restrict__ cstart,
                                                      int* __restrict__ tmp, int ncell, int* __restrict__ cnt,
                                                      int* __restrict__ own_cnt, int* __restrict__ err) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (!*flag) return;
    for (int c = i; c < ncell; c += gridDim.x * blockDim.x) {
        cnt[c] = 0;
        if (own_cnt) own_cnt[c] = 0;
    }
    if (i >= n) return;
    const int k = key[i], s = (unsigned)k < (unsigned)ncell ? cstart[k] + rank[i] : -1;
    if ((unsigned)s >= (unsigned)n) { atomicOr(err, kGuardCellBounds); return; }   // guard
    tmp[s] = i;
}

// one 256-thread block per cell: final position of each member = cell start + number of members
// before it in the cell order (members staged in LDS and read by broadcast, each member's count on
// one thread: ~0.7 members per thread at C3 instead of ~3 per lane with one wave per cell --
// round 4's form took 25 us per rebuild at C3, a quarter of the waves on the chip); multi-rank: an
// owned member's list row = the cell's first row + number of owned members before it.
// Cell order (zcol = S > 0): the cell is cut into S x S columns along its a and b lattice
// directions, members sorted by (column, fractional c coordinate, atom index), columns and the
// direction along c in serpentine order -- so that runs of
// 4 consecutive slots (the clusters of the cluster-pair list, cf_kernels_cluster.hip) are
// spatially compact whatever the atom order of the system; zcol = 0: by atom index (the order of
// a stable sort).  Both are total orders computed from the positions alone: deterministic.
constexpr int kOrderLds = 1024;

__global__ void __launch_bounds__(256) k_cell_order(int ncell, const int* __restrict__ flag,
                                                    const int* __restrict__ cstart, const int* __restrict__ cend,
                                                    const int* __restrict__ tmp, int* __restrict__ out, int lo, int hi,
                                                    const int* __restrict__ own_start, int* __restrict__ own_s,
                                                    const double* __restrict__ pos, double3 L, double3 T, int3 nc,
                                                    int zcol, int n, int* __restrict__ err) {
    // one 64-bit key per member: (column << 58 | quantized c coordinate << 26 | atom index), or the
    // atom index alone -- the rank is then one unsigned compare per member pair
    __shared__ unsigned long long memk[kOrderLds];
    const int tid = threadIdx.x;
    const int c = blockIdx.x;
    if (c >= ncell || !*flag) return;   // block-uniform
    const int b = cstart[c], m = cend[c] - b;
    if (b < 0 || m < 0 || b + m > n) {   // guard (k_cell_hist's bounds hold by construction)
        if (tid == 0) atomicOr(err, kGuardCellBounds);
        return;
    }
    const int* src = tmp + b;
    if (m > kOrderLds) {   // rare (an over-full cell): atom order, read from global memory
        for (int e = tid; e < m; e += 256) {
            const int v = src[e];
            int r = 0, ro = 0;
            for (int j = 0; j < m; j++) {
                const int u = src[j];
                r += u < v;
                if (own_s) ro += u < v && u >= lo && u < hi;
            }
            out[b + r] = v;
            if (own_s && v >= lo && v < hi) own_s[own_start[c] + ro] = b + r;
        }
        return;
    }
    const int cc[3] = {c / (nc.y * nc.z), (c / nc.z) % nc.y, c % nc.z};
    for (int e = tid; e < m; e += 256) {
        const int v = src[e];
        unsigned long long key = (unsigned long long)v;
        if (zcol > 0) {
            // the member's position inside its cell in fractional cell units (as k_cell_hist bins it)
            const double3 x = ld3(pos, v);
            const double3 f = fractional(wrap_by(x, floor3(fractional(x, L, T)), L, T), L, T);
            const double la = fmin(fmax(f.x * nc.x - cc[0], 0.0), 0.999999);
            const double lb = fmin(fmax(f.y * nc.y - cc[1], 0.0), 0.999999);
            const double lc = fmin(fmax(f.z * nc.z - cc[2], 0.0), 0.999999);
            // columns in serpentine order, c ascending in even and descending in odd columns:
            // consecutive slots stay neighbours across a column change (a cluster that straddles
            // two columns is still compact)
            const int ca = (int)(la * zcol), cb0 = (int)(lb * zcol);
            const int col = ca * zcol + ((ca & 1) ? zcol - 1 - cb0 : cb0);
            const unsigned zq = (unsigned)(((col & 1) ? 0.999999 - lc : lc) * 4294967296.0);
            key |= ((unsigned long long)col << 58) | ((unsigned long long)zq << 26);
        }
        memk[e] = key;
    }
    __syncthreads();
    const unsigned long long kIdx = zcol > 0 ? (1ull << 26) - 1 : ~0ull;   // (zcol > 0: n < 2^21, half lists)
    for (int e = tid; e < m; e += 256) {
        const unsigned long long kv = memk[e];
        const int v = (int)(kv & kIdx);
        int r = 0, ro = 0;
        int j = 0;
        for (; j + 2 <= m; j += 2) {   // two keys per 16-B LDS read (broadcast: every lane reads the same j)
            const ulonglong2 u2 = *reinterpret_cast<const ulonglong2*>(&memk[j]);
            r += (u2.x < kv) + (u2.y < kv);
            if (own_s) {
                const int ux = (int)(u2.x & kIdx), uy = (int)(u2.y & kIdx);
                ro += (u2.x < kv && ux >= lo && ux < hi) + (u2.y < kv && uy >= lo && uy < hi);
            }
        }
        if (j < m) {
            const unsigned long long u = memk[j];
            r += u < kv;
            if (own_s) ro += u < kv && (int)(u & kIdx) >= lo && (int)(u & kIdx) < hi;
        }
        out[b + r] = v;
        if (own_s && v >= lo && v < hi) own_s[own_start[c] + ro] = b + r;
    }
}

// rebuild (flag set): commit the new order (scratch -> live), sorted wrapped (x,y,z,q) +
// LJ, build positions.  Wrapped = moved into the unit cell by a lattice translation (for a
// reduced triclinic box a per-axis wrap by the diagonal would not be one).  No rebuild: the
// sorted order and every atom's periodic image are kept from the last build (the lattice
// translation recomputed from the build positions, so bit-identical to the commit); only
// coordinates and flux charges are refreshed.
__global__ void __launch_bounds__(256) k_cell_commit(int n, const int* __restrict__ flag,
                                                     const int* __restrict__ key, const int* __restrict__ idx_new,
                                                     const double* __restrict__ pos, const double* __restrict__ q,
                                                     const double2* __restrict__ lj, double3 L, double3 T,
                                                     int* __restrict__ key_s, int* __restrict__ idx_s,
                                                     double4* __restrict__ pos4s, double2* __restrict__ ljs,
                                                     const int* __restrict__ atype, int* __restrict__ typ_s,
                                                     double* __restrict__ pos_ref, long long* __restrict__ n_builds,
                                                     float4* __restrict__ pos4f, int* __restrict__ slot_of, int3 nc,
                                                     int* __restrict__ err) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    double4 p4;
    int i, c;
    const bool rebuild = *flag != 0;
    // guard: a kept list needs the build positions; without a skin (pos_ref null) every evaluation
    // sets the rebuild flag first (launch_force_rebuild), so a clear flag here is a broken ordering
    if (!rebuild && !pos_ref) { if (s == 0) atomicOr(err, kGuardRebuildFlag); return; }
    if (rebuild) {
        i = idx_new[s];
        if ((unsigned)i >= (unsigned)n) { atomicOr(err, kGuardCellBounds); return; }   // guard
        c = key[i];
        key_s[s] = key[i];
        idx_s[s] = i;
        double3 x = ld3(pos, i);
        const double3 w = wrap_by(x, floor3(fractional(x, L, T)), L, T);
        p4 = make_double4(w.x, w.y, w.z, q[i]);
        ljs[s] = lj[i];
        if (typ_s) typ_s[s] = atype[i];
        if (pos_ref) { pos_ref[3 * i] = x.x; pos_ref[3 * i + 1] = x.y; pos_ref[3 * i + 2] = x.z; }
        if (slot_of) slot_of[i] = s;
        if (s == 0) *n_builds += 1;
    } else {
        i = idx_s[s];
        if ((unsigned)i >= (unsigned)n) { atomicOr(err, kGuardCellBounds); return; }   // guard
        c = pos4f ? key_s[s] : 0;
        double3 x = ld3(pos, i), r = ld3(pos_ref, i);
        const double3 w = wrap_by(x, floor3(fractional(r, L, T)), L, T);
        p4 = make_double4(w.x, w.y, w.z, q[i]);
    }
    pos4s[s] = p4;
    // cluster-pair path (cf_kernels_cluster.hip): fp32 position relative to the corner of the atom's
    // (build-time) cell -- a few nm at most, so fp32 keeps ~1e-7 nm whatever the box size -- and the
    // LJ type in w
    if (pos4f) {
        const double3 o = lattice(L, T, (double)(c / (nc.y * nc.z)) / nc.x, (double)((c / nc.z) % nc.y) / nc.y,
                                  (double)(c % nc.z) / nc.z);
        pos4f[s] = make_float4((float)(p4.x - o.x), (float)(p4.y - o.y), (float)(p4.z - o.z),
                               __int_as_float(typ_s ? atype[i] : 0));
    }
}

// ---------------------------------------------------------------------------------
// 4. direct space + exclusion correction (full neighbour list: every pair is evaluated
//    from both sides, so every per-atom sum is a gather and no atomics are needed).
//    Real-space pair RCK:562-593, exclusion erf correction RCK:596-622.
//
//    4a k_nlist: one lane per owned atom (cell-sorted order) scans the 27 neighbour cells
//       and appends every non-excluded partner with r^2 <= rc^2 (the reference's voxel-hash
//       list, RCK:559) to a transposed list nl[k*N + s] = t | shift<<26.  Only ~12% of the
//       candidates pass the cutoff, so the expensive erfc/exp math is kept out of this
//       divergent loop.
//    4b k_pairs: lanes per owned atom walk its list with every lane busy and store the raw
//       pair sums; k_excl applies the exclusion correction and the self term.
// ---------------------------------------------------------------------------------
// List layout: sub-list seg of row c holds its entries in chunks of kChunk = 4 consecutive
// entries (16 B), chunk q of every row contiguous in row order:
//   nl[((seg * nb_cap/4 + q) * nlr + c) * 4 + (k & 3)],  q = k / 4.
// The builder's lane c then fills whole 16-B granules (and, with its 7 neighbours, whole
// 128-B lines) instead of scattering single 4-B entries over lines shared with 63 other rows
// at different fill levels (which evicted partly written lines: ~4x write amplification);
// the pair walk loads a chunk of 4 entries per lane with one 16-B load, 16 rows of a wave
// reading 256 contiguous bytes per sub-list.
constexpr int kChunk = 4;
typedef int v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ size_t nl_index(const DirectArgs& a, int seg, int k, int c) {
    return ((size_t)(seg * (a.nb_cap / kChunk) + (k >> 2)) * a.nlr + c) * kChunk + (k & 3);
}

__device__ __forceinline__ bool in_excl(int j, const int* reg, int cnt, const int* ex_list, int ex0) {
    int m = cnt < kMaxRegExcl ? cnt : kMaxRegExcl;
#pragma unroll
    for (int k = 0; k < kMaxRegExcl; k++)
        if (k < m && reg[k] == j) return true;
    for (int k = kMaxRegExcl; k < cnt; k++)
        if (ex_list[ex0 + k] == j) return true;
    return false;
}

__device__ __forceinline__ double3 shift_of(int code, double3 L) {
    // code = kx*9 + ky*3 + kz in [0, 27) -> image offsets (k - 1) * L, by multiply-shift division
    const unsigned c = (unsigned)code;
    const unsigned kx = (c * 57u) >> 9, r = c - 9u * kx;
    const unsigned ky = (r * 11u) >> 5, kz = r - 3u * ky;
    return make_double3(((int)kx - 1) * L.x, ((int)ky - 1) * L.y, ((int)kz - 1) * L.z);
}

// Visit the 27 neighbour cells of sorted atom s; fn(t, code, dx, dy, dz, r2) for every
// candidate t != s within the cutoff (exclusions are left to the caller).
template <class F>
__device__ __forceinline__ void scan_cells(const DirectArgs& a, int s, double4 pi, double r2max, F&& fn,
                                           int part = 0, int nparts = 1) {
    if (!a.brute) {
        int ord = 0;
        int key = a.key_sorted[s];
        int cz = key % a.nc.z, cy = (key / a.nc.z) % a.nc.y, cx = key / (a.nc.y * a.nc.z);
        for (int ox = -1; ox <= 1; ox++) {
            int x = cx + ox; int kx;
            if (x < 0) { x += a.nc.x; kx = 0; } else if (x >= a.nc.x) { x -= a.nc.x; kx = 2; } else kx = 1;
            for (int oy = -1; oy <= 1; oy++) {
                int y = cy + oy; int ky;
                if (y < 0) { y += a.nc.y; ky = 0; } else if (y >= a.nc.y) { y -= a.nc.y; ky = 2; } else ky = 1;
                for (int oz = -1; oz <= 1; oz++) {
                    int z = cz + oz; int kz;
                    if (z < 0) { z += a.nc.z; kz = 0; } else if (z >= a.nc.z) { z -= a.nc.z; kz = 2; } else kz = 1;
                    int code = kx * 9 + ky * 3 + kz;
                    int c = (x * a.nc.y + y) * a.nc.z + z;
                    if (ord++ % nparts != part) continue;
                    // the image of the wrapped neighbour cell adjacent to this one (a lattice translate)
                    const double3 sh = lattice(a.L, a.T, kx - 1, ky - 1, kz - 1);
                    const int t1 = min(a.cend[c], a.n);   // (bounds past N are a guard case: k_cell_hist)
                    for (int t = max(a.cstart[c], 0); t < t1; t++) {
                        double4 pj = a.pos4s[t];
                        double dx = pi.x - (pj.x + sh.x), dy = pi.y - (pj.y + sh.y), dz = pi.z - (pj.z + sh.z);
                        double r2 = dx * dx + dy * dy + dz * dz;
                        if (r2 > r2max || t == s) continue;
                        fn(t, code, dx, dy, dz, r2);
                    }
                }
            }
        }
    } else {
        for (int t = part; t < a.n; t += nparts) {
            if (t == s) continue;
            double4 pj = a.pos4s[t];
            double3 d = delta_r(make_double3(pj.x, pj.y, pj.z), make_double3(pi.x, pi.y, pi.z), a.L, 1, a.T);
            double r2 = d.x * d.x + d.y * d.y + d.z * d.z;
            if (r2 > r2max) continue;
            fn(t, kBruteShift, d.x, d.y, d.z, r2);
        }
    }
}

__global__ void __launch_bounds__(256) k_nlist(DirectArgs a) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.nlr || !*a.flag) return;
    int s = own_slot(a, c);
    int i = a.atom_sorted[s];
    const double4 pi = a.pos4s[s];
    const int ex0 = a.ex_start[i], exc = a.ex_start[i + 1] - ex0;
    int reg[kMaxRegExcl];
#pragma unroll
    for (int k = 0; k < kMaxRegExcl; k++) reg[k] = k < exc ? a.ex_list[ex0 + k] : -1;
    for (int seg = 0; seg < kSeg; seg++) {
        int cnt = 0;
        scan_cells(a, s, pi, a.rl2, [&](int t, int code, double, double, double, double) {
            if (exc && in_excl(a.atom_sorted[t], reg, exc, a.ex_list, ex0)) return;
            if (cnt < a.nb_cap) a.nl[nl_index(a, seg, cnt, c)] = t | ((a.typ_s ? a.typ_s[t] : code) << kShiftBits);
            cnt++;
        }, seg, kSeg);
        a.nl_cnt[(size_t)seg * a.nlr + c] = cnt;
    }
}

// Wave-cooperative list build (the fast path): one 64-lane workgroup owns 64 consecutive
// cell-sorted atoms.  The union of their 27-cell neighbourhoods is a small box of cells in
// unwrapped cell coordinates; candidates of each cell are loaded coalesced (one per lane),
// shifted to the image adjacent to the block, staged in LDS and tested by every lane with
// broadcast LDS reads.  Falls back to the per-lane scan when the box would wrap onto itself.
// Wave-cooperative list build (the fast path): one 64-lane workgroup owns 64 consecutive
// cell-sorted atoms.  The union of their 27-cell neighbourhoods is a small box of cells in
// unwrapped cell coordinates.  Each cell's candidates (up to 256 per step) are loaded
// coalesced, moved to the block frame (fp64 shift, then fp32), staged in LDS and tested by
// every lane with broadcast reads; the next cell is prefetched into registers meanwhile.
// The fp32 test uses a margin; k_pairs applies the exact fp64 r <= rc test.  Falls back to
// the per-lane scan when the box would wrap onto itself.
constexpr int kWaveNL = 64;
constexpr int kStageU = 2;                 // candidates per lane staged per cell pass
constexpr int kStage = kStageU * kWaveNL;

__global__ void __launch_bounds__(kWaveNL * kSeg) k_nlist_wave(DirectArgs a) {
    // staged candidates, SoA so that one ds_read_b128 gives 4 candidates' x (two packed-fp32
    // operands): x, y, z in the block frame, (half lists) the x key; atom index | LJ type << 26
    __shared__ __attribute__((aligned(16))) float cand_all[kSeg][4][kStage + 16];
    __shared__ int cand_j_all[kSeg][kStage + 16];
    const int lane = threadIdx.x & 63;
    const int seg = threadIdx.x >> 6;   // this wave's share of the cell box and its sub-list
    float* cx = cand_all[seg][0];
    float* cy = cand_all[seg][1];
    float* cz = cand_all[seg][2];
    float* cxk = cand_all[seg][3];
    int* cand_j = cand_j_all[seg];
    if (!*a.flag) return;  // list still valid (skin): nothing to build
    const int base = xcd_block() * kWaveNL;
    const int c = base + lane;  // list row (owned atom, cell-sorted order)
    const bool active = c < a.nlr;
    const int s = own_slot(a, active ? c : a.nlr - 1);
    const int i = a.atom_sorted[s];
    const double4 pi = a.pos4s[s];
    const int key = a.key_sorted[s];
    const int cl[3] = {key / (a.nc.y * a.nc.z), (key / a.nc.z) % a.nc.y, key % a.nc.z};
    const int key0 = a.key_sorted[__shfl(s, 0)];
    const int c0[3] = {key0 / (a.nc.y * a.nc.z), (key0 / a.nc.z) % a.nc.y, key0 % a.nc.z};
    const int ncs[3] = {a.nc.x, a.nc.y, a.nc.z};
    int lo3[3], hi3[3], lsh[3], ucell[3];
    bool fits = true;
#pragma unroll
    for (int d = 0; d < 3; d++) {
        int dd = cl[d] - c0[d];
        if (dd > ncs[d] / 2) dd -= ncs[d];
        if (dd < -(ncs[d] / 2)) dd += ncs[d];
        int u = c0[d] + dd;  // unwrapped cell coordinate of this lane in the block frame
        ucell[d] = u;
        lsh[d] = u < 0 ? -1 : (u >= ncs[d] ? 1 : 0);  // image of this lane's (wrapped) position
        int mn = u, mx = u;
        for (int off = 32; off > 0; off >>= 1) {
            mn = min(mn, __shfl_xor(mn, off));
            mx = max(mx, __shfl_xor(mx, off));
        }
        lo3[d] = mn - 1; hi3[d] = mx + 1;
        if (hi3[d] - lo3[d] + 1 > ncs[d]) fits = false;
        // half lists: partners only at x offset 0 or +1, so the box starts at the lowest row cell
        if (d == 0 && a.half) lo3[d] = mn;
    }
    const int ex0 = a.ex_start[i], exc = a.ex_start[i + 1] - ex0;
    int reg[kMaxRegExcl];
#pragma unroll
    for (int k = 0; k < kMaxRegExcl; k++) reg[k] = k < exc ? a.ex_list[ex0 + k] : -1;
    // exclusion lists are sorted: a candidate outside [ex_min, ex_max] needs no lookup
    const int ex_min = exc ? a.ex_list[ex0] : 1, ex_max = exc ? a.ex_list[ex0 + exc - 1] : 0;
    int cnt = 0;
    int* const nl_row = a.nl + ((size_t)seg * (a.nb_cap / kChunk) * a.nlr + c) * kChunk;   // = nl_index(a, seg, 0, c)
    const unsigned nl_qstride = (unsigned)a.nlr * kChunk;   // a row's entries lie within nb_cap * nlr < 2^31 ints of nl_row
    // store list entry `entry` unless partner j is excluded (one branch: the store)
    auto put_entry = [&](int entry, int j) {
        const bool keep = !(j >= ex_min && j <= ex_max && in_excl(j, reg, exc, a.ex_list, ex0));
        if (keep && cnt < a.nb_cap) nl_row[(unsigned)(cnt >> 2) * nl_qstride + (unsigned)(cnt & 3)] = entry;
        cnt += keep;
    };
    // high bits of a list entry: the partner's LJ type when types are used, else the image code
    auto emit = [&](int t, int j, int hb) { put_entry(t | (hb << kShiftBits), j); };
    if (!fits) {  // wave-uniform (and block-uniform: every wave sees the same 64 atoms)
        if (a.half) {
            // half lists need the block frame: these rows get no entries and an overflowed
            // count, so k_pairs_half raises half_flag on EVERY evaluation that uses this list
            // (also the later ones that keep it under a skin, when this kernel does not run)
            // and k_excl rescans with the fp64 cell scan
            if (active) a.nl_cnt[(size_t)seg * a.nlr + c] = a.nb_cap + 1;
            return;
        }
        if (active)
            scan_cells(a, s, pi, a.rl2, [&](int t, int code, double, double, double, double) {
                emit(t, a.atom_sorted[t], a.typ_s ? a.typ_s[t] : code);
            }, seg, kSeg);
        if (active) a.nl_cnt[(size_t)seg * a.nlr + c] = cnt;
        return;
    }

    // block frame: every lane's position moved to the image of its unwrapped cell; origin =
    // lane 0 (lsh = 0 there), so frame coordinates stay within a few cells of 0
    const double3 lu = lattice(a.L, a.T, lsh[0], lsh[1], lsh[2]);
    const double3 pu = make_double3(pi.x + lu.x, pi.y + lu.y, pi.z + lu.z);
    const double3 org = make_double3(__shfl(pu.x, 0), __shfl(pu.y, 0), __shfl(pu.z, 0));
    const float3 pf = make_float3((float)(pu.x - org.x), (float)(pu.y - org.y), (float)(pu.z - org.z));
    const float rc2f = (float)(a.rl2 * (1.0 + 1e-5)) + 1e-6f;

    const int by = hi3[1] - lo3[1] + 1, bz = hi3[2] - lo3[2] + 1;
    const int ncell = (hi3[0] - lo3[0] + 1) * by * bz;
    // half mode: window cell index of box cell q for this lane (x offset 0: 0..8, +1: 9..17;
    // negative: x offset -1 or not adjacent -- no entries)
    auto half_k = [&](int q) {
        const int w[3] = {lo3[0] + q / (by * bz), lo3[1] + (q / bz) % by, lo3[2] + q % bz};
        const int dx = w[0] - ucell[0], dy = w[1] - ucell[1], dz = w[2] - ucell[2];
        if (dx < 0 || dx > 1 || dy < -1 || dy > 1 || dz < -1 || dz > 1) return -1;
        return dx * 9 + (dy + 1) * 3 + (dz + 1);
    };
    const float xki = (float)pi.x;   // this row's x key (wrapped coordinate, as stored)
    // cell q of the box -> storage index, image code, frame offset (shift - origin)
    auto cell_of = [&](int q, int& code, double3& off) {
        int w[3] = {lo3[0] + q / (by * bz), lo3[1] + (q / bz) % by, lo3[2] + q % bz}, k[3];
#pragma unroll
        for (int d = 0; d < 3; d++) {
            k[d] = w[d] < 0 ? 0 : (w[d] >= ncs[d] ? 2 : 1);
            w[d] -= (k[d] - 1) * ncs[d];
        }
        code = (k[0] - lsh[0]) * 9 + (k[1] - lsh[1]) * 3 + (k[2] - lsh[2]);  // relative to this lane's image
        const double3 sh = lattice(a.L, a.T, k[0] - 1, k[1] - 1, k[2] - 1);
        off = make_double3(sh.x - org.x, sh.y - org.y, sh.z - org.z);
        return (w[0] * a.nc.y + w[1]) * a.nc.z + w[2];
    };
    // This wave's candidates of a cell are the atoms whose index in the cell, in groups of 4
    // (one 128-B line of pos4s), is this wave's group mod 4: candidate u of cell [cb, ce) is
    // slot cb + 16 (u / 4) + 4 seg + u % 4.  Interleaved because cells are sorted by atom
    // index, which follows space: contiguous quarters would give the sub-lists of a half list
    // very different lengths (lane efficiency 0.66 -> 0.83 at C3; 0.85 -> 0.88 full lists).
    static_assert(kSeg == 4, "the interleave below uses shifts");
    auto slot_of = [&](int cb, int u) { return cb + ((u >> 2) << 4) + (seg << 2) + (u & 3); };
    auto count_of = [&](int cb, int ce) {   // this wave's candidates in the cell
        const int n = ce - cb;
        return ((n >> 4) << 2) + min(4, max(0, (n & 15) - (seg << 2)));
    };
    double4 rp[kStageU];
    int rj[kStageU], rt[kStageU];
    auto fetch = [&](int cb, int nu) {   // candidates u = 0 .. kStage-1 of the cell
#pragma unroll
        for (int v = 0; v < kStageU; v++) {
            const int u = v * kWaveNL + lane;
            if (u < nu) {
                const int t = slot_of(cb, u);
                rp[v] = a.pos4s[t]; rj[v] = a.atom_sorted[t]; rt[v] = a.typ_s ? a.typ_s[t] : 0;
            }
        }
    };
    // staged candidate: fp32 block-frame position, x key, atom index | LJ type bits
    auto put = [&](int u, const double4& pj, int j, int tp, double3 off) {
        cx[u] = (float)(pj.x + off.x);
        cy[u] = (float)(pj.y + off.y);
        cz[u] = (float)(pj.z + off.z);
        cxk[u] = (float)pj.x;
        cand_j[u] = j | (tp << kShiftBits);
    };
    auto stage = [&](int nu, double3 off) {
#pragma unroll
        for (int v = 0; v < kStageU; v++) {
            int u = v * kWaveNL + lane;
            if (u < nu) put(u, rp[v], rj[v], rt[v], off);
        }
    };
    // 16 candidates per chunk, tested two at a time in packed fp32 (v_pk_add/mul/fma_f32: half
    // the VALU instructions of scalar fp32), then the lane's hits of the chunk are emitted
    // (a longer chunk amortizes the divergent emit loop: its trip count is the maximum hit
    // count over the wave's lanes).  Staged candidate u is candidate u0 + u of cell cb.
    // (Measured against emitting each candidate at once by the lanes it hits, exec-masked:
    // 54.8 vs 67.7 us per step at C3, profiles/r03i_*; the same list either way.)
    typedef float v2f __attribute__((ext_vector_type(2)));
    typedef float v4f __attribute__((ext_vector_type(4)));
    auto test = [&](int cb, int u0, int m, int code, int hk) {
        if (!active) return;
        if (a.half && hk < 0) return;   // x offset -1: those pairs belong to the partner's row
        const v2f px = {pf.x, pf.x}, py = {pf.y, pf.y}, pz = {pf.z, pf.z};
        for (int c0 = 0; c0 < m; c0 += 16) {
            unsigned bits = 0;
#pragma unroll
            for (int v = 0; v < 16; v += 4) {
                const v4f X = *reinterpret_cast<const v4f*>(cx + c0 + v);
                const v4f Y = *reinterpret_cast<const v4f*>(cy + c0 + v);
                const v4f Z = *reinterpret_cast<const v4f*>(cz + c0 + v);
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const v2f dx = px - (h ? X.zw : X.xy), dy = py - (h ? Y.zw : Y.xy), dz = pz - (h ? Z.zw : Z.xy);
                    const v2f r2 = dx * dx + dy * dy + dz * dz;
                    bits |= (r2.x <= rc2f ? 1u : 0u) << (v + 2 * h);
                    bits |= (r2.y <= rc2f ? 1u : 0u) << (v + 2 * h + 1);
                }
            }
            if (m - c0 < 16) bits &= (1u << (m - c0)) - 1u;
            if (a.half && hk < 9 && bits) {
                unsigned ahead = 0, tie = 0;
#pragma unroll
                for (int v = 0; v < 16; v += 4) {
                    const v4f K = *reinterpret_cast<const v4f*>(cxk + c0 + v);
                    ahead |= ((K.x > xki ? 1u : 0u) | (K.y > xki ? 2u : 0u) | (K.z > xki ? 4u : 0u) |
                              (K.w > xki ? 8u : 0u)) << v;
                    tie |= ((K.x == xki ? 1u : 0u) | (K.y == xki ? 2u : 0u) | (K.z == xki ? 4u : 0u) |
                            (K.w == xki ? 8u : 0u)) << v;
                }
                tie &= bits;
                while (tie) {
                    const int v = __builtin_ctz(tie);
                    tie &= tie - 1;
                    if (slot_of(cb, u0 + c0 + v) > s) ahead |= 1u << v;
                }
                bits &= ahead;
            }
            if (!a.half) {
                const int ds = s - cb;
                if (ds >= 0 && ((ds >> 2) & 3) == seg) {
                    const int us = (((ds >> 4) << 2) | (ds & 3)) - (u0 + c0);
                    if (us >= 0 && us < 16) bits &= ~(1u << us);
                }
                // the hits of the chunk, one per trip; the next hit's staged index is read before
                // this one is emitted (a trip's LDS read sat on its dependency chain: with one wave
                // per SIMD at W = 8 its latency was exposed on every trip, r06ap; rebuilds 155-180 ->
                // 156-169 us, r06aq)
                if (bits) {
                    int v = __builtin_ctz(bits);
                    bits &= bits - 1;
                    int cj = cand_j[c0 + v];
                    for (;;) {
                        const int vn = bits ? __builtin_ctz(bits) : v;
                        const int cjn = cand_j[c0 + vn];
                        emit(slot_of(cb, u0 + c0 + v), cj & kJMask, a.typ_s ? (int)((unsigned)cj >> kShiftBits) : code);
                        if (!bits) break;
                        bits &= bits - 1;
                        v = vn;
                        cj = cjn;
                    }
                }
            } else {
                if (bits) {
                    int v = __builtin_ctz(bits);
                    bits &= bits - 1;
                    int cj = cand_j[c0 + v];
                    for (;;) {
                        const int vn = bits ? __builtin_ctz(bits) : v;
                        const int cjn = cand_j[c0 + vn];
                        put_entry(slot_of(cb, u0 + c0 + v) | (hk << kHalfSlotBits) | (cj & ~kJMask), cj & kJMask);
                        if (!bits) break;
                        bits &= bits - 1;
                        v = vn;
                        cj = cjn;
                    }
                }
            }
        }
    };

    // every wave visits every cell of the box (its interleaved quarter of the atoms).
    // (LDS regions are per wave: wave barriers only.)
    int code_n; double3 off_n;
    int cc = cell_of(0, code_n, off_n);
    int cb_n = a.cstart[cc], nu_n = count_of(cb_n, a.cend[cc]);
    fetch(cb_n, nu_n);
    for (int q = 0; q < ncell; q++) {
        const int code = code_n, cb = cb_n, nu = nu_n;
        const double3 off = off_n;
        const int hk = a.half ? half_k(q) : 0;
        __builtin_amdgcn_wave_barrier();
        stage(nu, off);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (q + 1 < ncell) {  // prefetch the next cell while this one is tested
            cc = cell_of(q + 1, code_n, off_n);
            cb_n = a.cstart[cc];
            nu_n = count_of(cb_n, a.cend[cc]);
            fetch(cb_n, nu_n);
        }
        test(cb, 0, min(nu, kStage), code, hk);
        // rare: more than kStage candidates per wave in a cell (synchronous remainder)
        for (int u0 = kStage; u0 < nu; u0 += kStage) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int v = 0; v < kStageU; v++) {
                const int u = v * kWaveNL + lane;
                if (u0 + u < nu) {
                    const int t = slot_of(cb, u0 + u);
                    put(u, a.pos4s[t], a.atom_sorted[t], a.typ_s ? a.typ_s[t] : 0, off);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            test(cb, u0, min(nu - u0, kStage), code, hk);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    if (active) a.nl_cnt[(size_t)seg * a.nlr + c] = cnt;
}


// real-space Ewald + LJ pair (RCK:567-592), d = pos_i - pos_j (minimum image); tab = LDS
// copy of the erfcx table (the cutoff test r <= rc guarantees alpha r lies inside it)
__device__ __forceinline__ void pair_term(PairAcc& acc, const DirectArgs& a, const double* __restrict__ tab,
                                          double4 pi, double2 li, double4 pj, double2 lj2, double dx, double dy,
                                          double dz, double r2) {
    const double ke = a.ke;
    const double two_over_sqrtpi = 1.1283791670955126;
    double inv_r = rsqrt_fp64(r2);
    double r = r2 * inv_r;
    double ar = a.alpha * r;
    double e2;
    double ec = erfc_exp(ar, tab, a.erfc_scale, e2);
    const double qj = ke * pj.w * inv_r;   // potential of j at i per unit erfc; qq = q_i qj
    const double qq = pi.w * qj;
    double sig = li.x + lj2.x;
    double s2 = inv_r * sig; s2 *= s2;
    const double sig6 = s2 * s2 * s2;
    const double es6 = sig6 * li.y * lj2.y;
    if (a.include_forces) {
        const double dEdR = fma(qq, ec + ar * e2 * two_over_sqrtpi, es6 * (12 * sig6 - 6)) * (inv_r * inv_r);
        acc.fx += dEdR * dx; acc.fy += dEdR * dy; acc.fz += dEdR * dz;
        acc.dq += qj * ec;
    }
    acc.e += qq * ec + es6 * (sig6 - 1);   // the pair's full energy; halved once in store_pairs
}

// stage the erfcx table in LDS (all threads of the block; call before any early return)
__device__ __forceinline__ void load_erfc_tab(const DirectArgs& a, double* tab) {
    for (int e = threadIdx.x; e < kErfcMaxM * (kErfcDeg + 1); e += blockDim.x) tab[e] = a.erfc_tab[e];
    __syncthreads();
}

// pair-loop results of atom i: raw direct-space sums (dE/dq_i without the self term, forces,
// energy); k_excl then applies the exclusion correction and the self term in place.  Each
// pair's energy is shared half-and-half by its two atoms (full list): the 1/2 is applied here
// once per atom instead of once per pair (a power of two: the same bits either way).
__device__ __forceinline__ void store_pairs(const PairAcc& acc, const DirectArgs& a, int i) {
    a.e_atom[3 * i + 1] = 0.5 * acc.e;
    if (a.include_forces) {  // reciprocal partials are added by k_recip_add after the k-space pass
        a.dedq[i] = acc.dq;
        a.f_part[3 * i] = acc.fx;
        a.f_part[3 * i + 1] = acc.fy;
        a.f_part[3 * i + 2] = acc.fz;
    }
}

// exclusion correction of owned atom i (RCK:596-622: every excluded pair, minimum image,
// no cutoff, no LJ) on top of the stored pair sums, then dE/dq += the self term.  Run by
// k_excl after the pair kernels, so that the pair loop is not sized for the erf code
// (VGPRs -> occupancy).  The
// operation order per atom is that of one fused loop: pair sums, then exclusions in list
// order, then dE/dq_self + sum.
// (add_f, add_dq: the half list's partner-side sums of the atom, added to the stored pair sums)
__device__ __forceinline__ void excl_atom(const DirectArgs& a, int i, double3 add_f = make_double3(0.0, 0.0, 0.0),
                                          double add_dq = 0.0) {
    const double ke = a.ke;
    const double two_over_sqrtpi = 1.1283791670955126;
    const int ex0 = a.ex_start[i], exc = a.ex_start[i + 1] - ex0;
    double fx = 0, fy = 0, fz = 0, dq = 0, ex_e = 0;
    if (a.include_forces) {
        fx = a.f_part[3 * i] + add_f.x; fy = a.f_part[3 * i + 1] + add_f.y; fz = a.f_part[3 * i + 2] + add_f.z;
        dq = a.dedq[i] + add_dq;
    }
    if (exc) {
        double3 xi = ld3(a.pos, i);
        double qi = a.q[i];
        for (int k = 0; k < exc; k++) {
            int j = a.ex_list[ex0 + k];
            double3 d = delta_r(ld3(a.pos, j), xi, a.L, 1, a.T);
            double r = sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
            double inv_r = 1.0 / r, ar = a.alpha * r;
            double ef = erf(ar);
            double qj = a.q[j];
            if (a.include_forces) {
                double g = ke * qi * qj * inv_r * inv_r * inv_r * (ef - ar * exp(-ar * ar) * two_over_sqrtpi);
                fx -= g * d.x; fy -= g * d.y; fz -= g * d.z;
                dq -= ke * qj * inv_r * ef;
            }
            ex_e -= 0.5 * ke * qi * qj * inv_r * ef;
        }
    }
    a.e_atom[3 * i + 2] = ex_e;
    if (a.include_forces) {
        a.dedq[i] = a.dedq_self[i] + dq;
        a.f_part[3 * i] = fx;
        a.f_part[3 * i + 1] = fy;
        a.f_part[3 * i + 2] = fz;
    }
}

// dE/dq and non-chain forces += reciprocal partials (fixed part order: deterministic)
__global__ void __launch_bounds__(256) k_recip_add(int lo, int nown, int nparts, const double* __restrict__ t_part,
                                                   double* __restrict__ dedq, double* __restrict__ f_part) {
    int io = blockIdx.x * blockDim.x + threadIdx.x;
    if (io >= nown) return;
    double dr = 0, rx = 0, ry = 0, rz = 0;
    for (int p = 0; p < nparts; p++) {
        const double* tp = t_part + ((size_t)p * nown + io) * 4;
        dr += tp[0]; rx += tp[1]; ry += tp[2]; rz += tp[3];
    }
    int i = lo + io;
    dedq[i] += dr;
    f_part[3 * i] += rx;
    f_part[3 * i + 1] += ry;
    f_part[3 * i + 2] += rz;
}

// Walk the entries of one sub-list that belong to this lane (chunks q = part, part + step,
// ...) as a software pipeline: the gather of the next entry is in flight while the current
// one is evaluated, list chunks are loaded two chunks ahead (non-temporal: streamed once,
// L2 is kept for the coordinates), unrolled over two chunk registers (A, B) so that no
// freshly loaded value is ever copied (a register move of a pending load makes the compiler
// drain vmcnt).  Entries at or past cnt are gathered from slot 0 (always valid memory: the
// chunk may hold stale values there) and not evaluated.
template <class G, class E>
__device__ __forceinline__ void walk_list(const v4i* __restrict__ nl4, size_t stride, int cnt, int part, int step,
                                          G&& gather, E&& eval) {
    if (kChunk * part >= cnt) return;
    const int qlast = (cnt - 1) / kChunk;
    auto chunk = [&](int q) { return __builtin_nontemporal_load(nl4 + (size_t)min(q, qlast) * stride); };
    v4i A = chunk(part), B = chunk(part + step);
    auto c0 = gather(A.x, true);
    for (int q = part; kChunk * q < cnt; q += 2 * step) {
        const int k = kChunk * q;
        auto c1 = gather(A.y, k + 1 < cnt);
        eval(c0);
        c0 = gather(A.z, k + 2 < cnt);
        if (k + 1 < cnt) eval(c1);
        c1 = gather(A.w, k + 3 < cnt);
        A = chunk(q + 2 * step);
        if (k + 2 < cnt) eval(c0);
        const int kb = kChunk * (q + step);
        c0 = gather(B.x, kb < cnt);
        if (k + 3 < cnt) eval(c1);
        if (kb >= cnt) break;
        c1 = gather(B.y, kb + 1 < cnt);
        eval(c0);
        c0 = gather(B.z, kb + 2 < cnt);
        if (kb + 1 < cnt) eval(c1);
        c1 = gather(B.w, kb + 3 < cnt);
        B = chunk(q + 3 * step);
        if (kb + 2 < cnt) eval(c0);
        c0 = gather(A.x, kb + kChunk * step < cnt);
        if (kb + 3 < cnt) eval(c1);
    }
}

// 4b: walk the list — kSeg adjacent lanes per atom, lane g walks sub-list g; partial sums
// are combined with two xor-shuffles (fixed order: deterministic).  Atoms with an
// overflowed sub-list are left to k_excl (cell rescan).
// LPA lanes per atom (4, 8 or 16; more when few atoms are owned, so the grid still fills
// the chip): lane g walks chunks g/4, g/4 + LPA/4, ... of sub-list g%4.
// TYPES: the partner's LJ parameters come from the per-type table (LDS) indexed by the high
// bits of the list entry instead of a third gathered 16-B load per candidate.
template <int LPA, bool TYPES>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) k_pairs(DirectArgs a) {
    __shared__ double tab[kErfcMaxM * (kErfcDeg + 1)];
    __shared__ double2 ljt[kMaxLjTypes];
    if (TYPES)
        for (int e = threadIdx.x; e < a.lj_ntypes; e += blockDim.x) ljt[e] = a.lj_tab[e];
    load_erfc_tab(a, tab);
    const int gt = xcd_block() * blockDim.x + threadIdx.x;
    const int c = gt / LPA, g = gt % LPA;
    const int seg = g % kSeg, part = g / kSeg;
    bool active = c < a.nlr;
    const int cc = active ? c : a.nlr - 1;
    const int ss = own_slot(a, cc);
    const int i = a.atom_sorted[ss];
    int cnt = active ? a.nl_cnt[(size_t)seg * a.nlr + cc] : 0;
    bool over = cnt > a.nb_cap;
#pragma unroll
    for (int m = 1; m < LPA; m <<= 1) over = __shfl_xor(over, m) || over;
    if (over) active = false;
    PairAcc acc;
    bool bad_entry = false;
    if (active) {
        const double4 pi = a.pos4s[ss];
        const double2 li = a.ljs[ss];
        const v4i* nl4 = reinterpret_cast<const v4i*>(a.nl) + (size_t)seg * (a.nb_cap / kChunk) * a.nlr + cc;
        constexpr int kMask = (1 << kShiftBits) - 1;
        struct Cand { double4 p; double2 lj; };
        auto gather = [&](int e, bool ok) {
            int t = ok ? (e & kMask) : 0;
            if ((unsigned)t >= (unsigned)a.n) { bad_entry = true; t = 0; }   // guard (k_nlist writes t < n)
            Cand cd;
            cd.p = a.pos4s[t];
            cd.lj = TYPES ? ljt[(unsigned)e >> kShiftBits] : a.ljs[t];
            return cd;
        };
        // The pair vector is the minimum image d - L rint(d/L) (getDeltaRPeriodic's
        // floor(d/L + 0.5) up to exact half-box ties, which lie beyond the cutoff), so the
        // image code stored in the list is not needed.
        auto eval = [&](const Cand& cd) {
            double dx = pi.x - cd.p.x, dy = pi.y - cd.p.y, dz = pi.z - cd.p.z;
            min_image(a, dx, dy, dz);
            const double r2 = dx * dx + dy * dy + dz * dz;
            if (r2 <= a.rc2) pair_term(acc, a, tab, pi, li, cd.p, cd.lj, dx, dy, dz, r2);  // exact voxel-hash test
        };
        walk_list(nl4, a.nlr, cnt, part, LPA / kSeg, gather, eval);
    }
#pragma unroll
    for (int m = 1; m < LPA; m <<= 1) {
        acc.fx += __shfl_xor(acc.fx, m); acc.fy += __shfl_xor(acc.fy, m); acc.fz += __shfl_xor(acc.fz, m);
        acc.dq += __shfl_xor(acc.dq, m); acc.e += __shfl_xor(acc.e, m);
    }
    if (__ballot(bad_entry) && (threadIdx.x & 63) == 0) atomicOr(a.err, kGuardNeighbor);
    if (!active || g != 0) return;
    store_pairs(acc, a, i);
}

// ---------------------------------------------------------------------------------
// 4b'' half list: one 1024-thread workgroup per cell, 4 lanes per row
//     (passes of 256 rows).  Each pair is evaluated once, by the row that keeps it (the x
//     half-space rule above): the i side accumulates in fp64 registers as in k_pairs; the j
//     side (force -F_ij and dE/dq_j += k_e q_i erfc/r) is added in 64-bit fixed point to the
//     block's LDS window -- the atoms of the 18 cells at x offset 0 and +1 -- with integer LDS
//     atomics (exact: the sum does not depend on the order).  The window is then written to
//     win_out[cell] and k_excl adds, per atom, the 18 windows that contain it.  The
//     pair energy goes wholly to row i (no halving).  Any row whose list overflowed, any
//     j-side contribution too large for the fixed point, or a builder that could not encode
//     its block sets half_flag: k_excl then skips the windows and recomputes every
//     atom's pair sums with the fp64 cell rescan.
// ---------------------------------------------------------------------------------

// MIXED: the pair term in fp32 as in k_pairs_mixed (pair vector minimum-imaged in fp64, then
// rounded; fp32 forces and dE/dq per lane, fp64 energy), the partner side in the same fixed
// point (an fp32 value times 2^34 is exact in fp64)
// TRIC: reduced triclinic box (the box-vector minimum image, min_image); else the per-axis form
template <bool TYPES, bool MIXED, bool TRIC>
__global__ void __launch_bounds__(kHalfBlock) CF_LDS_UNPAIRED k_pairs_half(DirectArgs a) {
    __shared__ double tab[MIXED ? 1 : kErfcMaxM * (kErfcDeg + 1)];
    __shared__ float tabf[MIXED ? kErfcMaxMF * (kErfcDegF + 1) : 1];
    __shared__ double2 ljt[(TYPES && !MIXED) ? kMaxLjTypes : 1];
    __shared__ float2 ljtf[(TYPES && MIXED) ? kMaxLjTypes : 1];
    __shared__ int2 win[kHalfWin];                     // (first sorted slot, window offset) per window cell
    __shared__ int wdel[kHalfWin];                     // window offset - first sorted slot
    __shared__ unsigned long long accw[4][kHalfMaxWin];   // j-side fx, fy, fz, dE/dq (fixed point)
    // MIXED, orthorhombic: the translation that brings a window cell's (wrapped) atoms next to
    // this cell, so the pair vector is x_i - (x_j + t) -- three adds instead of the per-pair
    // minimum image (multiply, rint, fma per axis; round-3 review).  For a pair within rc <
    // L/2 it is the minimum image.
    constexpr bool kWrapTab = MIXED && !TRIC;
    __shared__ double3 wrt[kWrapTab ? kHalfWin : 1];
    __shared__ int wtot;
    const int cell = xcd_block();
    const int3 nc = a.nc;
    const int cz = cell % nc.z, cy = (cell / nc.z) % nc.y, cx = cell / (nc.y * nc.z);
    if (threadIdx.x < kHalfWin) {
        const int3 o = half_offset(threadIdx.x);
        const int ux = cx + o.x, uy = cy + o.y, uz = cz + o.z;
        const int wx = wrap_cell(ux, nc.x), wy = wrap_cell(uy, nc.y), wz = wrap_cell(uz, nc.z);
        const int w = (wx * nc.y + wy) * nc.z + wz;
        const int b = a.cstart[w];
        win[threadIdx.x] = make_int2(b, a.cend[w] - b);
        if constexpr (kWrapTab)
            wrt[threadIdx.x] = make_double3(ux == wx ? 0.0 : (ux > wx ? a.L.x : -a.L.x),
                                            uy == wy ? 0.0 : (uy > wy ? a.L.y : -a.L.y),
                                            uz == wz ? 0.0 : (uz > wz ? a.L.z : -a.L.z));
    }
    if constexpr (TYPES) {
        for (int e = threadIdx.x; e < a.lj_ntypes; e += kHalfBlock) {
            if constexpr (MIXED) ljtf[e] = make_float2((float)a.lj_tab[e].x, (float)a.lj_tab[e].y);
            else ljt[e] = a.lj_tab[e];
        }
    }
    if constexpr (MIXED) {
        for (int e = threadIdx.x; e < a.erfc_m_f * (kErfcDegF + 1); e += kHalfBlock) tabf[e] = a.erfc_tab_f[e];
    } else {
        for (int e = threadIdx.x; e < kErfcMaxM * (kErfcDeg + 1); e += kHalfBlock) tab[e] = a.erfc_tab[e];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int off = 0;
        for (int k = 0; k < kHalfWin; k++) {
            const int n = win[k].y;
            win[k].y = off;
            wdel[k] = off - win[k].x;
            off += n;
        }
        wtot = off;
        if (off > kHalfMaxWin) atomicOr(a.half_flag, kHalfWindowFull);
    }
    __syncthreads();
    const int nw = wtot;
    if (nw > kHalfMaxWin) return;   // block-uniform; k_excl recomputes everything
    if (threadIdx.x < kHalfWin) a.win_woff[cell * kHalfWin + threadIdx.x] = win[threadIdx.x].y;
    for (int e = threadIdx.x; e < nw; e += kHalfBlock) {
        accw[0][e] = 0; accw[1][e] = 0; accw[2][e] = 0; accw[3][e] = 0;
    }
    __syncthreads();
    const int r0 = win[kHalfOwn].x, nrows = a.cend[cell] - r0;
    const int g = threadIdx.x & 3;   // sub-list walked by this lane
    bool bad = false, bad_list = false;
    for (int rb = 0; rb < nrows; rb += 256) {
        const int rr = rb + (threadIdx.x >> 2);
        bool active = rr < nrows;
        const int row = r0 + (active ? rr : 0);
        const int cnt = active ? a.nl_cnt[(size_t)g * a.nlr + row] : 0;
        if (cnt > a.nb_cap) { bad_list = true; active = false; }
        std::conditional_t<MIXED, PairAccF, PairAcc> acc;
        if constexpr (MIXED) {
          if (active) {
            const double4 pi = a.pos4s[row];
            const float2 li = make_float2((float)a.ljs[row].x, (float)a.ljs[row].y);
            const float qi = (float)pi.w, ke = (float)a.ke, keqi = ke * qi;
            const float rc2 = (float)a.rc2, alpha = (float)a.alpha, escale = (float)a.erfc_scale_f;
            const v4i* nl4 = reinterpret_cast<const v4i*>(a.nl) + (size_t)g * (a.nb_cap / kChunk) * a.nlr + row;
            struct Cand { double4 p; float2 lj; int slot; double3 wr; };
            auto gather = [&](int e, bool ok) {
                const int t = ok ? (e & kHalfSlotMask) : 0;
                const int wc = ok ? (e >> kHalfSlotBits) & 31 : 0;
                Cand cd;
                cd.p = a.pos4s[t];
                if constexpr (TYPES) {
                    cd.lj = ljtf[(unsigned)e >> kShiftBits];
                } else {
                    const double2 d = a.ljs[t];
                    cd.lj = make_float2((float)d.x, (float)d.y);
                }
                cd.slot = wdel[wc] + t;
                if constexpr (kWrapTab) cd.wr = wrt[wc];
                return cd;
            };
            auto eval = [&](const Cand& cd) {
                double dxd, dyd, dzd;
                if constexpr (TRIC) {
                    dxd = pi.x - cd.p.x; dyd = pi.y - cd.p.y; dzd = pi.z - cd.p.z;
                    min_image(a, dxd, dyd, dzd);
                } else {
                    dxd = pi.x - (cd.p.x + cd.wr.x);
                    dyd = pi.y - (cd.p.y + cd.wr.y);
                    dzd = pi.z - (cd.p.z + cd.wr.z);
                }
                const float dx = (float)dxd, dy = (float)dyd, dz = (float)dzd;
                const float r2 = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
                if (r2 <= rc2) {
                    const float inv_r = rsqrtf(r2);
                    const float ar = alpha * (r2 * inv_r);
                    const float y = ar * escale;
                    const int it = (int)y;
                    const float u = 2.0f * (y - (float)it) - 1.0f;
                    const float* c = tabf + it * (kErfcDegF + 1);
                    float pc = c[kErfcDegF];
#pragma unroll
                    for (int j = kErfcDegF - 1; j >= 0; j--) pc = fmaf(pc, u, c[j]);
                    const float e2 = __expf(-ar * ar);
                    const float ec = e2 * pc;
                    const float sig = li.x + cd.lj.x;
                    float s2 = inv_r * sig;
                    s2 *= s2;
                    const float sig6 = s2 * s2 * s2;
                    const float es6 = sig6 * li.y * cd.lj.y;
                    const float qj = ke * (float)cd.p.w * inv_r;
                    const float qq = qi * qj;
                    if (a.include_forces) {
                        const float inv_r2 = inv_r * inv_r;
                        const float dEdR = qq * inv_r2 * fmaf(ar * e2, 1.1283791670955126f, ec) +
                                           es6 * (12.0f * sig6 - 6.0f) * inv_r2;
                        const float fx = dEdR * dx, fy = dEdR * dy, fz = dEdR * dz;
                        const float dqj = keqi * inv_r * ec;
                        acc.fx += fx; acc.fy += fy; acc.fz += fz;
                        acc.dq = fmaf(qj, ec, acc.dq);
                        bad |= !(fmaxf(fmaxf(fabsf(fx), fabsf(fy)), fmaxf(fabsf(fz), fabsf(dqj))) < (float)kFixMax);
                        atomicAdd(&accw[0][cd.slot], to_fix(-(double)fx));
                        atomicAdd(&accw[1][cd.slot], to_fix(-(double)fy));
                        atomicAdd(&accw[2][cd.slot], to_fix(-(double)fz));
                        atomicAdd(&accw[3][cd.slot], to_fix((double)dqj));
                    }
                    acc.e += (double)fmaf(qq, ec, es6 * (sig6 - 1.0f));   // the whole pair energy
                }
            };
            walk_list(nl4, a.nlr, cnt, 0, 1, gather, eval);
          }
        } else if (active) {
            const double4 pi = a.pos4s[row];
            const double2 li = a.ljs[row];
            const double kqis = a.ke * pi.w * kFixScale;   // k_e q_i in fixed-point units
            const v4i* nl4 = reinterpret_cast<const v4i*>(a.nl) + (size_t)g * (a.nb_cap / kChunk) * a.nlr + row;
            struct Cand { double4 p; double2 lj; int slot; };
            auto gather = [&](int e, bool ok) {
                const int t = ok ? (e & kHalfSlotMask) : 0;
                Cand cd;
                cd.p = a.pos4s[t];
                if constexpr (TYPES) cd.lj = ljt[(unsigned)e >> kShiftBits];
                else cd.lj = a.ljs[t];
                cd.slot = wdel[ok ? (e >> kHalfSlotBits) & 31 : 0] + t;
                return cd;
            };
            // minimum-image pair vector d = x_i - x_j and r^2
            auto sep = [&](const double4& pj, double& dx, double& dy, double& dz) {
                dx = pi.x - pj.x; dy = pi.y - pj.y; dz = pi.z - pj.z;
                if constexpr (TRIC) {
                    min_image(a, dx, dy, dz);
                } else {
                    dx -= a.L.x * rint(dx * a.invL.x);
                    dy -= a.L.y * rint(dy * a.invL.y);
                    dz -= a.L.z * rint(dz * a.invL.z);
                }
                return dx * dx + dy * dy + dz * dz;
            };
            // the pair term of a pair within rc: i side in registers, j side into the window
            auto term = [&](const double4& pj, const double2& lj, int slot, double dx, double dy, double dz,
                            double r2) {
                const double ke = a.ke;
                const double two_over_sqrtpi = 1.1283791670955126;
                const double inv_r = rsqrt_fp64(r2);
                const double ar = a.alpha * (r2 * inv_r);
                double e2;
                const double ec = erfc_exp(ar, tab, a.erfc_scale, e2);
                const double qj = ke * pj.w * inv_r;
                const double qq = pi.w * qj;
                const double sig = li.x + lj.x;
                double s2 = inv_r * sig;
                s2 *= s2;
                const double sig6 = s2 * s2 * s2;
                const double es6 = sig6 * li.y * lj.y;
                if (a.include_forces) {
                    // the force on j, -F_ij, in fixed-point units (x -2^34: exact), which the
                    // i side also accumulates (negated and unscaled once at the end: the same
                    // bits as summing F_ij) -- the conversion is then one add per value
                    const double ndEdRs = fma(qq, ec + ar * e2 * two_over_sqrtpi, es6 * (12 * sig6 - 6)) *
                                          ((inv_r * inv_r) * -kFixScale);
                    const double nfx = ndEdRs * dx, nfy = ndEdRs * dy, nfz = ndEdRs * dz;
                    const double dqjs = kqis * inv_r * ec;
                    acc.fx += nfx; acc.fy += nfy; acc.fz += nfz;
                    acc.dq += qj * ec;
                    // fixed-point range: |nf_c| <= |ndEdRs| r <= |ndEdRs| rc (one bound for the three
                    // components; an infinite or NaN term fails it)
                    bad |= !(fmax(fabs(ndEdRs) * a.rc, fabs(dqjs)) < kFixMax * kFixScale);
                    atomicAdd(&accw[0][slot], scaled_to_fix(nfx));
                    atomicAdd(&accw[1][slot], scaled_to_fix(nfy));
                    atomicAdd(&accw[2][slot], scaled_to_fix(nfz));
                    atomicAdd(&accw[3][slot], scaled_to_fix(dqjs));
                }
                acc.e += qq * ec + es6 * (sig6 - 1);   // the whole pair energy: each pair once
            };
            auto eval = [&](const Cand& cd) {
                double dx, dy, dz;
                const double r2 = sep(cd.p, dx, dy, dz);
                if (r2 <= a.rc2) term(cd.p, cd.lj, cd.slot, dx, dy, dz, r2);   // exact voxel-hash test
            };
            walk_list(nl4, a.nlr, cnt, 0, 1, gather, eval);
        }
#pragma unroll
        for (int m = 1; m < 4; m <<= 1) {
            acc.fx += __shfl_xor(acc.fx, m); acc.fy += __shfl_xor(acc.fy, m); acc.fz += __shfl_xor(acc.fz, m);
            acc.dq += __shfl_xor(acc.dq, m); acc.e += __shfl_xor(acc.e, m);
        }
        if (active && g == 0) {
            const int i = a.atom_sorted[row];
            a.e_atom[3 * i + 1] = acc.e;
            if (a.include_forces) {
                a.dedq[i] = acc.dq;
                if constexpr (MIXED) {
                    a.f_part[3 * i] = acc.fx;
                    a.f_part[3 * i + 1] = acc.fy;
                    a.f_part[3 * i + 2] = acc.fz;
                } else {   // accumulated as -F in fixed-point units
                    a.f_part[3 * i] = acc.fx * -kFixInv;
                    a.f_part[3 * i + 1] = acc.fy * -kFixInv;
                    a.f_part[3 * i + 2] = acc.fz * -kFixInv;
                }
            }
        }
    }
    {
        const int why = (__ballot(bad_list) ? kHalfListOverflow : 0) | (__ballot(bad) ? kHalfFixedRange : 0);
        if (why && (threadIdx.x & 63) == 0) atomicOr(a.half_flag, why);
    }
    if (!a.include_forces) return;
    __syncthreads();
    unsigned long long* out = a.win_out + (size_t)cell * kHalfMaxWin * 4;
    for (int e = threadIdx.x; e < nw; e += kHalfBlock)
        reinterpret_cast<ulonglong4*>(out)[e] = make_ulonglong4(accw[0][e], accw[1][e], accw[2][e], accw[3][e]);
}

// sorted slot s: the j-side sums of the 18 windows holding s (those of the cells at x offset
// 0 and -1 from its own), converted from fixed point once (k_excl, before the exclusions)
__device__ __forceinline__ void half_window_sums(const DirectArgs& a, int s, double3& f, double& dq) {
    const int key = a.key_s[s];
    const int3 nc = a.nc;
    const int cz = key % nc.z, cy = (key / nc.z) % nc.y, cx = key / (nc.y * nc.z);
    const int jj = s - a.cstart[key];
    long long sx = 0, sy = 0, sz = 0, sq = 0;
    // batches of kBatch windows: every offset load of a batch in flight, then every window
    // load (two memory latencies per batch instead of two per window; integer sums, so the
    // order does not change the result)
    constexpr int kBatch = 6;
    static_assert(kHalfWin % kBatch == 0, "window batches");
#pragma unroll
    for (int k0 = 0; k0 < kHalfWin; k0 += kBatch) {
        int b[kBatch], slot[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; u++) {
            const int3 o = half_offset(k0 + u);
            b[u] = (wrap_cell(cx - o.x, nc.x) * nc.y + wrap_cell(cy - o.y, nc.y)) * nc.z + wrap_cell(cz - o.z, nc.z);
            slot[u] = a.win_woff[b[u] * kHalfWin + k0 + u] + jj;
        }
        if (a.win32) {   // (kernel-uniform) 32-bit sums, 16 B per slot
            uint4 v[kBatch];
#pragma unroll
            for (int u = 0; u < kBatch; u++) v[u] = reinterpret_cast<const uint4*>(a.win_out)[(size_t)b[u] * kHalfMaxWin + slot[u]];
#pragma unroll
            for (int u = 0; u < kBatch; u++) {
                sx += (int)v[u].x; sy += (int)v[u].y; sz += (int)v[u].z; sq += (int)v[u].w;
            }
        } else {
            ulonglong4 v[kBatch];
#pragma unroll
            for (int u = 0; u < kBatch; u++) v[u] = reinterpret_cast<const ulonglong4*>(a.win_out)[(size_t)b[u] * kHalfMaxWin + slot[u]];
#pragma unroll
            for (int u = 0; u < kBatch; u++) {
                sx += (long long)v[u].x; sy += (long long)v[u].y; sz += (long long)v[u].z; sq += (long long)v[u].w;
            }
        }
    }
    const double inv = a.win32 ? kFix32Inv : kFixInv;
    f = make_double3((double)sx * inv, (double)sy * inv, (double)sz * inv);
    dq = (double)sq * inv;
}

// ---------------------------------------------------------------------------------
// 4b' mixed precision (CF_PRECISION_MIXED): the same list walk with the pair term in fp32.
//     Pair vectors are formed and minimum-imaged in fp64 from the sorted coordinates and then
//     rounded to fp32; r^2 and the cutoff test in fp32; erfc(alpha r) = e^{-x^2} erfcx(x) with erfcx from a
//     piecewise degree-6 fp32 polynomial (relative error ~1e-7 on [0, alpha rc], so the
//     energy tail of the many distant pairs keeps fp32 relative accuracy, unlike the
//     1.5e-7-absolute Abramowitz-Stegun form) and one v_exp_f32; forces and dE/dq accumulate
//     in fp32 per lane, the energy in fp64; lanes are combined and the exclusion correction
//     is applied in fp64 (excl_atom).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void pair_term_f(PairAccF& acc, float ke, float alpha, int include_forces, const float* tab,
                                            float scale, float4 pi, float2 li, float4 pj, float2 lj2, float dx,
                                            float dy, float dz, float r2) {
    const float inv_r = rsqrtf(r2);
    const float r = r2 * inv_r;
    const float ar = alpha * r;
    const float y = ar * scale;
    const int it = (int)y;
    const float u = 2.0f * (y - (float)it) - 1.0f;
    const float* c = tab + it * (kErfcDegF + 1);
    float pc = c[kErfcDegF];
#pragma unroll
    for (int j = kErfcDegF - 1; j >= 0; j--) pc = fmaf(pc, u, c[j]);
    const float e2 = __expf(-ar * ar);
    const float ec = e2 * pc;
    const float sig = li.x + lj2.x;
    float s2 = inv_r * sig;
    s2 *= s2;
    const float sig6 = s2 * s2 * s2;
    const float es6 = sig6 * li.y * lj2.y;
    const float qq = ke * pi.w * pj.w * inv_r;
    if (include_forces) {
        const float inv_r2 = inv_r * inv_r;
        const float dEdR = qq * inv_r2 * fmaf(ar * e2, 1.1283791670955126f, ec) + es6 * (12.0f * sig6 - 6.0f) * inv_r2;
        acc.fx = fmaf(dEdR, dx, acc.fx);
        acc.fy = fmaf(dEdR, dy, acc.fy);
        acc.fz = fmaf(dEdR, dz, acc.fz);
        acc.dq = fmaf(ke * pj.w * inv_r, ec, acc.dq);
    }
    acc.e += (double)fmaf(qq, ec, es6 * (sig6 - 1.0f));   // halved once in store_pairs
}

template <int LPA, bool TYPES>
__global__ void __launch_bounds__(256) k_pairs_mixed(DirectArgs a) {
    __shared__ float2 ljt[kMaxLjTypes];
    __shared__ float tabf[kErfcMaxMF * (kErfcDegF + 1)];
    if (TYPES)
        for (int e = threadIdx.x; e < a.lj_ntypes; e += blockDim.x)
            ljt[e] = make_float2((float)a.lj_tab[e].x, (float)a.lj_tab[e].y);
    for (int e = threadIdx.x; e < a.erfc_m_f * (kErfcDegF + 1); e += blockDim.x) tabf[e] = a.erfc_tab_f[e];
    __syncthreads();
    const float escale = (float)a.erfc_scale_f;
    const int gt = xcd_block() * blockDim.x + threadIdx.x;
    const int c = gt / LPA, g = gt % LPA;
    const int seg = g % kSeg, part = g / kSeg;
    bool active = c < a.nlr;
    const int cc = active ? c : a.nlr - 1;
    const int ss = own_slot(a, cc);
    const int i = a.atom_sorted[ss];
    int cnt = active ? a.nl_cnt[(size_t)seg * a.nlr + cc] : 0;
    bool over = cnt > a.nb_cap;
#pragma unroll
    for (int m = 1; m < LPA; m <<= 1) over = __shfl_xor(over, m) || over;
    if (over) active = false;
    PairAccF acc;
    if (active) {
        const double4 pid = a.pos4s[ss];
        const float4 pi = make_float4(0.f, 0.f, 0.f, (float)pid.w);
        const double2 lid = a.ljs[ss];
        const float2 li = make_float2((float)lid.x, (float)lid.y);
        const float rc2 = (float)a.rc2, alpha = (float)a.alpha;
        const v4i* nl4 = reinterpret_cast<const v4i*>(a.nl) + (size_t)seg * (a.nb_cap / kChunk) * a.nlr + cc;
        constexpr int kMask = (1 << kShiftBits) - 1;
        struct Cand { double4 p; float2 lj; };
        auto gather = [&](int e, bool ok) {
            const int t = ok ? (e & kMask) : 0;
            Cand cd;
            cd.p = a.pos4s[t];
            if (TYPES) {
                cd.lj = ljt[(unsigned)e >> kShiftBits];
            } else {
                const double2 d = a.ljs[t];
                cd.lj = make_float2((float)d.x, (float)d.y);
            }
            return cd;
        };
        // the pair vector is formed and minimum-imaged in fp64 and only then rounded to fp32, so
        // its error is ~ulp(r) rather than ~ulp(L): independent of the box size (an fp32 copy of
        // the absolute coordinates loses 2e-6 nm at C5's L = 19.7 nm)
        auto eval = [&](const Cand& cd) {
            double dxd = pid.x - cd.p.x, dyd = pid.y - cd.p.y, dzd = pid.z - cd.p.z;
            min_image(a, dxd, dyd, dzd);
            const float dx = (float)dxd, dy = (float)dyd, dz = (float)dzd;
            const float r2 = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
            const float4 pj = make_float4(0.f, 0.f, 0.f, (float)cd.p.w);
            if (r2 <= rc2) pair_term_f(acc, (float)a.ke, alpha, a.include_forces, tabf, escale, pi, li, pj, cd.lj, dx, dy, dz, r2);
        };
        walk_list(nl4, a.nlr, cnt, part, LPA / kSeg, gather, eval);
    }
#pragma unroll
    for (int m = 1; m < LPA; m <<= 1) {
        acc.fx += __shfl_xor(acc.fx, m); acc.fy += __shfl_xor(acc.fy, m); acc.fz += __shfl_xor(acc.fz, m);
        acc.dq += __shfl_xor(acc.dq, m); acc.e += __shfl_xor(acc.e, m);
    }
    if (!active || g != 0) return;
    PairAcc ad;
    ad.fx = acc.fx; ad.fy = acc.fy; ad.fz = acc.fz; ad.dq = acc.dq; ad.e = acc.e;
    store_pairs(ad, a, i);
}

__device__ __forceinline__ void pair_rescan(const DirectArgs& a, const double* tab, int s, int i) {
    const double4 pi = a.pos4s[s];
    const double2 li = a.ljs[s];
    const int ex0 = a.ex_start[i], exc = a.ex_start[i + 1] - ex0;
    int reg[kMaxRegExcl];
#pragma unroll
    for (int k = 0; k < kMaxRegExcl; k++) reg[k] = k < exc ? a.ex_list[ex0 + k] : -1;
    PairAcc acc;
    scan_cells(a, s, pi, a.rc2, [&](int t, int, double dx, double dy, double dz, double r2) {
        if (exc && in_excl(a.atom_sorted[t], reg, exc, a.ex_list, ex0)) return;
        pair_term(acc, a, tab, pi, li, a.pos4s[t], a.ljs[t], dx, dy, dz, r2);
    });
    store_pairs(acc, a, i);
}

// 4c: per list row (owned atom): an atom whose neighbour list overflowed (denser than
//     planned; k_pairs skipped it) first rescans its cells, then the exclusion correction +
//     self term (one launch for both: the overflow check costs 4 coalesced count loads)
__global__ void __launch_bounds__(256) k_excl(DirectArgs a) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.nlr) return;
    const int s = own_slot(a, c);
    const int i = a.atom_sorted[s];
    bool over = false;
    if (a.half) {
        over = *a.half_flag != 0;   // the half-list sums are unusable: every atom is rescanned
    } else {
#pragma unroll
        for (int g = 0; g < kSeg; g++) over = over || a.nl_cnt[(size_t)g * a.nlr + c] > a.nb_cap;
    }
    if (over) {   // rare: erfcx table read from global memory
        pair_rescan(a, a.erfc_tab, s, i);
        if (!a.half && a.fallback) atomicAdd((unsigned long long*)&a.fallback[1], 1ull);
    }
    if (a.half && !over && a.include_forces) {    // the partner-side sums of the half list
        double3 f;
        double dq;
        half_window_sums(a, s, f, dq);
        excl_atom(a, i, f, dq);
    } else {
        excl_atom(a, i);
    }
}

// ---------------------------------------------------------------------------------
// 5. non-periodic all pairs (RCK:436-491).  The reference adds every pair i<j and then
//    subtracts the excluded ones with the same formula; here excluded pairs are simply
//    skipped.  One lane per owned atom, j tiles staged in LDS.
// ---------------------------------------------------------------------------------
constexpr int kNopbcTile = 256;

__global__ void __launch_bounds__(kNopbcTile) k_nopbc(int n, int lo, int hi, int include_forces, int include_energy, double ke,
                                                      const double* __restrict__ pos, const double* __restrict__ q,
                                                      const double2* __restrict__ lj, const int* __restrict__ ex_start,
                                                      const int* __restrict__ ex_list, double* __restrict__ dedq,
                                                      double* __restrict__ f_part, double* __restrict__ e_atom) {
    __shared__ double4 sp[kNopbcTile];
    __shared__ double2 sl[kNopbcTile];
    int i = lo + blockIdx.x * blockDim.x + threadIdx.x;
    bool active = i < hi;
    double4 pi = make_double4(0, 0, 0, 0);
    double2 li = make_double2(0, 0);
    int ex0 = 0, exc = 0;
    int reg[kMaxRegExcl];
    if (active) {
        pi = make_double4(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2], q[i]);
        li = lj[i];
        ex0 = ex_start[i]; exc = ex_start[i + 1] - ex0;
    }
#pragma unroll
    for (int k = 0; k < kMaxRegExcl; k++) reg[k] = k < exc ? ex_list[ex0 + k] : -1;
    double fx = 0, fy = 0, fz = 0, dq = 0, e = 0;
    for (int base = 0; base < n; base += kNopbcTile) {
        int j = base + threadIdx.x;
        __syncthreads();
        if (j < n) {
            sp[threadIdx.x] = make_double4(pos[3 * j], pos[3 * j + 1], pos[3 * j + 2], q[j]);
            sl[threadIdx.x] = lj[j];
        }
        __syncthreads();
        int m = min(kNopbcTile, n - base);
        if (!active) continue;
        for (int t = 0; t < m; t++) {
            int jj = base + t;
            if (jj == i) continue;
            if (exc && in_excl(jj, reg, exc, ex_list, ex0)) continue;
            double4 pj = sp[t];
            double2 lj2 = sl[t];
            double dx = pj.x - pi.x, dy = pj.y - pi.y, dz = pj.z - pi.z;  // getDeltaR(i, j)
            double inv_r = 1.0 / sqrt(dx * dx + dy * dy + dz * dz);
            double sig = li.x + lj2.x;
            double s2 = inv_r * sig; s2 *= s2;
            double sig6 = s2 * s2 * s2;
            double es6 = sig6 * li.y * lj2.y;
            double qq = ke * pi.w * pj.w * inv_r;
            if (include_energy) e += 0.5 * (qq + es6 * (sig6 - 1));
            if (include_forces) {
                double dEdR = (es6 * (12 * sig6 - 6) + qq) * inv_r * inv_r;
                fx -= dEdR * dx; fy -= dEdR * dy; fz -= dEdR * dz;
                dq += ke * pj.w * inv_r;
            }
        }
    }
    if (!active) return;
    e_atom[3 * i + 1] = e;
    e_atom[3 * i + 2] = 0;
    if (include_forces) {
        dedq[i] = dq;
        f_part[3 * i] = fx; f_part[3 * i + 1] = fy; f_part[3 * i + 2] = fz;
    }
}

// ---------------------------------------------------------------------------------
// 6. assemble + energy, one launch.  Assemble: F_b += F_part_b - sum_e dE/dq[a_e] *
//    dq_{a_e}/dx_b (chain rule as a per-x-atom gather; reference scatter RCK:493-499,
//    626-632), skipped when out is null.  Energy: fixed-order two-stage tree reduction
//    (deterministic): each block sums its kEChunk atoms' (self, direct, exclusion) energies;
//    the block that finishes last (atomic ticket) sums the block partials and the
//    reciprocal-space partials in fixed order, so the result does not depend on block
//    scheduling.  It also clears the neighbour-list rebuild flag for the next evaluation,
//    re-arms the multi-rank x-slab and (last_block_done) the ticket.
// ---------------------------------------------------------------------------------
constexpr int kEChunk = 256;

// block sums of four values, the same fixed order in every block (deterministic): a butterfly
// within each wave (shfl_xor), then the four waves' sums added in wave order by every thread --
// one barrier instead of the eight of an LDS tree (round 5: the last block's final sums sit on
// the step's exposed tail)
__device__ __forceinline__ void block_sum4(double& a0, double& a1, double& a2, double& a3, double (*red)[4]) {
    static_assert(kEChunk == 256, "four waves");
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        a0 += __shfl_xor(a0, m); a1 += __shfl_xor(a1, m); a2 += __shfl_xor(a2, m); a3 += __shfl_xor(a3, m);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[w][0] = a0; red[w][1] = a1; red[w][2] = a2; red[w][3] = a3; }
    __syncthreads();
    a0 = (red[0][0] + red[1][0]) + (red[2][0] + red[3][0]);
    a1 = (red[0][1] + red[1][1]) + (red[2][1] + red[3][1]);
    a2 = (red[0][2] + red[1][2]) + (red[2][2] + red[3][2]);
    a3 = (red[0][3] + red[1][3]) + (red[2][3] + red[3][3]);
}

__global__ void __launch_bounds__(kEChunk) k_assemble_energy(int lo, int hi, const int* __restrict__ cs,
                                                             const int2* __restrict__ ce, const double* __restrict__ dedq,
                                                             const double* __restrict__ dqdx,
                                                             const double* __restrict__ f_part, double* __restrict__ out,
                                                             const double* __restrict__ dedq_rec,
                                                             const double4* __restrict__ f_rec, double3 gscale,
                                                             const double* __restrict__ e_atom, double* __restrict__ part,
                                                             const double* __restrict__ e_rec_part, int nrec, int pbc,
                                                             double* __restrict__ terms, double* __restrict__ energy_out,
                                                             double* __restrict__ energy_int, int* __restrict__ ticket,
                                                             int* __restrict__ flag, int* __restrict__ xrange,
                                                             int* __restrict__ half_flag,
                                                             long long* __restrict__ fallback, int per,
                                                             const int* __restrict__ err, int* __restrict__ err_host) {
    __shared__ double red[4][4];
    double a0 = 0, a1 = 0, a2 = 0;
    // `per` chunks of kEChunk atoms per block at large N: fewer partials and fewer increments
    // of the one ticket address (as k_g_bin); each thread's energies are summed in chunk order
    for (int it = 0; it < per; it++) {
    const int b = lo + (blockIdx.x * per + it) * kEChunk + threadIdx.x;
    if (b < hi) {
        if (out) {
            double fx = f_part[3 * b], fy = f_part[3 * b + 1], fz = f_part[3 * b + 2];
            if (f_rec) {   // reciprocal part from the second stream, added as k_g_interp adds it
                const double4 r = f_rec[b];
                fx = fma(r.w * gscale.x, r.x, fx);
                fy = fma(r.w * gscale.y, r.y, fy);
                fz = fma(r.w * gscale.z, r.z, fz);
            }
            // entries in batches of 4: the entry loads, then their dE/dq and dq/dx gathers, all
            // in flight together (two memory latencies per batch, not per entry); the sums keep
            // the entry order
            const int k1 = cs[b + 1];
            for (int k0 = cs[b]; k0 < k1; k0 += 4) {
                int2 en[4];
#pragma unroll
                for (int u = 0; u < 4; u++) en[u] = ce[min(k0 + u, k1 - 1)];
                double g[4], d[4][3];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    g[u] = dedq[en[u].y];
                    d[u][0] = dqdx[3 * en[u].x]; d[u][1] = dqdx[3 * en[u].x + 1]; d[u][2] = dqdx[3 * en[u].x + 2];
                }
                if (dedq_rec) {
#pragma unroll
                    for (int u = 0; u < 4; u++) g[u] += dedq_rec[en[u].y];
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (k0 + u < k1) {
                        fx -= g[u] * d[u][0];
                        fy -= g[u] * d[u][1];
                        fz -= g[u] * d[u][2];
                    }
                }
            }
            out[3 * b] += fx;
            out[3 * b + 1] += fy;
            out[3 * b + 2] += fz;
        }
        a0 += e_atom[3 * b]; a1 += e_atom[3 * b + 1]; a2 += e_atom[3 * b + 2];
    }
    }
    double unused = 0;
    block_sum4(a0, a1, a2, unused, red);
    if (threadIdx.x == 0) {   // agent-scope stores, read back by the last block (last_block_done)
        st_agent(part + 3 * blockIdx.x, a0); st_agent(part + 3 * blockIdx.x + 1, a1); st_agent(part + 3 * blockIdx.x + 2, a2);
    }
    if (!last_block_done(ticket)) return;
    const int nparts = gridDim.x;
    a0 = 0; a1 = 0; a2 = 0;
    for (int k = threadIdx.x; k < nparts; k += 256) {
        a0 += ld_agent(part + 3 * k); a1 += ld_agent(part + 3 * k + 1); a2 += ld_agent(part + 3 * k + 2);
    }
    double r = 0;
    for (int k = threadIdx.x; k < nrec; k += 256) r += e_rec_part[k];
    __syncthreads();   // (red is reused)
    block_sum4(a0, a1, a2, r, red);
    if (threadIdx.x == 0) {
        const double t0 = a0, t1 = r, t2 = a1, t3 = a2;
        terms[0] = t0; terms[1] = t1; terms[2] = t2; terms[3] = t3;
        const double e = pbc ? (t0 + t1 + t2 + t3) : t2;
        *energy_int = e;
        if (energy_out) *energy_out = e;
        if (flag) *flag = 0;
        if (half_flag) {
            if (*half_flag && fallback) { fallback[0] += 1; fallback[2] |= *half_flag; }
            *half_flag = 0;
        }
        if (xrange) { xrange[0] = INT_MAX; xrange[1] = INT_MIN; }   // re-arm the grid x-slab
        // a tripped index guard (sticky: the handle stays failed) becomes visible to the host
        // (pinned, mapped) without any synchronisation; the normal path reads one word
        if (err && err_host) {
            const int v = ld_agent(err);
            if (v) __hip_atomic_store(err_host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ---------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------
static inline int nblk(int64_t n, int b) { return (int)((n + b - 1) / b); }

// erfcx(x) = erfc(x) e^{x^2} on [0, xmax]: Chebyshev interpolation in long double on
// intervals of width w, stored as monomials in u in [-1, 1] per interval.  fp64: width 1/16,
// degree 7 (max relative error 3.6e-16 on [0, 3.2], host sweep against erfcl*expl: the same
// accuracy as width 0.375 / degree 12, for 5 FMAs and 5 LDS coefficient reads fewer per pair).
std::vector<double> erfc_table(double xmax, double* scale, int* m) {
    // stored coefficient-major with a fixed stride of kErfcMaxM intervals (erfc_exp)
    std::vector<double> t = erfc_table_deg(xmax, kErfcDeg, 0.0625, kErfcMaxM, scale, m);
    std::vector<double> cm((size_t)(kErfcDeg + 1) * kErfcMaxM, 0.0);
    for (int i = 0; i < *m; i++)
        for (int j = 0; j <= kErfcDeg; j++) cm[(size_t)j * kErfcMaxM + i] = t[(size_t)i * (kErfcDeg + 1) + j];
    return cm;
}

std::vector<float> erfc_table_f(double xmax, double* scale, int* m) {
    std::vector<double> t = erfc_table_deg(xmax, kErfcDegF, 0.375, kErfcMaxMF, scale, m);
    return std::vector<float>(t.begin(), t.end());
}

std::vector<double> erfc_table_deg(double xmax, int deg, double width, int max_m, double* scale, int* m) {
    const long double w = width;
    int M = (int)std::ceil((long double)xmax / w) + 1;
    if (M > max_m) throw std::invalid_argument("alpha * cutoff too large for the erfc table");
    const int n = deg + 1;
    std::vector<double> tab((size_t)M * n);
    for (int i = 0; i < M; i++) {
        std::vector<long double> f(n), c(n, 0.0L);
        for (int k = 0; k < n; k++) {
            const long double t = cosl(3.14159265358979323846264338327950288L * (k + 0.5L) / n);
            const long double x = w * (i + 0.5L * (t + 1.0L));
            f[k] = erfcl(x) * expl(x * x);
        }
        for (int j = 0; j < n; j++) {
            long double sum = 0;
            for (int k = 0; k < n; k++)
                sum += f[k] * cosl(3.14159265358979323846264338327950288L * j * (k + 0.5L) / n);
            c[j] = (j == 0 ? 1.0L : 2.0L) * sum / n;
        }
        // Chebyshev -> monomial: T_0 = 1, T_1 = u, T_{j+1} = 2u T_j - T_{j-1}
        std::vector<std::vector<long double>> T(n, std::vector<long double>(n, 0.0L));
        T[0][0] = 1.0L;
        if (n > 1) T[1][1] = 1.0L;
        for (int j = 1; j + 1 < n; j++)
            for (int e = 0; e < n; e++) T[j + 1][e] = (e > 0 ? 2.0L * T[j][e - 1] : 0.0L) - T[j - 1][e];
        for (int e = 0; e < n; e++) {
            long double v = 0;
            for (int j = 0; j < n; j++) v += c[j] * T[j][e];
            tab[(size_t)i * n + e] = (double)v;
        }
    }
    *scale = (double)(1.0L / w);
    *m = M;
    return tab;
}

void launch_flux_terms(Handle& h, const double* pos) {
    if (h.nterms == 0) return;
    double3 L = make_double3(h.box_L[0], h.box_L[1], h.box_L[2]);
    hipLaunchKernelGGL(k_flux_terms, dim3(nblk(h.nterms, 256)), dim3(256), 0, h.stream, h.nterms, h.nb, h.na,
                       h.term_idx, h.term_par, pos, L, make_double3(h.box_t[0], h.box_t[1], h.box_t[2]), h.pbc,
                       h.dq_slot, h.dqdx);
}

void launch_atoms_prep(Handle& h, const double* pos, bool skin_check) {
    // the flag is 0 here: cleared at cf_create and by k_energy at the end of every evaluation
    const double lim = 0.5 * h.list_skin;
    hipLaunchKernelGGL(k_atoms_prep, dim3(nblk(h.n, 256)), dim3(256), 0, h.stream, h.n, h.q0, h.qcsr_start,
                       h.qcsr_slot, h.dq_slot, h.pbc, h.alpha, h.ke, h.q, h.dedq_self, h.e_atom, pos, h.pos_ref, lim * lim,
                       skin_check ? h.skin_flag : nullptr);
}

void launch_cell_sort(Handle& h, const double* pos) {
    double3 L = make_double3(h.box_L[0], h.box_L[1], h.box_L[2]);
    int3 nc = make_int3(h.nc[0], h.nc[1], h.nc[2]);
    int ncell = nc.x * nc.y * nc.z;
    const int* f = h.skin_flag;
    // scratch: cell_key = per-atom key, atom_val = provisional rank, key_tmp = per-cell
    // counts, atom_tmp = scattered order, cell_key_sorted's partner atom_new = final order
    // multi-rank: the owned rows in cell-sorted order come out of the same three launches
    int* oc = h.own_s ? h.own_cnt : nullptr;
    const double3 T = make_double3(h.box_t[0], h.box_t[1], h.box_t[2]);
    hipLaunchKernelGGL(k_cell_hist, dim3(nblk(h.n, 256)), dim3(256), 0, h.stream, h.n, f, pos, L, T, nc, h.cell_key,
                       h.atom_val, h.cell_cnt, h.e_ticket + kTicketCells, h.cell_start, h.cell_end, h.lo, h.hi, oc,
                       h.own_start, h.err_dev);
    hipLaunchKernelGGL(k_cell_scatter, dim3(nblk(h.n, 256)), dim3(256), 0, h.stream, h.n, f, h.cell_key, h.atom_val,
                       h.cell_start, h.atom_tmp, ncell, h.cell_cnt, oc, h.err_dev);
    hipLaunchKernelGGL(k_cell_order, dim3(ncell), dim3(256), 0, h.stream, ncell, f, h.cell_start,
                       h.cell_end, h.atom_tmp, h.key_tmp, h.lo, h.hi, h.own_start, oc ? h.own_s : nullptr, pos, L, T,
                       nc, h.zcol, h.n, h.err_dev);
    hipLaunchKernelGGL(k_cell_commit, dim3(nblk(h.n, 256)), dim3(256), 0, h.stream, h.n, f, h.cell_key, h.key_tmp,
                       pos, h.q, h.lj, L, T, h.cell_key_sorted, h.atom_sorted, h.pos4s, h.ljs,
                       h.atom_type, h.typ_s,
                       h.pos_ref, h.n_builds_dev, h.cluster ? h.pos4f : nullptr, h.cluster ? h.slot_of : nullptr, nc,
                       h.err_dev);
}

// the rebuild flag set by a one-thread kernel, not hipMemsetD32Async: in graph mode a captured memset
// node was seen to leave the flag clear when the direct chain's graph was replayed (C2, no skin:
// the forces / energy-only / forces captures and a replay queued without host syncs,
// CF_GUARD_REBUILD_FLAG, profiles/r06h_graph_flag_probe.txt); a kernel node is ordered like the
// chain's other kernels
__global__ void k_set_flag(int* __restrict__ flag) {
    if (threadIdx.x == 0) *flag = 1;
}

void launch_force_rebuild(Handle& h) {
    hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(64), 0, h.stream, h.skin_flag);
}

// zero-fill by a kernel, for the same reason (launch sequences that may be captured into graphs
// use no memset nodes)
__global__ void __launch_bounds__(256) k_zero(double* __restrict__ p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0.0;
}

void launch_zero(Handle& h, double* p, int64_t n) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_zero, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 2048)), dim3(256), 0, h.stream, p, n);
}

DirectArgs direct_args(Handle& h, const double* pos, int include_forces) {
    DirectArgs a;
    a.n = h.n; a.lo = h.lo; a.hi = h.hi; a.include_forces = include_forces;
    a.L = make_double3(h.box_L[0], h.box_L[1], h.box_L[2]);
    a.T = make_double3(h.box_t[0], h.box_t[1], h.box_t[2]);
    a.tric = h.tric ? 1 : 0;
    a.invL = make_double3(1.0 / h.box_L[0], 1.0 / h.box_L[1], 1.0 / h.box_L[2]);
    a.nc = make_int3(h.nc[0], h.nc[1], h.nc[2]);
    a.brute = (h.nc[0] < 3 || h.nc[1] < 3 || h.nc[2] < 3) ? 1 : 0;
    a.rc2 = h.cutoff * h.cutoff; a.rc = h.cutoff; a.alpha = h.alpha; a.ke = h.ke;
    a.erfc_tab = h.erfc_tab; a.erfc_scale = h.erfc_scale; a.erfc_m = h.erfc_m;
    a.erfc_tab_f = h.erfc_tab_f; a.erfc_scale_f = h.erfc_scale_f; a.erfc_m_f = h.erfc_m_f;
    a.rl2 = (h.cutoff + h.list_skin) * (h.cutoff + h.list_skin);
    a.nb_cap = h.nb_cap;
    a.nlr = h.hi - h.lo;
    a.own_s = h.own_s;
    a.own_start = h.world > 1 ? h.own_start : nullptr;
    a.flag = h.skin_flag;
    a.atom_sorted = h.atom_sorted; a.key_sorted = h.cell_key_sorted;
    a.cstart = h.cell_start; a.cend = h.cell_end;
    a.pos4s = h.pos4s; a.ljs = h.ljs;
    a.typ_s = h.typ_s; a.lj_tab = h.lj_tab; a.lj_ntypes = h.lj_ntypes;
    a.q = h.q; a.ex_start = h.ex_start; a.ex_list = h.ex_list;
    a.dedq_self = h.dedq_self;
    a.nl = h.nl; a.nl_cnt = h.nl_cnt;
    a.dedq = h.dedq; a.f_part = h.f_part; a.e_atom = h.e_atom;
    a.pos = pos;
    a.half = h.half ? 1 : 0;
    a.half_flag = h.half_flag;
    a.win_out = h.win_out;
    a.win_woff = h.win_woff;
    a.key_s = h.cell_key_sorted;
    a.fallback = h.n_fallback_dev;
    a.cl_start = h.cl_start; a.cl_info = h.cl_info; a.cpl = h.cpl; a.cpl_cnt = h.cpl_cnt; a.cpl_cap = h.cpl_cap;
    a.pos4f = h.pos4f; a.slot_of = h.slot_of;
    a.ncl_cap = h.ncl_cap;
    a.win32 = h.mixed && h.cluster ? 1 : 0;
    a.err = h.err_dev;
    {   // fp32 prefilter: |d| from fp32 coordinates of magnitude <= ~2 L carries an error below 8 ulp(L)
        const double Lmax = std::max(h.box_L[0], std::max(h.box_L[1], h.box_L[2])) + std::fabs(h.box_t[0]) +
                            std::fabs(h.box_t[1]) + std::fabs(h.box_t[2]);
        const double rcm = h.cutoff * (1.0 + 1e-5) + 8.0 * Lmax * 1.1920928955078125e-07;
        a.rcm2f = (float)(rcm * rcm);
    }
    return a;
}

void launch_nlist(Handle& h, const double* pos) {
    if (h.cluster) { launch_cluster_list(h); return; }   // cf_kernels_cluster.hip
    DirectArgs a = direct_args(h, pos, 0);
    if (a.brute || h.nc[0] < 4 || h.nc[1] < 4 || h.nc[2] < 4)
        hipLaunchKernelGGL(k_nlist, dim3(nblk(a.nlr, 256)), dim3(256), 0, h.stream, a);
    else
        hipLaunchKernelGGL(k_nlist_wave, dim3(nblk(a.nlr, kWaveNL)), dim3(kWaveNL * kSeg), 0, h.stream, a);
}

void launch_direct(Handle& h, const double* pos, int include_forces) {
    if (h.cluster) { launch_pairs_cluster(h, pos, include_forces); return; }   // cf_kernels_cluster.hip
    DirectArgs a = direct_args(h, pos, include_forces);
    if (a.half) {
        const int ncell = h.nc[0] * h.nc[1] * h.nc[2];
#define CF_PAIRS_HALF(TY_, MX_)                                                                              \
    if (a.tric) hipLaunchKernelGGL((k_pairs_half<TY_, MX_, true>), dim3(ncell), dim3(kHalfBlock), 0, h.stream, a); \
    else hipLaunchKernelGGL((k_pairs_half<TY_, MX_, false>), dim3(ncell), dim3(kHalfBlock), 0, h.stream, a)
        if (h.mixed) {
            if (a.typ_s) { CF_PAIRS_HALF(true, true); } else { CF_PAIRS_HALF(false, true); }
        } else {
            if (a.typ_s) { CF_PAIRS_HALF(true, false); } else { CF_PAIRS_HALF(false, false); }
        }
#undef CF_PAIRS_HALF
        return;
    }
    // lanes per atom: enough threads for ~2 waves per SIMD on 256 CUs
    const int64_t want = 256LL * 4 * 2 * 64;   // (LPA 4 measured best at C3: 0.296 vs 0.299 / 0.322 ms for 8 / 16)
    const bool ty = a.typ_s != nullptr;
    if (h.mixed) {
#define CF_PAIRS_MIXED(LPA_)                                                                                        \
    if (ty) hipLaunchKernelGGL((k_pairs_mixed<LPA_, true>), dim3(nblk((int64_t)a.nlr * LPA_, 256)), dim3(256), 0,   \
                               h.stream, a);                                                                        \
    else hipLaunchKernelGGL((k_pairs_mixed<LPA_, false>), dim3(nblk((int64_t)a.nlr * LPA_, 256)), dim3(256), 0,     \
                            h.stream, a)
        if ((int64_t)a.nlr * 4 >= want) { CF_PAIRS_MIXED(4); }
        else if ((int64_t)a.nlr * 8 >= want) { CF_PAIRS_MIXED(8); }
        else { CF_PAIRS_MIXED(16); }
#undef CF_PAIRS_MIXED
    } else if ((int64_t)a.nlr * 4 >= want) {
        if (ty) hipLaunchKernelGGL((k_pairs<4, true>), dim3(nblk((int64_t)a.nlr * 4, 256)), dim3(256), 0, h.stream, a);
        else hipLaunchKernelGGL((k_pairs<4, false>), dim3(nblk((int64_t)a.nlr * 4, 256)), dim3(256), 0, h.stream, a);
    } else if ((int64_t)a.nlr * 8 >= want) {
        if (ty) hipLaunchKernelGGL((k_pairs<8, true>), dim3(nblk((int64_t)a.nlr * 8, 256)), dim3(256), 0, h.stream, a);
        else hipLaunchKernelGGL((k_pairs<8, false>), dim3(nblk((int64_t)a.nlr * 8, 256)), dim3(256), 0, h.stream, a);
    } else {
        if (ty) hipLaunchKernelGGL((k_pairs<16, true>), dim3(nblk((int64_t)a.nlr * 16, 256)), dim3(256), 0, h.stream, a);
        else hipLaunchKernelGGL((k_pairs<16, false>), dim3(nblk((int64_t)a.nlr * 16, 256)), dim3(256), 0, h.stream, a);
    }
}

// overflowed atoms' rescan + the exclusion correction (after launch_direct)
void launch_direct_finish(Handle& h, const double* pos, int include_forces) {
    DirectArgs a = direct_args(h, pos, include_forces);
    hipLaunchKernelGGL(k_excl, dim3(nblk(a.nlr, 256)), dim3(256), 0, h.stream, a);
}

void launch_recip_add(Handle& h) {
    int nown = h.hi - h.lo;
    int nparts = h.kspace_algo == 0 ? h.fp.nparts() : 1;
    hipLaunchKernelGGL(k_recip_add, dim3(nblk(nown, 256)), dim3(256), 0, h.stream, h.lo, nown, nparts, h.t_part,
                       h.dedq, h.f_part);
}

void launch_nopbc(Handle& h, const double* pos, int include_forces, int include_energy) {
    int nown = h.hi - h.lo;
    hipLaunchKernelGGL(k_nopbc, dim3(nblk(nown, kNopbcTile)), dim3(kNopbcTile), 0, h.stream, h.n, h.lo, h.hi,
                       include_forces, include_energy, h.ke, pos, h.q, h.lj, h.ex_start, h.ex_list, h.dedq, h.f_part,
                       h.e_atom);
}

// The producer side of a fork / join hand-over: one thread adds 1 to the flag with a system-scope
// release (the consumer is the runtime's hipStreamWaitValue64 poller, which reads memory).  An
// increment rather than a stored value, so that a captured graph replays it unchanged; the host
// counts the evaluations (Handle::sync_seq / join_seq).  This kernel replaces
// hipStreamWriteValue64, whose runtime kernel started ~13 us after its predecessor on the
// producer's queue (the runtime's fences; profiles/r04q_stream_sync.txt).
__global__ void k_signal(unsigned long long* __restrict__ flag) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(flag, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_signal(Handle& h, unsigned long long* flag) {
    hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, h.stream, flag);
    // a signal that was not enqueued would leave its consumer's wait pending forever: fail inside
    // the hand-over's scope (SyncGuard, cf_api.hip), which resynchronises the counts
    check_hip(hipPeekAtLastError(), "k_signal launch");
}

void launch_assemble_energy(Handle& h, double* forces_out, int include_energy, double* energy_out) {
    const int nown = std::max(0, h.hi - h.lo);
    int nrec = (h.pbc && include_energy && h.rank == 0) ? h.e_rec_nblk : 0;
    const int per = h.block_rounds() > 0 ? std::min(8, h.block_rounds()) : std::max(1, std::min(8, nown / (kEChunk * 512)));   // as launch_grid_sort
    const int nparts = std::max(1, nblk(nown, kEChunk * per));
    hipLaunchKernelGGL(k_assemble_energy, dim3(nparts), dim3(kEChunk), 0, h.stream, h.lo, h.hi, h.ccsr_start,
                       h.ccsr_ent, h.dedq, h.dqdx, h.f_part, forces_out, h.rec_split ? h.dedq_rec : nullptr,
                       h.rec_split ? reinterpret_cast<const double4*>(h.f_rec) : nullptr,
                       make_double3(h.gp.ng[0] / h.box_L[0], h.gp.ng[1] / h.box_L[1], h.gp.ng[2] / h.box_L[2]), h.e_atom, h.e_part, h.e_rec_part, nrec, h.pbc,
                       h.terms_dev, energy_out, h.energy_dev, h.e_ticket + kTicketEnergy, h.skin_flag, h.g_xrange,
                       h.half ? h.half_flag : nullptr, h.n_fallback_dev, per, h.err_dev, h.err_host_dev);
}

}  // namespace cf
