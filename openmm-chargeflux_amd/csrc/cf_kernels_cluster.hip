// cf_kernels_cluster.hip -- the cluster-pair half list on one rank.
//
// Replaces the per-atom half list (k_nlist_wave + k_pairs_half) for the real-space erfc + LJ
// pair loop of RCK:562-593 (the reference's voxel-hash list, RCK:559, evaluates every
// non-excluded pair with minimum-image r <= rc).  Same pair set, same fixed-point partner side
// (the 18-cell LDS window, win_out, k_excl), a different traversal:
//
//  * clusters: runs of <= 4 consecutive sorted slots of one cell (cells are sorted by
//    z-columns, k_cell_order, so a cluster is spatially compact), with a bounding box taken at
//    the list build;
//  * cluster-pair list (k_cl_build, rebuilt only with the cell list): for every i-cluster the
//    j-clusters of its cell's 18-cell window whose boxes come within rc + skin, one 8-B entry
//    each -- the first slot of j, its window cell, and a 16-bit mask of the (i, j) atom pairs
//    to evaluate (exclusions, the lower triangle of a self pair and the empty slots of a
//    partial cluster cleared), so no exclusion test and no per-pair list entry remain;
//  * k_pairs_cq, one 1024-thread block per cell: a wave takes one i-cluster at a time.
//    Phase A tests 256 (i, j) atom pairs per step (16 entries x 4 j atoms, one j per lane,
//    against the 4 i atoms) against the cutoff in fp32 (a superset of r <= rc by a margin above
//    the fp32 rounding) and compacts the hits into 4 per-i-atom queues in LDS; whenever every
//    queue holds 16, phase B
//    evaluates 64 pairs -- 16 lanes per i atom -- in fp64 with the exact r <= rc test: i side
//    in registers, j side as 64-bit fixed point into the LDS window (ds_add_u64).  The fp64
//    term therefore runs on ~0.9 full waves instead of on every list entry within rc + skin
//    (1.5 entries per pair, with divergence), and the j coordinates of phase A come from one
//    128-B run per j-cluster instead of one scattered 32-B gather per entry.
#include <type_traits>

#include "cf_pair.h"

namespace cf {

constexpr int kClSize = 4;               // atoms per cluster
constexpr int kCqWaves = 16;             // waves per k_pairs_cq block (one cell, one block per CU: the LDS)
constexpr int kCqThreads = 64 * kCqWaves;
constexpr int kCqQ = kCqWaves > 12 ? 88 : 112;   // queue entries per i atom (a ring; what the 160 KB LDS leaves)
constexpr int kCqBatch = 16;             // list entries tested per phase-A step (64 j atoms, one per lane)
constexpr int kCqLpi = 16;               // phase-B lanes per i atom
constexpr int kClBuildThreads = 512;
constexpr int kClMaxCand = 1536;         // window clusters staged by k_cl_build (>= 4096 / 4 + 18 * 3)
constexpr unsigned kClSelfMask = 0x08CEu;
typedef float v2f __attribute__((ext_vector_type(2)));   // (il, jl) bits il*4 + jl with jl > il: a self pair's upper triangle

// window cell k of cell (cx, cy, cz): the wrapped cell index, and the vector from the cell's
// corner to the window cell's (unwrapped) corner, in which frame pos4f (corner-relative fp32
// positions, k_cell_commit) of the two cells compare: d = (p_i - p_j) - off
// (wrap: the lattice translation that brings the window cell's wrapped positions, pos4s, next to
// the cell: pos_j + wrap is the image of j within rc of the cell's atoms)
__device__ __forceinline__ int window_cell(int k, int cx, int cy, int cz, int3 nc, double3 L, double3 T,
                                           float4& off, double3* wrap = nullptr) {
    const int3 o = half_offset(k);
    const int u[3] = {cx + o.x, cy + o.y, cz + o.z}, n[3] = {nc.x, nc.y, nc.z};
    int w[3], m[3];
#pragma unroll
    for (int d = 0; d < 3; d++) {
        m[d] = u[d] >= n[d] ? 1 : (u[d] < 0 ? -1 : 0);
        w[d] = u[d] - m[d] * n[d];
    }
    const double3 v = lattice(L, T, (double)o.x / nc.x, (double)o.y / nc.y, (double)o.z / nc.z);
    off = make_float4((float)v.x, (float)v.y, (float)v.z, 0.f);
    if (wrap) *wrap = lattice(L, T, m[0], m[1], m[2]);
    return (w[0] * nc.y + w[1]) * nc.z + w[2];
}

// ---------------------------------------------------------------------------------
// cluster table (rebuild only): cl_start = exclusive scan of ceil(n_c / 4) over the cells (one
// block), then per cell its clusters' (first slot, count) and fp32 bounding boxes
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_cl_scan(int ncell, const int* __restrict__ flag, const int* __restrict__ cstart,
                                                  const int* __restrict__ cend, int* __restrict__ cl_start, int ncl_cap,
                                                  int* __restrict__ err) {
    __shared__ int sh[1024];
    if (!*flag) return;
    int carry = 0;
    for (int base = 0; base < ncell; base += 1024) {
        const int c = base + threadIdx.x;
        const int v = c < ncell ? (cend[c] - cstart[c] + kClSize - 1) / kClSize : 0;
        const int x = block_exclusive_scan_t<1024>(v, sh);
        if (c < ncell) cl_start[c] = carry + x;
        carry += sh[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        cl_start[ncell] = carry;
        // guard: sum ceil(n_c / 4) <= n / 4 + ncell = the table's size (cf_api.hip set_cells); the
        // kernels after it skip every cell whose clusters would pass the end
        if (carry > ncl_cap) atomicOr(err, kGuardClusterTable);
    }
}

// boxes in the cell's corner frame (pos4f); lo.w = the cluster's x key for the half rule: the
// absolute x of the box centre, a function of the cluster alone (both sides of a pair see the same)
__global__ void __launch_bounds__(256) k_cl_bbox(int ncell, const int* __restrict__ flag, const int* __restrict__ cstart,
                                                 const int* __restrict__ cend, const int* __restrict__ cl_start,
                                                 const float4* __restrict__ pos4f, int2* __restrict__ cl_info,
                                                 float4* __restrict__ cl_bb, int3 nc, double3 L, double3 T,
                                                 const int* __restrict__ atom_sorted, int lo, int hi, int n,
                                                 int ncl_cap) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= ncell || !*flag) return;
    const int b = cstart[c], e = cend[c], k0 = cl_start[c];
    if (cl_start[c + 1] > ncl_cap) return;   // guard (k_cl_scan flagged it)
    const double ox = lattice(L, T, (double)(c / (nc.y * nc.z)) / nc.x, (double)((c / nc.z) % nc.y) / nc.y,
                              (double)(c % nc.z) / nc.z).x;
    for (int k = lane; k * kClSize < e - b; k += 64) {
        const int first = b + k * kClSize, cnt = min(kClSize, e - first);
        float4 bl = pos4f[first], bh = bl;
        bool own = lo == 0 && hi == n;   // one rank: every cluster is owned
        for (int u = 0; u < cnt; u++) {
            const float4 p = pos4f[first + u];
            bl.x = fminf(bl.x, p.x); bl.y = fminf(bl.y, p.y); bl.z = fminf(bl.z, p.z);
            bh.x = fmaxf(bh.x, p.x); bh.y = fmaxf(bh.y, p.y); bh.z = fmaxf(bh.z, p.z);
            const int ai = atom_sorted[first + u];
            own = own || (ai >= lo && ai < hi);
        }
        cl_info[k0 + k] = make_int2(first, cnt);
        bl.w = (float)(ox + 0.5 * ((double)bl.x + (double)bh.x));
        bh.w = own ? 1.f : 0.f;   // the cluster holds an atom this rank owns (k_cl_build's filter)
        cl_bb[2 * (k0 + k)] = bl;
        cl_bb[2 * (k0 + k) + 1] = bh;
    }
}

// ---------------------------------------------------------------------------------
// cluster-pair list (rebuild only): one block per cell.  The j-clusters of the cell's 18-cell
// window are staged in LDS with their boxes moved to the cell's image; each wave takes the
// cell's i-clusters in turn and tests 64 candidates per step: box distance <= rc + skin, the
// half rule at cluster level -- the x rule of the per-atom half list with the box centres as
// keys: window cells at x offset +1, every cluster; x offset 0, the clusters with a larger x key
// (ties: the larger cluster index, the pair itself included), so each unordered pair is listed
// once and every i-cluster keeps about half of its partners -- then the pair mask.
// Entries are written compacted in candidate order (deterministic); a count above the capacity
// is stored as it is and makes k_pairs_cq raise the list-overflow fallback on every evaluation
// that uses this list.
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(kClBuildThreads) k_cl_build(DirectArgs a, const float4* __restrict__ cl_bb,
                                                              uint2* __restrict__ cpl, int* __restrict__ cpl_cnt,
                                                              float rlm2) {
    __shared__ float4 cand_lo[kClMaxCand], cand_hi[kClMaxCand];   // w: cluster index | (count - 1) << 29 / first | k << 21
    __shared__ float cand_x[kClMaxCand];                             // x keys (k_cl_bbox)
    __shared__ int woff[kHalfWin + 1];
    __shared__ int wcl[kHalfWin];
    __shared__ float4 wsh[kHalfWin];
    __shared__ int exs[kClBuildThreads / 64][64];   // per wave: the i-cluster's excluded partners, il << 24 | slot
    if (!*a.flag) return;
    const int cell = xcd_block();
    const int3 nc = a.nc;
    const int cz = cell % nc.z, cy = (cell / nc.z) % nc.y, cx = cell / (nc.y * nc.z);
    if (threadIdx.x < kHalfWin) {
        float4 off;
        wcl[threadIdx.x] = window_cell(threadIdx.x, cx, cy, cz, nc, a.L, a.T, off);
        wsh[threadIdx.x] = off;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int off = 0;
        for (int k = 0; k < kHalfWin; k++) {
            woff[k] = off;
            off += a.cl_start[wcl[k] + 1] - a.cl_start[wcl[k]];
        }
        woff[kHalfWin] = off;
    }
    __syncthreads();
    const int ncand = woff[kHalfWin];
    if (ncand > kClMaxCand) {   // block-uniform: a window this full also exceeds k_pairs_cq's LDS window
        if (threadIdx.x == 0) atomicOr(a.half_flag, kHalfWindowFull);
        // overflowed counts: every evaluation that keeps this list falls back, not only this one
        for (int ci = a.cl_start[cell] + threadIdx.x; ci < a.cl_start[cell + 1]; ci += kClBuildThreads)
            cpl_cnt[ci] = a.cpl_cap + 1;
        return;
    }
    for (int t = threadIdx.x; t < ncand; t += kClBuildThreads) {
        int k = 0;
        while (woff[k + 1] <= t) k++;
        const int cj = a.cl_start[wcl[k]] + (t - woff[k]);
        const float4 sh = wsh[k];
        const float4 lo = cl_bb[2 * cj], hi = cl_bb[2 * cj + 1];
        const int first = a.cl_info[cj].x;
        const unsigned ownj = hi.w != 0.f ? 0x80000000u : 0u;
        cand_lo[t] = make_float4(lo.x + sh.x, lo.y + sh.y, lo.z + sh.z,
                                 __int_as_float((int)((unsigned)cj | ((unsigned)(a.cl_info[cj].y - 1) << 29) | ownj)));
        cand_hi[t] = make_float4(hi.x + sh.x, hi.y + sh.y, hi.z + sh.z, __int_as_float(first | (k << kHalfSlotBits)));
        cand_x[t] = lo.w;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int c0 = a.cl_start[cell], c1 = a.cl_start[cell + 1];
    if (c1 > a.ncl_cap) return;   // guard (k_cl_scan flagged it; block-uniform)
    for (int ci = c0 + wv; ci < c1; ci += kClBuildThreads / 64) {
        const float4 ilo = cl_bb[2 * ci], ihi = cl_bb[2 * ci + 1];
        const float xki = ilo.w;
        const bool owni = ihi.w != 0.f;   // several ranks: a pair is listed when either cluster holds an owned atom
        const int2 ii = a.cl_info[ci];
        const unsigned rows = (1u << (4 * ii.y)) - 1u;   // bits of the valid i atoms (il < count)
        uint2* out = cpl + (size_t)ci * a.cpl_cap;
        int cnt = 0;
        // the i atoms' excluded partners as sorted slots, gathered once per i-cluster (lane il * 16 + e:
        // exclusion e of atom il; an atom with more than 16 exclusions takes the slow loop below)
        int nex = 0;
        bool many = false;
        // the sorted-slot range of the i atoms' excluded partners: a j cluster whose 4 slots lie
        // outside it needs no exclusion pass (for molecules, every cluster but the few holding
        // the i atoms' own molecule partners)
        int exlo = INT_MAX, exhi = INT_MIN;
        {
            const int il = lane >> 4, e = lane & 15;
            int v = -1;
            if (il < ii.y) {
                const int ai = a.atom_sorted[ii.x + il];
                const int e0 = a.ex_start[ai], ne = a.ex_start[ai + 1] - e0;
                many = ne > 16;
                if (e < ne) v = (il << 24) | a.slot_of[a.ex_list[e0 + e]];
            }
            many = __ballot(many) != 0;
            const unsigned long long has = __ballot(v >= 0);
            const int r = __popcll(has & ((1ull << lane) - 1ull));
            if (v >= 0) exs[wv][r] = v;
            nex = __popcll(has);
            int mn = v >= 0 ? (v & 0xFFFFFF) : INT_MAX, mx = v >= 0 ? (v & 0xFFFFFF) : INT_MIN;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                mn = min(mn, __shfl_xor(mn, o));
                mx = max(mx, __shfl_xor(mx, o));
            }
            exlo = __builtin_amdgcn_readfirstlane(mn);
            exhi = __builtin_amdgcn_readfirstlane(mx);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        for (int t0 = 0; t0 < ncand; t0 += 64) {
            const int t = t0 + lane;
            bool hit = false;
            unsigned mask = 0;
            int ent = 0;
            if (t < ncand) {
                const float4 lo = cand_lo[t], hi = cand_hi[t];
                const float dx = fmaxf(0.f, fmaxf(lo.x - ihi.x, ilo.x - hi.x));
                const float dy = fmaxf(0.f, fmaxf(lo.y - ihi.y, ilo.y - hi.y));
                const float dz = fmaxf(0.f, fmaxf(lo.z - ihi.z, ilo.z - hi.z));
                const int cj = __float_as_int(lo.w) & 0x1FFFFFFF;
                ent = __float_as_int(hi.w);
                const int k = ent >> kHalfSlotBits;
                const float xkj = cand_x[t];
                const bool ownj = (unsigned)__float_as_int(lo.w) >> 31;
                if (dx * dx + dy * dy + dz * dz <= rlm2 && (k >= 9 || xkj > xki || (xkj == xki && cj >= ci)) &&
                    (owni || ownj)) {
                    const int jcnt = (((unsigned)__float_as_int(lo.w) >> 29) & 3u) + 1;
                    const unsigned cols = 0x1111u * ((1u << jcnt) - 1u);   // bits of the valid j atoms
                    mask = rows & cols & (cj == ci ? kClSelfMask : 0xFFFFu);
                    hit = true;
                }
            }
            if (!__ballot(hit)) continue;
            // exclusions of the i atoms (wave-uniform loop over their partners' sorted slots), for
            // the batches with a hit whose slots can hold one of them
            const int jfirst = ent & kHalfSlotMask;
            if (many || __ballot(hit && jfirst + kClSize > exlo && jfirst <= exhi)) {
            if (!many) {
                for (int x = 0; x < nex; x++) {
                    const int v = exs[wv][x];
                    const int d = (v & 0xFFFFFF) - jfirst;
                    if (hit && d >= 0 && d < kClSize) mask &= ~(1u << (4 * (v >> 24) + d));
                }
            } else {
                for (int il = 0; il < ii.y; il++) {
                    const int ai = a.atom_sorted[ii.x + il];
                    for (int e = a.ex_start[ai]; e < a.ex_start[ai + 1]; e++) {
                        const int d = a.slot_of[a.ex_list[e]] - jfirst;
                        if (hit && d >= 0 && d < kClSize) mask &= ~(1u << (4 * il + d));
                    }
                }
            }
            }
            hit = hit && mask != 0;
            const unsigned long long bal = __ballot(hit);
            const int rank = __popcll(bal & ((1ull << lane) - 1ull));
            if (hit && cnt + rank < a.cpl_cap) out[cnt + rank] = make_uint2((unsigned)ent, mask);
            cnt += __popcll(bal);
        }
        if (lane == 0) cpl_cnt[ci] = cnt;
    }
}

// ---------------------------------------------------------------------------------
// k_pairs_cq: the pair loop over the cluster-pair list (see the top of this file)
// ---------------------------------------------------------------------------------
// MIXED (CF_PRECISION_MIXED, C5): phase B in fp32 -- the pair vector from the corner-relative
// fp32 positions and the window cell's offset (no fp64 minimum image: the corner frame keeps the
// coordinates small, so fp32 carries ~1e-7 nm whatever the box size), erfc from the degree-6 fp32
// table, fp32 i-side sums, fp64 energy, the j side in the same fixed point (an fp32 value times
// 2^34 is exact in fp64)
// One block per cell (xcd_block: XCD blockIdx % 8 takes a contiguous eighth of the cells).  Round 5
// measured the alternative of persistent blocks taking cells from per-XCD counters and leaving CUs
// to the other stream's DFT stages: with ~2.3 cells per block the last round of cells leaves most
// CUs idle, the kernel ran 250 against 171 us and the step gained nothing
// (profiles/r05o_persistent_pair_kernel.txt).
template <bool TYPES, bool MIXED>
__global__ void __launch_bounds__(kCqThreads) CF_LDS_UNPAIRED k_pairs_cq(DirectArgs a, int cell0) {
    __shared__ double tab[MIXED ? 1 : kErfcMaxM * (kErfcDeg + 1)];
    __shared__ float tabf[MIXED ? kErfcMaxMF * (kErfcDegF + 1) : 1];
    __shared__ double2 ljt[TYPES ? kMaxLjTypes : 1];
    __shared__ int2 win[kHalfWin];          // (first sorted slot, window offset) per window cell
    __shared__ int wdel[kHalfWin];          // window offset - first sorted slot
    __shared__ float4 shf[kHalfWin];        // corner offset of each window cell (phase A, window_cell)
    __shared__ double3 shd[kHalfWin];       // wrap translation of each window cell (phase B, window_cell)
    // j-side fx, fy, fz, dE/dq in fixed point: 64-bit (2^-34) in fp64, 32-bit (2^-13) in mixed precision
    __shared__ std::conditional_t<MIXED, unsigned, unsigned long long> accw[4][kHalfMaxWin];
    __shared__ int qbuf[kCqWaves][4][kCqQ];  // per wave, per i atom: ring of hit entries
    __shared__ int wtot, next_ci, nown;
    const int3 nc = a.nc;
    if constexpr (TYPES)
        for (int e = threadIdx.x; e < a.lj_ntypes; e += kCqThreads) ljt[e] = a.lj_tab[e];
    if constexpr (MIXED) {
        for (int e = threadIdx.x; e < a.erfc_m_f * (kErfcDegF + 1); e += kCqThreads) tabf[e] = a.erfc_tab_f[e];
    } else {
        for (int e = threadIdx.x; e < kErfcMaxM * (kErfcDeg + 1); e += kCqThreads) tab[e] = a.erfc_tab[e];
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    bool bad = false, bad_list = false, bad_idx = false;
    auto process = [&](const int cell) {
    const int cz = cell % nc.z, cy = (cell / nc.z) % nc.y, cx = cell / (nc.y * nc.z);
    if (threadIdx.x == 0) nown = 0;
    __syncthreads();
    if (threadIdx.x < kHalfWin) {
        float4 off;
        double3 wr;
        const int w = window_cell(threadIdx.x, cx, cy, cz, nc, a.L, a.T, off, &wr);
        const int b = a.cstart[w];
        win[threadIdx.x] = make_int2(b, a.cend[w] - b);
        shf[threadIdx.x] = off;
        shd[threadIdx.x] = wr;
        // several ranks: owned atoms in the window (its own cell is window cell 0)
        if (a.own_start && a.own_start[w + 1] > a.own_start[w]) atomicAdd(&nown, 1);
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
        next_ci = 0;
        if (off > kHalfMaxWin) atomicOr(a.half_flag, kHalfWindowFull);
    }
    __syncthreads();
    const int nw = wtot;
    if (nw > kHalfMaxWin) return;   // block-uniform; k_excl recomputes everything
    // several ranks: no owned atom in the cell or its window -- no pair this rank keeps has an atom
    // here, and k_excl reads this window only for owned atoms of the window's cells (none): skip
    if (a.own_start && nown == 0) return;   // block-uniform
    if (threadIdx.x < kHalfWin) a.win_woff[cell * kHalfWin + threadIdx.x] = win[threadIdx.x].y;
    for (int e = threadIdx.x; e < nw; e += kCqThreads) {
        accw[0][e] = 0; accw[1][e] = 0; accw[2][e] = 0; accw[3][e] = 0;
    }
    __syncthreads();

    const int il = lane >> 4, kk = lane & 15;          // phase B: i atom il, lane kk of its 16
    const int jl = lane & 3, el = lane >> 2;           // phase A: entry el of the batch, j atom jl
    int* const qw = qbuf[wv][il];
    const int c0 = a.cl_start[cell], ncl = a.cl_start[cell + 1] - c0;
    if (c0 + ncl > a.ncl_cap) return;   // guard (k_cl_scan flagged it; block-uniform)
    // x < 2 kCqQ -> x mod kCqQ (x - kCqQ underflows to a larger unsigned when x < kCqQ)
    auto ring = [](int x) { return (int)min((unsigned)x, (unsigned)x - (unsigned)kCqQ); };
    for (;;) {
        int ci = 0;
        if (lane == 0) ci = atomicAdd(&next_ci, 1);
        ci = __builtin_amdgcn_readfirstlane(__shfl(ci, 0));
        if (ci >= ncl) break;
        ci += c0;
        const int2 inf = a.cl_info[ci];
        const int islot = inf.x + min(il, inf.y - 1);
        const double4 pi = a.pos4s[islot];
        const double2 li = TYPES ? ljt[__float_as_int(a.pos4f[islot].w)] : a.ljs[islot];
        const double kqis = a.ke * pi.w * kFixScale;   // k_e q_i in fixed-point units
        const float kef = (float)a.ke, kqisf = kef * (float)pi.w * kFix32Scale;   // (mixed: 2^13 units)
        // the 4 i atoms' fp32 positions, wave-uniform (phase A tests every lane's j against all 4)
        float4 pif[4];   // (readfirstlane: kept in SGPRs, VOP2 operands of the tests)
        auto sgpr = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const float4 v = a.pos4f[inf.x + min(k, inf.y - 1)];
            pif[k] = make_float4(sgpr(v.x), sgpr(v.y), sgpr(v.z), 0.f);
        }
        int ne = a.cpl_cnt[ci];
        if (ne > a.cpl_cap) { bad_list = true; ne = 0; }   // the evaluation falls back (k_excl rescans)
        const uint2* lst = a.cpl + (size_t)ci * a.cpl_cap;
        std::conditional_t<MIXED, PairAccF, PairAcc> acc;
        int q0 = 0, q1 = 0, q2 = 0, q3 = 0;   // queue lengths (wave-uniform)
        int qh = 0;     // ring head, equal for the 4 queues (every phase-B step pops 16 from each)

        // phase B: lanes kk < qlen of each i atom evaluate the pair of queue entry qh + kk
        // Prefetch: whenever every queue holds a full step, its entries and j coordinates are
        // loaded at once (issue_pf) and used by the next phase B, which therefore does not wait
        // for them.  Phase B runs while every queue holds 32 (keeping 16 in reserve for the next
        // prefetch; the same lane efficiency as draining at 16: the ends of the lists decide it,
        // tools/cluster_proto.py), so the prefetched loads complete during the next batch's tests.
        bool pf_ok = false;   // (wave-uniform)
        int pf_wq = 0;
        double4 pf_pj = make_double4(0.0, 0.0, 0.0, 0.0);
        auto all_ge = [&](int v) { return q0 >= v && q1 >= v && q2 >= v && q3 >= v; };
        auto issue_pf = [&]() {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            pf_wq = qw[ring(qh + kk)];
            pf_pj = a.pos4s[pf_wq & kHalfSlotMask];
            pf_ok = true;
        };
        auto phase_b = [&]() {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // this lane's queue length: the four packed one byte each (lengths < 256)
            const unsigned qpack = (unsigned)q0 | ((unsigned)q1 << 8) | ((unsigned)q2 << 16) | ((unsigned)q3 << 24);
            const int qlen = (int)((qpack >> (8 * il)) & 255u);
            const bool act = kk < qlen;
            int wq;
            double4 pj;
            if (pf_ok) {
                wq = pf_wq;
                pj = pf_pj;
                pf_ok = false;
            } else {
                wq = act ? qw[ring(qh + kk)] : islot;
                pj = a.pos4s[wq & kHalfSlotMask];
            }
            const int j = wq & kHalfSlotMask;
            const double3 wr = shd[(wq >> kHalfSlotBits) & 31];
            // the pair vector to j's image next to the cell: the wrap translation of j's window cell
            // (for a pair within rc < L/2 the same image, and for an orthorhombic box the same bits,
            // as the minimum image d - L rint(d / L))
            const double ddx = pi.x - (pj.x + wr.x), ddy = pi.y - (pj.y + wr.y), ddz = pi.z - (pj.z + wr.z);
            if constexpr (MIXED) {
                // formed in fp64 from the wrapped coordinates, then rounded: its error is ~ulp(r),
                // not ulp of a coordinate
                const float qjv = (float)pj.w;
                const float dx = (float)ddx, dy = (float)ddy, dz = (float)ddz;
                const float r2 = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
                if (act && r2 <= (float)a.rc2) {
                    const int slot = wdel[(wq >> kHalfSlotBits) & 31] + j;
                    const double2 ljd = TYPES ? ljt[(unsigned)wq >> kShiftBits] : a.ljs[j];
                    const float qi = (float)pi.w;
                    const float inv_r = rsqrtf(r2);
                    const float ar = (float)a.alpha * (r2 * inv_r);
                    const float y = ar * (float)a.erfc_scale_f;
                    const int it = (int)y;
                    const float u = 2.0f * (y - (float)it) - 1.0f;
                    const float* c = tabf + it * (kErfcDegF + 1);
                    float pc = c[kErfcDegF];
#pragma unroll
                    for (int q = kErfcDegF - 1; q >= 0; q--) pc = fmaf(pc, u, c[q]);
                    const float e2 = __expf(-ar * ar);
                    const float ec = e2 * pc;
                    const float sig = (float)li.x + (float)ljd.x;
                    float s2 = inv_r * sig;
                    s2 *= s2;
                    const float sig6 = s2 * s2 * s2;
                    const float es6 = sig6 * (float)li.y * (float)ljd.y;
                    const float qj = kef * qjv * inv_r;
                    const float qq = qi * qj;
                    if (a.include_forces) {
                        // -F_ij and dE/dq_j in fixed-point units (x -2^13 / x 2^13: exact), the
                        // i side accumulated in the same units (unscaled at the end, exactly)
                        const float inv_r2 = inv_r * inv_r;
                        const float ndEdRs = (qq * inv_r2 * fmaf(ar * e2, 1.1283791670955126f, ec) +
                                              es6 * (12.0f * sig6 - 6.0f) * inv_r2) * -kFix32Scale;
                        const float nfx = ndEdRs * dx, nfy = ndEdRs * dy, nfz = ndEdRs * dz;
                        const float dqjs = kqisf * inv_r * ec;
                        acc.fx += nfx; acc.fy += nfy; acc.fz += nfz;
                        acc.dq = fmaf(qj, ec, acc.dq);
                        bad |= !(fmaxf(fmaxf(fabsf(nfx), fabsf(nfy)), fmaxf(fabsf(nfz), fabsf(dqjs))) <
                                 (float)kFixMax * kFix32Scale);
                        atomicAdd(&accw[0][slot], scaled_to_fix32(nfx));
                        atomicAdd(&accw[1][slot], scaled_to_fix32(nfy));
                        atomicAdd(&accw[2][slot], scaled_to_fix32(nfz));
                        atomicAdd(&accw[3][slot], scaled_to_fix32(dqjs));
                    }
                    acc.e += (double)fmaf(qq, ec, es6 * (sig6 - 1.0f));   // the whole pair energy
                }
                qh = ring(qh + kCqLpi);
                q0 = max(q0 - kCqLpi, 0); q1 = max(q1 - kCqLpi, 0); q2 = max(q2 - kCqLpi, 0); q3 = max(q3 - kCqLpi, 0);
                if (all_ge(kCqLpi)) issue_pf();
                return;
            }
            const double2 lj = TYPES ? ljt[(unsigned)wq >> kShiftBits] : a.ljs[j];
            const double dx = ddx, dy = ddy, dz = ddz;
            const double r2 = dx * dx + dy * dy + dz * dz;
            if (act && r2 <= a.rc2) {   // exact voxel-hash test (RCK:567-569)
                const int slot = wdel[(wq >> kHalfSlotBits) & 31] + j;
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
                    // -F_ij in fixed-point units (x -2^34: exact), accumulated on both sides
                    const double ndEdRs = fma(qq, ec + ar * e2 * two_over_sqrtpi, es6 * (12 * sig6 - 6)) *
                                          ((inv_r * inv_r) * -kFixScale);
                    const double nfx = ndEdRs * dx, nfy = ndEdRs * dy, nfz = ndEdRs * dz;
                    const double dqjs = kqis * inv_r * ec;
                    acc.fx += nfx; acc.fy += nfy; acc.fz += nfz;
                    acc.dq += qj * ec;
                    bad |= !(fmax(fabs(ndEdRs) * a.rc, fabs(dqjs)) < kFixMax * kFixScale);
                    atomicAdd(&accw[0][slot], scaled_to_fix(nfx));
                    atomicAdd(&accw[1][slot], scaled_to_fix(nfy));
                    atomicAdd(&accw[2][slot], scaled_to_fix(nfz));
                    atomicAdd(&accw[3][slot], scaled_to_fix(dqjs));
                }
                acc.e += qq * ec + es6 * (sig6 - 1);   // the whole pair energy: each pair once
            }
            qh = ring(qh + kCqLpi);
            q0 = max(q0 - kCqLpi, 0); q1 = max(q1 - kCqLpi, 0); q2 = max(q2 - kCqLpi, 0); q3 = max(q3 - kCqLpi, 0);
            if (all_ge(kCqLpi)) issue_pf();
        };

        // phase A: a batch of 16 entries = 64 j atoms, one per lane (entry el, atom jl), each tested
        // against the 4 i atoms; the next batch's entries and positions are loaded while this
        // one is tested and its hits queued
        // (an entry past the count -- the next i-cluster's, or the allocation's padding -- is read
        // and its pair mask cleared; every slot of a j-cluster is loaded, the mask decides: pos4f is
        // padded by a cluster's width)
        auto entry = [&](int s) {
            uint2 en = lst[s + el];
            const bool listed = s + el < ne && en.y != 0u;
            // guard: a listed entry's j cluster lies inside the sorted slots and its window cell is
            // one of the 18 (k_cl_build writes no other); an entry past the count reads slot 0
            const bool bad_en = listed && ((en.x & kHalfSlotMask) >= (unsigned)a.n || (en.x >> kHalfSlotBits) >= kHalfWin);
            bad_idx |= bad_en;
            en.x = listed && !bad_en ? en.x : 0u;
            en.y = listed && !bad_en ? en.y : 0u;
            return en;
        };
        auto jpos = [&](uint2 en) { return a.pos4f[(en.x & kHalfSlotMask) + jl]; };
        uint2 en_c = entry(0);
        float4 pj_c = jpos(en_c);
        uint2 en_n = entry(kCqBatch);
        for (int s = 0; s < ne; s += kCqBatch) {
            const float4 pj_n = jpos(en_n);
            const uint2 en_nn = entry(s + 2 * kCqBatch);
            const int wc = en_c.x >> kHalfSlotBits;
            const float4 sh = shf[wc];
            const float xj = pj_c.x + sh.x, yj = pj_c.y + sh.y, zj = pj_c.z + sh.z;
            unsigned long long m[4];
            int cnt[4];
            // two i atoms per packed-fp32 instruction (v_pk_add / v_pk_mul / v_pk_fma_f32)
            const unsigned bits = (en_c.y >> jl) & 0x1111u;   // bit 4k: pair (i atom k, this j) listed
#pragma unroll
            for (int k = 0; k < 4; k += 2) {
                const v2f dx = v2f{pif[k].x, pif[k + 1].x} - v2f{xj, xj};
                const v2f dy = v2f{pif[k].y, pif[k + 1].y} - v2f{yj, yj};
                const v2f dz = v2f{pif[k].z, pif[k + 1].z} - v2f{zj, zj};
                const v2f r2 = dx * dx + dy * dy + dz * dz;
                // two ballots ANDed on the scalar unit (a ballot of `listed && in range` was
                // compiled as compare, s_and, select, compare: two VALU instructions more per atom)
                const bool in0 = r2.x <= a.rcm2f, in1 = r2.y <= a.rcm2f;
                const bool ls0 = (bits >> (4 * k)) & 1u, ls1 = (bits >> (4 * k + 4)) & 1u;
                m[k] = __builtin_amdgcn_ballot_w64(in0) & __builtin_amdgcn_ballot_w64(ls0);
                m[k + 1] = __builtin_amdgcn_ballot_w64(in1) & __builtin_amdgcn_ballot_w64(ls1);
                cnt[k] = __popcll(m[k]);
                cnt[k + 1] = __popcll(m[k + 1]);
            }
            // room for this batch's hits, then queue them
            // any q_k + cnt_k > kCqQ, the four as bytes of one word (sums <= kCqQ + 64 + 127 - kCqQ < 256:
            // no carry between bytes; a byte reaches 128 exactly when its sum exceeds kCqQ) -- scalar ops
            const unsigned cpack = (unsigned)cnt[0] | ((unsigned)cnt[1] << 8) | ((unsigned)cnt[2] << 16) | ((unsigned)cnt[3] << 24);
            auto no_room = [&]() {
                const unsigned qp = (unsigned)q0 | ((unsigned)q1 << 8) | ((unsigned)q2 << 16) | ((unsigned)q3 << 24);
                return ((qp + cpack + (127u - kCqQ) * 0x01010101u) & 0x80808080u) != 0u;
            };
            if (__builtin_expect(no_room(), 0)) {
                do phase_b(); while (no_room());
            }
            const int word = (int)((en_c.x & kHalfSlotMask) + jl) | (wc << kHalfSlotBits) |
                             (__float_as_int(pj_c.w) << kShiftBits);
            const int qs[4] = {q0, q1, q2, q3};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (__builtin_amdgcn_inverse_ballot_w64(m[k])) {   // this lane's bit of m[k]: the mask as exec
                    // ring position qh + q_k + (hits below this lane): mbcnt adds the base
                    const unsigned x = __builtin_amdgcn_mbcnt_hi((unsigned)(m[k] >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((unsigned)m[k], (unsigned)(qh + qs[k])));
                    qbuf[wv][k][ring((int)x)] = word;
                }
            }
            q0 += cnt[0]; q1 += cnt[1]; q2 += cnt[2]; q3 += cnt[3];
            if (!pf_ok && all_ge(kCqLpi)) issue_pf();
            while (all_ge(2 * kCqLpi)) phase_b();   // full steps, one in reserve
            en_c = en_n; pj_c = pj_n; en_n = en_nn;
        }
        while (q0 > 0 || q1 > 0 || q2 > 0 || q3 > 0) phase_b();   // the rest, partly filled
#pragma unroll
        for (int m = 1; m < kCqLpi; m <<= 1) {
            acc.fx += __shfl_xor(acc.fx, m); acc.fy += __shfl_xor(acc.fy, m); acc.fz += __shfl_xor(acc.fz, m);
            acc.dq += __shfl_xor(acc.dq, m); acc.e += __shfl_xor(acc.e, m);
        }
        const int i = a.atom_sorted[islot];
        if (kk == 0 && il < inf.y && i >= a.lo && i < a.hi) {   // this rank's atoms only
            a.e_atom[3 * i + 1] = acc.e;
            if (a.include_forces) {
                a.dedq[i] = acc.dq;
                if constexpr (MIXED) {   // accumulated as -F in 2^13 units
                    a.f_part[3 * i] = acc.fx * -(double)kFix32Inv;
                    a.f_part[3 * i + 1] = acc.fy * -(double)kFix32Inv;
                    a.f_part[3 * i + 2] = acc.fz * -(double)kFix32Inv;
                } else {   // accumulated as -F in fixed-point units
                    a.f_part[3 * i] = acc.fx * -kFixInv;
                    a.f_part[3 * i + 1] = acc.fy * -kFixInv;
                    a.f_part[3 * i + 2] = acc.fz * -kFixInv;
                }
            }
        }
    }
    if (!a.include_forces) return;
    __syncthreads();
    if constexpr (MIXED) {   // 16 B per slot (k_excl reads win_out as uint4 when DirectArgs::win32)
        uint4* out = reinterpret_cast<uint4*>(a.win_out) + (size_t)cell * kHalfMaxWin;
        for (int e = threadIdx.x; e < nw; e += kCqThreads) out[e] = make_uint4(accw[0][e], accw[1][e], accw[2][e], accw[3][e]);
    } else {
        unsigned long long* out = a.win_out + (size_t)cell * kHalfMaxWin * 4;
        for (int e = threadIdx.x; e < nw; e += kCqThreads)
            reinterpret_cast<ulonglong4*>(out)[e] = make_ulonglong4(accw[0][e], accw[1][e], accw[2][e], accw[3][e]);
    }
    };   // process
    process(cell0 + xcd_block());
    {
        const int why = (__ballot(bad_list) ? kHalfListOverflow : 0) | (__ballot(bad) ? kHalfFixedRange : 0);
        if (why && lane == 0) atomicOr(a.half_flag, why);
        if (__ballot(bad_idx) && lane == 0) {
            atomicOr(a.half_flag, kHalfListOverflow);   // the pair sums are incomplete: k_excl rescans
            atomicOr(a.err, kGuardListEntry);
        }
    }
}

// ---------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------
void launch_cluster_table(Handle& h) {
    DirectArgs a = direct_args(h, nullptr, 0);
    const int ncell = h.nc[0] * h.nc[1] * h.nc[2];
    hipLaunchKernelGGL(k_cl_scan, dim3(1), dim3(1024), 0, h.stream, ncell, h.skin_flag, h.cell_start, h.cell_end,
                       h.cl_start, h.ncl_cap, h.err_dev);
    hipLaunchKernelGGL(k_cl_bbox, dim3((ncell + 3) / 4), dim3(256), 0, h.stream, ncell, h.skin_flag, h.cell_start,
                       h.cell_end, h.cl_start, h.pos4f, h.cl_info, h.cl_bb, make_int3(h.nc[0], h.nc[1], h.nc[2]),
                       make_double3(h.box_L[0], h.box_L[1], h.box_L[2]), make_double3(h.box_t[0], h.box_t[1], h.box_t[2]),
                       a.atom_sorted, a.lo, a.hi, a.n, h.ncl_cap);
}

void launch_cluster_list(Handle& h) {
    DirectArgs a = direct_args(h, nullptr, 0);
    const int ncell = h.nc[0] * h.nc[1] * h.nc[2];
    launch_cluster_table(h);
    const double rl = (h.cutoff + h.list_skin) * (1.0 + 1e-5) + 1e-5;
    hipLaunchKernelGGL(k_cl_build, dim3(ncell), dim3(kClBuildThreads), 0, h.stream, a, h.cl_bb, h.cpl, h.cpl_cnt,
                       (float)(rl * rl));
}

void launch_pairs_cluster(Handle& h, const double* pos, int include_forces) {
    DirectArgs a = direct_args(h, pos, include_forces);
    const int ncell = h.nc[0] * h.nc[1] * h.nc[2];
// (any reduced box: the pair vector comes from the window cell's lattice translation, which for a
// pair within rc is the image of the reference's c, b, a minimum image when rc is at most half of
// each perpendicular width -- set_box checks rc <= L/2, and the cells are at least rc + skin wide)
#define CF_PAIRS_CQ(TY_, MX_) hipLaunchKernelGGL((k_pairs_cq<TY_, MX_>), dim3(ncell), dim3(kCqThreads), 0, h.stream, a, 0)
    if (h.mixed) {
        if (a.typ_s) CF_PAIRS_CQ(true, true);
        else CF_PAIRS_CQ(false, true);
    } else {
        if (a.typ_s) CF_PAIRS_CQ(true, false);
        else CF_PAIRS_CQ(false, false);
    }
#undef CF_PAIRS_CQ
}

}  // namespace cf
