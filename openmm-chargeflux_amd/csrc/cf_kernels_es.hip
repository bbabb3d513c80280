// cf_kernels_es.hip -- the octant (eighth-shell) cluster-pair list on one rank.
//
// The real-space erfc + LJ pair loop of RCK:562-593 over the pairs of the reference's voxel-hash
// list (RCK:559: every non-excluded pair with minimum-image r <= rc), each pair once, with both
// sides summed in 64-bit fixed point in an LDS window -- like the 18-cell half list of
// cf_kernels_cluster.hip, but with an 8-cell window:
//
//  * a block owns the octant of its cell c: the 8 cells c + (px, py, pz), p in {0,1}^3 (octant
//    position p = 4 px + 2 py + pz).  A pair of cells within one cell of each other in every axis
//    lies in exactly one octant under the rule "an axis on which both cells agree is the octant's
//    lower layer" (eighth-shell method): the block evaluates the self pair of c and 13 cell pairs,
//    (0, p) for p = 1..7 and the six cross pairs (1,2) (1,4) (1,6) (2,4) (2,5) (3,4);
//  * the window holds the 8 cells' atoms (fx, fy, fz, dE/dq as int64, 2^-34 units): at water
//    density 1 500 atoms = 48 KB, so two 512-thread blocks share a CU, and each atom's sums leave
//    the chip from 8 blocks (es_part[p][slot], 8 x 32 B per atom) instead of 18 windows;
//  * rows: every cluster of the octant's cells 0..3 with the partners its cell pairs with --
//    a cluster of cell 0 (octant position 0) meets ~89 % of its partners in its own octant
//    (long rows, as the 18-cell list's), those of cells 1..3 only an edge or corner (short rows);
//  * the pair loop is k_pairs_cq's: phase A tests 16 entries x 4 j atoms against the row's 4 i
//    atoms in fp32 and queues the hits per i atom, phase B evaluates 16 per i atom in fp64 (the
//    i side in registers, the j side by ds_add_u64 into the window); at the end of a row the i
//    side is summed over its 16 lanes and added to the i atoms' window slots.  Integer adds of
//    per-row sums: the results do not depend on which wave took which row.
#include "cf_pair.h"

namespace cf {

constexpr int kEsWaves = 8;                 // waves per k_pairs_es / k_es_build block
constexpr int kEsThreads = 64 * kEsWaves;
constexpr int kEsQ = 76;                    // queue entries per i atom (ring)
constexpr int kEsBatch = 16;                // list entries tested per phase-A step
constexpr int kEsLpi = 16;                  // phase-B lanes per i atom
constexpr int kEsMaxCand = 1024;            // clusters of one octant staged by k_es_build
constexpr int kEsStage = 384;               // entries of one row staged by the builder (a longer row overflows)
constexpr unsigned kEsSelfMask = 0x08CEu;   // (il, jl) bits il*4 + jl with jl > il
constexpr int kEsPBits = 21;                // entry.x = first slot of j | octant position << 21
typedef float v2f __attribute__((ext_vector_type(2)));

// the p_j a row of octant position p_i pairs with (bit p_j; p_i = 0 also its own cell, j >= i)
__host__ __device__ constexpr unsigned es_allowed(int pi) {
    return pi == 0 ? 0xFFu : pi == 1 ? 0x54u : pi == 2 ? 0x30u : pi == 3 ? 0x10u : 0u;
}

// octant position p of the block whose base cell is (cx, cy, cz): the wrapped cell index, its
// corner offset from the base cell's corner (fp32; the frame of pos4f) and the lattice translation
// that brings its wrapped positions (pos4s) next to the base cell
__device__ __forceinline__ int octant_cell(int p, int cx, int cy, int cz, int3 nc, double3 L, double3 T,
                                           float4& off, double3& wrap) {
    const int o[3] = {p >> 2, (p >> 1) & 1, p & 1};
    const int u[3] = {cx + o[0], cy + o[1], cz + o[2]}, n[3] = {nc.x, nc.y, nc.z};
    int w[3], m[3];
#pragma unroll
    for (int d = 0; d < 3; d++) {
        m[d] = u[d] >= n[d] ? 1 : 0;
        w[d] = u[d] - m[d] * n[d];
    }
    const double3 v = lattice(L, T, (double)o[0] / nc.x, (double)o[1] / nc.y, (double)o[2] / nc.z);
    off = make_float4((float)v.x, (float)v.y, (float)v.z, 0.f);
    wrap = lattice(L, T, m[0], m[1], m[2]);
    return (w[0] * nc.y + w[1]) * nc.z + w[2];
}

// ---------------------------------------------------------------------------------
// list (rebuild only): one block per octant.  The octant's clusters are staged with their boxes
// in the octant frame; each wave takes rows (clusters of positions 0..3) and tests the row's
// partner range 64 candidates at a time: box distance <= rc + skin, the cell pair allowed, then
// the pair mask (exclusions, the lower triangle of the self pair, empty slots cleared).  A row's
// entries are staged in LDS in candidate order (deterministic), then copied to the block's pool at
// an offset taken from a block counter: es_row[block][r] = (offset, count).  A row longer than the
// stage, a full pool or an octant of too many clusters stores an overflowed count, which makes
// k_pairs_es raise the list-overflow fallback on every evaluation that keeps this list.
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(kEsThreads) k_es_build(DirectArgs a, const float4* __restrict__ cl_bb,
                                                         uint2* __restrict__ pool, int2* __restrict__ rows,
                                                         float rlm2) {
    __shared__ float4 cand_lo[kEsMaxCand], cand_hi[kEsMaxCand];   // w: cluster | (count - 1) << 29 / first | p << 21
    __shared__ int cbase[9], clb[8];
    __shared__ float4 offs[8];
    __shared__ int exs[kEsWaves][64];
    __shared__ uint2 stage[kEsWaves][kEsStage];
    __shared__ int pool_used;
    if (!*a.flag) return;
    const int cell = xcd_block();
    const int3 nc = a.nc;
    const int cz = cell % nc.z, cy = (cell / nc.z) % nc.y, cx = cell / (nc.y * nc.z);
    int2* const rrow = rows + (size_t)cell * a.es_rows_max;
    uint2* const rpool = pool + (size_t)cell * a.es_pool_cap;
    if (threadIdx.x < 8) {
        float4 off;
        double3 wr;
        const int w = octant_cell(threadIdx.x, cx, cy, cz, nc, a.L, a.T, off, wr);
        offs[threadIdx.x] = off;
        clb[threadIdx.x] = a.cl_start[w];
        cbase[threadIdx.x] = a.cl_start[w + 1] - a.cl_start[w];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;
        for (int p = 0; p < 8; p++) {
            const int c = cbase[p];
            cbase[p] = s;
            s += c;
        }
        cbase[8] = s;
        pool_used = 0;
    }
    __syncthreads();
    const int ncand = cbase[8], nrows = cbase[4];
    if (ncand > kEsMaxCand || nrows > a.es_rows_max) {   // block-uniform: also beyond k_pairs_es's window
        if (threadIdx.x == 0) atomicOr(a.half_flag, kHalfWindowFull);
        for (int r = threadIdx.x; r < min(nrows, a.es_rows_max); r += kEsThreads) rrow[r] = make_int2(0, -1);
        return;
    }
    for (int t = threadIdx.x; t < ncand; t += kEsThreads) {
        int p = 0;
        while (cbase[p + 1] <= t) p++;
        const int cj = clb[p] + (t - cbase[p]);
        const float4 sh = offs[p];
        const float4 lo = cl_bb[2 * cj], hi = cl_bb[2 * cj + 1];
        const int2 inf = a.cl_info[cj];
        cand_lo[t] = make_float4(lo.x + sh.x, lo.y + sh.y, lo.z + sh.z,
                                 __int_as_float((int)((unsigned)cj | ((unsigned)(inf.y - 1) << 29))));
        cand_hi[t] = make_float4(hi.x + sh.x, hi.y + sh.y, hi.z + sh.z, __int_as_float(inf.x | (p << kEsPBits)));
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int r = wv; r < nrows; r += kEsWaves) {
        const float4 ilo = cand_lo[r], ihi = cand_hi[r];
        const int ci = __float_as_int(ilo.w) & 0x1FFFFFFF;
        const int pi = (__float_as_int(ihi.w) >> kEsPBits) & 7;
        const int2 ii = a.cl_info[ci];
        const unsigned rowbits = (1u << (4 * ii.y)) - 1u;   // bits of the valid i atoms
        const unsigned allow = es_allowed(pi);
        // partner range: position 0 from the row itself on (j >= i in the own cell), 1: 2..6, 2: 4..5, 3: 4
        const int t_lo = pi == 0 ? r : pi == 1 ? cbase[2] : cbase[4];
        const int t_hi = pi == 0 ? ncand : pi == 1 ? cbase[7] : pi == 2 ? cbase[6] : cbase[5];
        // the i atoms' excluded partners as sorted slots (lane il * 16 + e), as k_cl_build
        int nex = 0;
        bool many = false;
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
            const int rk = __popcll(has & ((1ull << lane) - 1ull));
            if (v >= 0) exs[wv][rk] = v;
            nex = __popcll(has);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        int cnt = 0;
        for (int t0 = t_lo; t0 < t_hi; t0 += 64) {
            const int t = t0 + lane;
            bool hit = false;
            unsigned mask = 0;
            int ent = 0;
            if (t < t_hi) {
                const float4 lo = cand_lo[t], hi = cand_hi[t];
                ent = __float_as_int(hi.w);
                const int pj = (ent >> kEsPBits) & 7;
                const float dx = fmaxf(0.f, fmaxf(lo.x - ihi.x, ilo.x - hi.x));
                const float dy = fmaxf(0.f, fmaxf(lo.y - ihi.y, ilo.y - hi.y));
                const float dz = fmaxf(0.f, fmaxf(lo.z - ihi.z, ilo.z - hi.z));
                if (((allow >> pj) & 1u) && dx * dx + dy * dy + dz * dz <= rlm2) {
                    const int cj = __float_as_int(lo.w) & 0x1FFFFFFF;
                    const int jcnt = (((unsigned)__float_as_int(lo.w) >> 29) & 3u) + 1;
                    const unsigned cols = 0x1111u * ((1u << jcnt) - 1u);
                    mask = rowbits & cols & (cj == ci ? kEsSelfMask : 0xFFFFu);
                    hit = true;
                }
            }
            if (!__ballot(hit)) continue;
            const int jfirst = ent & ((1 << kEsPBits) - 1);
            if (!many) {
                for (int x = 0; x < nex; x++) {
                    const int v = exs[wv][x];
                    const int d = (v & 0xFFFFFF) - jfirst;
                    if (hit && d >= 0 && d < 4) mask &= ~(1u << (4 * (v >> 24) + d));
                }
            } else {
                for (int il = 0; il < ii.y; il++) {
                    const int ai = a.atom_sorted[ii.x + il];
                    for (int e = a.ex_start[ai]; e < a.ex_start[ai + 1]; e++) {
                        const int d = a.slot_of[a.ex_list[e]] - jfirst;
                        if (hit && d >= 0 && d < 4) mask &= ~(1u << (4 * il + d));
                    }
                }
            }
            hit = hit && mask != 0;
            const unsigned long long bal = __ballot(hit);
            const int rk = __popcll(bal & ((1ull << lane) - 1ull));
            if (hit && cnt + rk < kEsStage) stage[wv][cnt + rk] = make_uint2((unsigned)ent, mask);
            cnt += __popcll(bal);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int off = 0;
        if (lane == 0 && cnt <= kEsStage && cnt <= a.cpl_cap) off = atomicAdd(&pool_used, cnt);
        off = __builtin_amdgcn_readfirstlane(__shfl(off, 0));
        if (cnt > kEsStage || cnt > a.cpl_cap || off + cnt > a.es_pool_cap) {   // (cpl_cap: cf_options.list_capacity)
            if (lane == 0) rrow[r] = make_int2(0, -1);   // overflowed: k_pairs_es falls back
            continue;
        }
        for (int e = lane; e < cnt; e += 64) rpool[off + e] = stage[wv][e];
        if (lane == 0) rrow[r] = make_int2(off, cnt);
    }
}

// ---------------------------------------------------------------------------------
// k_pairs_es: the pair loop (see the top of this file).  Dynamic LDS: the window, [4][wcap]
// int64.  MIXED (CF_PRECISION_MIXED): phase B in fp32 from the fp64-formed pair vector, as
// k_pairs_cq.
// ---------------------------------------------------------------------------------
template <bool TYPES, bool MIXED>
__global__ void __launch_bounds__(kEsThreads) __attribute__((amdgpu_waves_per_eu(4))) CF_LDS_UNPAIRED k_pairs_es(DirectArgs a, int wcap) {
    extern __shared__ unsigned long long accw_dyn[];
    __shared__ double tab[MIXED ? 1 : kErfcMaxM * (kErfcDeg + 1)];
    __shared__ float tabf[MIXED ? kErfcMaxMF * (kErfcDegF + 1) : 1];
    __shared__ double2 ljt[TYPES ? kMaxLjTypes : 1];
    __shared__ int wdel[8];          // window offset - first sorted slot, per octant position
    __shared__ int wbeg[9];          // window offsets (prefix over the positions)
    __shared__ int cfirst[8];        // first sorted slot of each position's cell
    __shared__ int clb[8], rb[5];    // first cluster per position; row bases of positions 0..3
    __shared__ float4 shf[8];        // corner offsets (phase A)
    __shared__ double3 shd[8];       // wrap translations (phase B)
    __shared__ int qbuf[kEsWaves][4][kEsQ];
    __shared__ int next_row;
    __shared__ unsigned long long eacc;   // the block's pair energy (fixed point)
    unsigned long long* const accx = accw_dyn;
    unsigned long long* const accy = accw_dyn + wcap;
    unsigned long long* const accz = accw_dyn + 2 * wcap;
    unsigned long long* const accq = accw_dyn + 3 * wcap;
    const int cell = xcd_block();
    const int3 nc = a.nc;
    const int cz = cell % nc.z, cy = (cell / nc.z) % nc.y, cx = cell / (nc.y * nc.z);
    if (threadIdx.x < 8) {
        float4 off;
        double3 wr;
        const int w = octant_cell(threadIdx.x, cx, cy, cz, nc, a.L, a.T, off, wr);
        cfirst[threadIdx.x] = a.cstart[w];
        wbeg[threadIdx.x] = a.cend[w] - a.cstart[w];
        clb[threadIdx.x] = a.cl_start[w];
        if (threadIdx.x < 4) rb[threadIdx.x] = a.cl_start[w + 1] - a.cl_start[w];
        shf[threadIdx.x] = off;
        shd[threadIdx.x] = wr;
    }
    if constexpr (TYPES)
        for (int e = threadIdx.x; e < a.lj_ntypes; e += kEsThreads) ljt[e] = a.lj_tab[e];
    if constexpr (MIXED) {
        for (int e = threadIdx.x; e < a.erfc_m_f * (kErfcDegF + 1); e += kEsThreads) tabf[e] = a.erfc_tab_f[e];
    } else {
        for (int e = threadIdx.x; e < kErfcMaxM * (kErfcDeg + 1); e += kEsThreads) tab[e] = a.erfc_tab[e];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;
        for (int p = 0; p < 8; p++) {
            const int c = wbeg[p];
            wbeg[p] = s;
            wdel[p] = s - cfirst[p];
            s += c;
        }
        wbeg[8] = s;
        int r = 0;
        for (int p = 0; p < 4; p++) {
            const int c = rb[p];
            rb[p] = r;
            r += c;
        }
        rb[4] = r;
        next_row = 0;
        eacc = 0;
        if (s > wcap || r > a.es_rows_max) atomicOr(a.half_flag, kHalfWindowFull);
    }
    __syncthreads();
    const int nw = wbeg[8], nrows = rb[4];
    if (nw > wcap || nrows > a.es_rows_max) return;   // block-uniform; k_excl recomputes everything
    for (int e = threadIdx.x; e < nw; e += kEsThreads) {
        accx[e] = 0; accy[e] = 0; accz[e] = 0; accq[e] = 0;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int il = lane >> 4, kk = lane & 15;          // phase B: i atom il, lane kk of its 16
    const int jl = lane & 3, el = lane >> 2;           // phase A: entry el of the batch, j atom jl
    int* const qw = qbuf[wv][il];
    const int2* const rrow = a.es_row + (size_t)cell * a.es_rows_max;
    const uint2* const rpool = a.es_pool + (size_t)cell * a.es_pool_cap;
    bool bad = false, bad_list = false;
    auto ring = [](int x) { return x >= kEsQ ? x - kEsQ : x; };   // x < 2 kEsQ
    for (;;) {
        int r = 0;
        if (lane == 0) r = atomicAdd(&next_row, 1);
        r = __builtin_amdgcn_readfirstlane(__shfl(r, 0));
        if (r >= nrows) break;
        const int pi_ = r < rb[1] ? 0 : r < rb[2] ? 1 : r < rb[3] ? 2 : 3;   // the row's octant position
        const int ci = clb[pi_] + (r - rb[pi_]);
        const int2 inf = a.cl_info[ci];
        const int islot = inf.x + min(il, inf.y - 1);
        const double3 wi = shd[pi_];
        double4 pi = a.pos4s[islot];
        pi.x += wi.x; pi.y += wi.y; pi.z += wi.z;
        const double2 li = TYPES ? ljt[__float_as_int(a.pos4f[islot].w)] : a.ljs[islot];
        const double kqis = a.ke * pi.w * kFixScale;   // k_e q_i in fixed-point units
        float4 pif[4];
        auto sgpr = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
        {
            const float4 so = shf[pi_];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float4 v = a.pos4f[inf.x + min(k, inf.y - 1)];
                pif[k] = make_float4(sgpr(v.x + so.x), sgpr(v.y + so.y), sgpr(v.z + so.z), 0.f);
            }
        }
        const int2 rl = rrow[r];
        int ne = rl.y;
        if (ne < 0) { bad_list = true; ne = 0; }   // the evaluation falls back (k_excl rescans)
        if (ne == 0) continue;                      // (wave-uniform) no partner: nothing to add
        const uint2* lst = rpool + rl.x;
        std::conditional_t<MIXED, PairAccF, PairAcc> acc;
        int q0 = 0, q1 = 0, q2 = 0, q3 = 0;   // queue lengths (wave-uniform)
        int qh = 0;                            // ring head, equal for the 4 queues

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
            const int pj_ = (wq >> kHalfSlotBits) & 7;
            const double3 wr = shd[pj_];
            // the pair vector between the two atoms' images in the octant frame (for a pair within
            // rc < L/2 the image of the reference's minimum image; orthorhombic: the same bits as
            // d - L rint(d / L) up to the exact translations)
            const double ddx = pi.x - (pj.x + wr.x), ddy = pi.y - (pj.y + wr.y), ddz = pi.z - (pj.z + wr.z);
            if constexpr (MIXED) {
                const float qjv = (float)pj.w;
                const float dx = (float)ddx, dy = (float)ddy, dz = (float)ddz;
                const float r2 = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
                if (act && r2 <= (float)a.rc2) {
                    const int slot = wdel[pj_] + j;
                    const double2 ljd = TYPES ? ljt[(unsigned)wq >> kShiftBits] : a.ljs[j];
                    const float ke = (float)a.ke, qi = (float)pi.w;
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
                    const float qj = ke * qjv * inv_r;
                    const float qq = qi * qj;
                    if (a.include_forces) {
                        const float inv_r2 = inv_r * inv_r;
                        const float dEdR = qq * inv_r2 * fmaf(ar * e2, 1.1283791670955126f, ec) +
                                           es6 * (12.0f * sig6 - 6.0f) * inv_r2;
                        const float fx = dEdR * dx, fy = dEdR * dy, fz = dEdR * dz;
                        const float dqj = ke * qi * inv_r * ec;
                        acc.fx += fx; acc.fy += fy; acc.fz += fz;
                        acc.dq = fmaf(qj, ec, acc.dq);
                        bad |= !(fmaxf(fmaxf(fabsf(fx), fabsf(fy)), fmaxf(fabsf(fz), fabsf(dqj))) < (float)kFixMax);
                        atomicAdd(&accx[slot], to_fix(-(double)fx));
                        atomicAdd(&accy[slot], to_fix(-(double)fy));
                        atomicAdd(&accz[slot], to_fix(-(double)fz));
                        atomicAdd(&accq[slot], to_fix((double)dqj));
                    }
                    acc.e += (double)fmaf(qq, ec, es6 * (sig6 - 1.0f));   // the whole pair energy
                }
            } else {
                const double2 lj = TYPES ? ljt[(unsigned)wq >> kShiftBits] : a.ljs[j];
                const double dx = ddx, dy = ddy, dz = ddz;
                const double r2 = dx * dx + dy * dy + dz * dz;
                if (act && r2 <= a.rc2) {   // exact voxel-hash test (RCK:567-569)
                    const int slot = wdel[pj_] + j;
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
                        atomicAdd(&accx[slot], scaled_to_fix(nfx));
                        atomicAdd(&accy[slot], scaled_to_fix(nfy));
                        atomicAdd(&accz[slot], scaled_to_fix(nfz));
                        atomicAdd(&accq[slot], scaled_to_fix(dqjs));
                    }
                    acc.e += qq * ec + es6 * (sig6 - 1);   // the whole pair energy: each pair once
                }
            }
            qh = ring(qh + kEsLpi);
            q0 = max(q0 - kEsLpi, 0); q1 = max(q1 - kEsLpi, 0); q2 = max(q2 - kEsLpi, 0); q3 = max(q3 - kEsLpi, 0);
            if (all_ge(kEsLpi)) issue_pf();
        };

        // phase A (k_pairs_cq): a batch of 16 entries = 64 j atoms against the row's 4 i atoms
        auto entry = [&](int s) { return s + el < ne ? lst[s + el] : make_uint2(0u, 0u); };
        auto jpos = [&](uint2 en) {
            const bool on = (en.y >> jl) & 0x1111u;
            return a.pos4f[on ? (int)(en.x & kHalfSlotMask) + jl : inf.x];
        };
        uint2 en_c = entry(0);
        float4 pj_c = jpos(en_c);
        uint2 en_n = entry(kEsBatch);
        for (int s = 0; s < ne; s += kEsBatch) {
            const float4 pj_n = jpos(en_n);
            const uint2 en_nn = entry(s + 2 * kEsBatch);
            const int pj_ = (en_c.x >> kEsPBits) & 7;
            const float4 sh = shf[pj_];
            const float xj = pj_c.x + sh.x, yj = pj_c.y + sh.y, zj = pj_c.z + sh.z;
            unsigned long long m[4];
            int cnt[4];
            const unsigned bits = (en_c.y >> jl) & 0x1111u;
#pragma unroll
            for (int k = 0; k < 4; k += 2) {
                const v2f dx = v2f{pif[k].x, pif[k + 1].x} - v2f{xj, xj};
                const v2f dy = v2f{pif[k].y, pif[k + 1].y} - v2f{yj, yj};
                const v2f dz = v2f{pif[k].z, pif[k + 1].z} - v2f{zj, zj};
                const v2f r2 = dx * dx + dy * dy + dz * dz;
                m[k] = __ballot(r2.x <= a.rcm2f) & __ballot((bits >> (4 * k)) & 1u);
                m[k + 1] = __ballot(r2.y <= a.rcm2f) & __ballot((bits >> (4 * k + 4)) & 1u);
                cnt[k] = __popcll(m[k]);
                cnt[k + 1] = __popcll(m[k + 1]);
            }
            while (q0 + cnt[0] > kEsQ || q1 + cnt[1] > kEsQ || q2 + cnt[2] > kEsQ || q3 + cnt[3] > kEsQ) phase_b();
            const int word = (int)((en_c.x & kHalfSlotMask) + jl) | (pj_ << kHalfSlotBits) |
                             (__float_as_int(pj_c.w) << kShiftBits);
            const int qs[4] = {q0, q1, q2, q3};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if ((m[k] >> lane) & 1ull) {
                    const int rk = __builtin_amdgcn_mbcnt_hi((unsigned)(m[k] >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m[k], 0u));
                    qbuf[wv][k][ring(qh + qs[k] + rk)] = word;
                }
            }
            q0 += cnt[0]; q1 += cnt[1]; q2 += cnt[2]; q3 += cnt[3];
            if (!pf_ok && all_ge(kEsLpi)) issue_pf();
            while (all_ge(2 * kEsLpi)) phase_b();
            en_c = en_n; pj_c = pj_n; en_n = en_nn;
        }
        while (q0 > 0 || q1 > 0 || q2 > 0 || q3 > 0) phase_b();
        // the i side: summed over the row's 16 lanes, added to the i atoms' window slots
#pragma unroll
        for (int m = 1; m < kEsLpi; m <<= 1) {
            acc.fx += __shfl_xor(acc.fx, m); acc.fy += __shfl_xor(acc.fy, m); acc.fz += __shfl_xor(acc.fz, m);
            acc.dq += __shfl_xor(acc.dq, m); acc.e += __shfl_xor(acc.e, m);
        }
        if (kk < 5 && il < inf.y) {
            const int slot = wdel[pi_] + islot;
            double v;
            if constexpr (MIXED) {
                v = kk == 0 ? (double)acc.fx : kk == 1 ? (double)acc.fy : kk == 2 ? (double)acc.fz
                  : kk == 3 ? (double)acc.dq : acc.e;
                bad |= !(fabs(v) < kFixMax);
                const unsigned long long f = to_fix(v);
                if (kk == 4) atomicAdd(&eacc, f);
                else if (a.include_forces) atomicAdd(&accw_dyn[(size_t)kk * wcap + slot], f);
            } else {   // forces accumulated as -F in fixed-point units
                v = kk == 0 ? -acc.fx : kk == 1 ? -acc.fy : kk == 2 ? -acc.fz : kk == 3 ? acc.dq : acc.e;
                if (kk < 3) {
                    bad |= !(fabs(v) < kFixMax * kFixScale);
                    if (a.include_forces) atomicAdd(&accw_dyn[(size_t)kk * wcap + slot], scaled_to_fix(v));
                } else {
                    bad |= !(fabs(v) < kFixMax);
                    if (kk == 4) atomicAdd(&eacc, to_fix(v));
                    else if (a.include_forces) atomicAdd(&accq[slot], to_fix(v));
                }
            }
        }
    }
    {
        const int why = (__ballot(bad_list) ? kHalfListOverflow : 0) | (__ballot(bad) ? kHalfFixedRange : 0);
        if (why && lane == 0) atomicOr(a.half_flag, why);
    }
    __syncthreads();
    if (threadIdx.x == 0) a.e_blk[cell] = (double)(long long)eacc * kFixInv;
    if (!a.include_forces) return;
    // the window's sums to es_part[p][slot]: each atom's 8 octant partials (k_excl adds them)
    for (int e = threadIdx.x; e < nw; e += kEsThreads) {
        int p = 0;
#pragma unroll
        for (int u = 1; u < 8; u++) p += e >= wbeg[u] ? 1 : 0;
        const int s = e - wdel[p];
        a.es_part[(size_t)p * a.n + s] = make_ulonglong4(accx[e], accy[e], accz[e], accq[e]);
    }
}

// ---------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------
int es_static_lds_bytes(bool mixed, bool types) {
    const size_t tabs = mixed ? (size_t)kErfcMaxMF * (kErfcDegF + 1) * 4 + 8 : (size_t)kErfcMaxM * (kErfcDeg + 1) * 8 + 4;
    return (int)(tabs + (types ? kMaxLjTypes * 16 : 16) + 8 * (4 + 4 + 4 + 16 + 24) + 9 * 4 + 5 * 4 +
                 (size_t)kEsWaves * 4 * kEsQ * 4 + 16 + 64);
}

void launch_es_list(Handle& h) {
    DirectArgs a = direct_args(h, nullptr, 0);
    const int ncell = h.nc[0] * h.nc[1] * h.nc[2];
    // cluster table and boxes: k_cl_scan / k_cl_bbox of the 18-cell list (cf_kernels_cluster.hip)
    launch_cluster_table(h);
    const double rl = (h.cutoff + h.list_skin) * (1.0 + 1e-5) + 1e-5;
    hipLaunchKernelGGL(k_es_build, dim3(ncell), dim3(kEsThreads), 0, h.stream, a, h.cl_bb, h.es_pool, h.es_row,
                       (float)(rl * rl));
}

void launch_pairs_es(Handle& h, const double* pos, int include_forces) {
    DirectArgs a = direct_args(h, pos, include_forces);
    const int ncell = h.nc[0] * h.nc[1] * h.nc[2];
    const size_t dyn = (size_t)32 * h.es_wcap;
#define CF_PAIRS_ES(TY_, MX_) hipLaunchKernelGGL((k_pairs_es<TY_, MX_>), dim3(ncell), dim3(kEsThreads), dyn, h.stream, a, h.es_wcap)
    if (h.mixed) {
        if (a.typ_s) CF_PAIRS_ES(true, true);
        else CF_PAIRS_ES(false, true);
    } else {
        if (a.typ_s) CF_PAIRS_ES(true, false);
        else CF_PAIRS_ES(false, false);
    }
#undef CF_PAIRS_ES
}

// dynamic LDS above the 64-KB default: set once per process for the four instantiations
void es_set_lds_limit(int bytes) {
    check_hip(hipFuncSetAttribute((const void*)k_pairs_es<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes), "es lds");
    check_hip(hipFuncSetAttribute((const void*)k_pairs_es<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes), "es lds");
    check_hip(hipFuncSetAttribute((const void*)k_pairs_es<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes), "es lds");
    check_hip(hipFuncSetAttribute((const void*)k_pairs_es<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes), "es lds");
}

}  // namespace cf
