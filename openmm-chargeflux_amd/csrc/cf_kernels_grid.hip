// cf_kernels_grid.hip — reciprocal-space Ewald sum on a grid (kspace_algo = 2).
//
// Reference: the half-space k loop of ReferenceCoulKernels.cpp:513-556 (RCK), O(N*K)
// with cos/sin twice per (atom, k).  The same truncated k-sum (identical k-set,
// weights and box) is evaluated here as a type-1 / type-2 non-uniform DFT pair with an
// exponential-of-semicircle (ES) kernel of width W on an oversampled grid:
//
//   b[g]   = sum_j q_j phi(g - s_j)                    spread        (N W^3)
//   B(n)   = sum_g b[g] e^{+i 2pi n.g/ng}             pruned DFT, |n_a| < K_a
//   S(n)   = B(n) / (phih_x phih_y phih_z)(n)           = sum_j q_j e^{i k.r_j}  (to ~1e-13)
//   E      = 1/2 sum_{n != 0} c a_k |S(n)|^2            (RCK:549-551, half space doubled)
//   f(n)   = c a_k conj(S(n)) / phih(n)                 (RCK:528, 546)
//   G[g]   = sum_n f(n) e^{+i 2pi n.g/ng}              pruned inverse DFT
//   dE/dq_j = sum_g G[g] phi(g - s_j),   F_j = -q_j grad_j (same sum)   interpolation
//
// s_j = ng * frac(x_j / L) (grid units), phi(t) = exp(beta (sqrt(1 - (2t/W)^2) - 1)).
// The error is set by W and the oversampling ng/(2K-1) (tools/nufft_proto.py: W = 14,
// ng ~ 2(2K-1) -> |dF| ~ 5e-9 kJ/mol/nm at C2 and 12k atoms).  Every sum is a gather in a
// fixed order (atoms are sorted by grid tile each evaluation with a deterministic counting
// sort), so results are bitwise reproducible.  All fp64.
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <utility>
#include <vector>

#include "cf_internal.h"

namespace cf {

static inline int nblk(int64_t n, int b) { return (int)((n + b - 1) / b); }

// native 2-vector for register staging (HIP's double2 struct arrays stay in scratch memory)
typedef double v2d __attribute__((ext_vector_type(2)));
typedef float v2f __attribute__((ext_vector_type(2)));   // packed fp32 (v_pk_fma_f32)

// wave index within the workgroup as a wave-uniform (SGPR) value, so that everything
// derived from it is scalar (the compiler treats threadIdx.x >> 6 as divergent)
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// phi(t) and d/ds phi(g - s) (= -phi'(t)) at t = g - s; zero outside the open support.
// sqrt(u) = u * rsqrt(u) and z / sqrt(u) = z * rsqrt(u) from one v_rsq_f64 + Newton step
// (relative 4e-15), exp of the non-positive exponent by exp_nonpos: no sqrt, divide or libm
// exp on the per-atom path.
__device__ __forceinline__ void es_tap(double t, double hw_inv, double beta, double& v, double& dv) {
    const double z = t * hw_inv;
    const double u = 1.0 - z * z;
    if (u > 0.0) {
        const double rs = rsqrt_fp64(u);
        v = exp_nonpos(beta * (u * rs - 1.0));
        dv = v * beta * z * rs * hw_inv;
    } else {
        v = 0.0;
        dv = 0.0;
    }
}

__device__ __forceinline__ double es_val(double t, double hw_inv, double beta) {
    const double z = t * hw_inv;
    const double u = 1.0 - z * z;
    return u > 0.0 ? exp_nonpos(beta * (u * rsqrt_fp64(u) - 1.0)) : 0.0;
}

// Mixed precision (CF_PRECISION_MIXED): the same taps in fp32 -- v_rsq_f32 and v_exp_f32 instead of
// the fp64 Newton step and exp polynomial (~45 fp64 VALU slots per tap against ~10).  t = g - s
// is formed in fp64 (s is a grid coordinate up to ng) and only then rounded, and the exponent
// beta (sqrt(u) - 1) is taken as -beta z^2 / (1 + sqrt(u)): the difference form cancels near the
// centre (u -> 1), where its absolute error beta * 6e-8 ~ 1e-6 biased every tap the same way
// (C5: the reciprocal energy moved by -0.97 kJ/mol, r6v); this form's error is ~1e-7 relative
// to the exponent.  Below the W <= 8 grid's own ~1e-6 (the mixed bars: tests/test_gpu_configs.py).
__device__ __forceinline__ float es_arg_f(float z, float u, float rs, float b) {
    return -b * (z * z) * __frcp_rn(1.0f + u * rs);
}

__device__ __forceinline__ void es_tap_f(double t, double hw_inv, double beta, double& v, double& dv) {
    const float z = (float)(t * hw_inv);
    const float u = 1.0f - z * z;
    if (u > 0.0f) {
        const float rs = __frsqrt_rn(u);
        const float b = (float)beta;
        const float vf = __expf(es_arg_f(z, u, rs, b));
        v = vf;
        dv = vf * b * z * rs * (float)hw_inv;
    } else {
        v = 0.0;
        dv = 0.0;
    }
}

__device__ __forceinline__ double es_val_f(double t, double hw_inv, double beta) {
    const float z = (float)(t * hw_inv);
    const float u = 1.0f - z * z;
    return u > 0.0f ? (double)__expf(es_arg_f(z, u, __frsqrt_rn(u), (float)beta)) : 0.0;
}

// ---------------------------------------------------------------------------------
// Multi-rank x-slab: on a rank that owns a spatially compact set of atoms, only the grid
// x-planes its atoms' taps reach carry data.  xr[0..1] = min / max over owned atoms of the
// first x tap relative to xr[2] (the first owned atom's first tap, folded into
// [-ng/2, ng/2)), accumulated by k_g_bin with atomics (order-independent) and reset by
// k_energy.  Planes outside [xr[2] + xr[0], xr[2] + xr[1] + W) (mod ng) are skipped by the
// spread, both DFT passes and are never read by the interpolation.  xr == null: all planes.
// ---------------------------------------------------------------------------------
// slab as (first plane in [0, ngx), number of planes); len >= ngx means every plane
__device__ __forceinline__ void slab_of(const int* __restrict__ xr, int W, int ngx, int& s0, int& len) {
    len = xr[1] - xr[0] + W;
    s0 = (xr[2] + xr[0]) % ngx;
    s0 += s0 < 0 ? ngx : 0;
}

__device__ __forceinline__ bool x_in_slab(int x, const int* __restrict__ xr, int W, int ngx) {
    if (!xr) return true;
    const int len = xr[1] - xr[0] + W;
    if (len >= ngx) return true;
    int d = (x - (xr[2] + xr[0])) % ngx;
    d += d < 0 ? ngx : 0;
    return d < len;
}

__device__ __forceinline__ bool x_range_in_slab(int x0, int x1, const int* __restrict__ xr, int W, int ngx) {
    if (!xr) return true;
    for (int x = x0; x <= x1; x++)
        if (x_in_slab(x, xr, W, ngx)) return true;
    return false;
}

// ---------------------------------------------------------------------------------
// 1. bin owned atoms by the 8^3 grid tile holding their first tap; deterministic counting
//    sort: k_g_bin (wave-aggregated atomic provisional rank; the block that finishes last
//    turns the counts into bin bounds), k_g_scatter, then k_g_order_taps fixes the order of
//    a stable sort by atom index and writes each sorted atom's tap rows
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_g_bin(int lo, int nown, const double* __restrict__ pos,
                                               const double* __restrict__ q, double3 L, int3 ng, int W, int3 nb,
                                               double4* __restrict__ srec, int4* __restrict__ g0u,
                                               int* __restrict__ rank, int* __restrict__ cnt, int* __restrict__ xr,
                                               int* __restrict__ ticket, int* __restrict__ start, int per,
                                               int* __restrict__ err) {
    __shared__ int sh[256];
    __shared__ int xs[2][4];
    // several ranks: this thread's x-slab extremes over its rounds, reduced per block and written
    // to the block's own slot of xr; the last block reduces the slots (two same-address atomics
    // from every wave serialized at one L2 channel; k_g_bin took 17 us at W = 8 for 12k atoms, r06ax)
    int bmin = INT_MAX, bmax = INT_MIN;
    // `per` rounds of 256 atoms per block: the ticket of last_block_done is one address that
    // every block increments, so fewer, longer blocks at large N (launch_grid_sort)
    for (int it = 0; it < per; it++) {
    const int io = (blockIdx.x * per + it) * blockDim.x + threadIdx.x;
    const bool valid = io < nown;
    if (xr) {   // x-slab of the owned atoms' first taps, relative to the first owned atom's
        double u0 = pos[3 * lo] / L.x;
        u0 -= floor(u0);
        double s0 = u0 * ng.x;
        if (s0 >= ng.x) s0 -= ng.x;
        const int gref = (int)ceil(s0 - 0.5 * W);
        if (valid) {
            double u = pos[3 * (lo + io)] / L.x;
            u -= floor(u);
            double sd = u * ng.x;
            if (sd >= ng.x) sd -= ng.x;
            int rel = ((int)ceil(sd - 0.5 * W) - gref) % ng.x;
            rel += rel < 0 ? ng.x : 0;
            rel -= rel >= ng.x / 2 ? ng.x : 0;
            bmin = min(bmin, rel);
            bmax = max(bmax, rel);
        }
        if (io == 0) xr[2] = gref;
    }
    int bin = 0;
    if (valid) {
        const int i = lo + io;
        const double x[3] = {pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]};
        const double Ls[3] = {L.x, L.y, L.z};
        const int n[3] = {ng.x, ng.y, ng.z};
        double s[3];
        int g[3], gw[3];
#pragma unroll
        for (int d = 0; d < 3; d++) {
            double u = x[d] / Ls[d];
            u -= floor(u);
            double sd = u * n[d];
            if (sd >= n[d]) sd -= n[d];
            s[d] = sd;
            g[d] = (int)ceil(sd - 0.5 * W);
            gw[d] = g[d] < 0 ? g[d] + n[d] : g[d];
        }
        bin = ((gw[0] >> 3) * nb.y + (gw[1] >> 3)) * nb.z + (gw[2] >> 3);
        srec[io] = make_double4(s[0], s[1], s[2], q[i]);
        g0u[io] = make_int4(g[0], g[1], g[2], bin);
    }
    const int r = wave_agg_inc(cnt, bin, valid);
    if (valid) rank[io] = r;
    }
    const int wv = threadIdx.x >> 6;
    auto block_minmax = [&](int& mn, int& mx) {   // over the block's 4 waves, into every thread
        for (int off = 32; off > 0; off >>= 1) {
            mn = min(mn, __shfl_xor(mn, off));
            mx = max(mx, __shfl_xor(mx, off));
        }
        if ((threadIdx.x & 63) == 0) { xs[0][wv] = mn; xs[1][wv] = mx; }
        __syncthreads();
        mn = min(min(xs[0][0], xs[0][1]), min(xs[0][2], xs[0][3]));
        mx = max(max(xs[1][0], xs[1][1]), max(xs[1][2], xs[1][3]));
    };
    if (xr) {   // (block-uniform)
        block_minmax(bmin, bmax);
        if (threadIdx.x == 0) { st_agent(xr + 3 + 2 * blockIdx.x, bmin); st_agent(xr + 4 + 2 * blockIdx.x, bmax); }
    }
    if (!last_block_done(ticket)) return;
    if (xr) {
        int mn = INT_MAX, mx = INT_MIN;
        for (int b = threadIdx.x; b < (int)gridDim.x; b += blockDim.x) {
            mn = min(mn, ld_agent(xr + 3 + 2 * b));
            mx = max(mx, ld_agent(xr + 4 + 2 * b));
        }
        __syncthreads();   // (xs is reused)
        block_minmax(mn, mx);
        if (threadIdx.x == 0) { xr[0] = mn; xr[1] = mx; }   // read by the later kernels of the chain
    }
    const int nbins = nb.x * nb.y * nb.z;
    const int total = block_counts_to_bounds<256>(nbins, cnt, start, nullptr, true, sh);
    // guard: the counts add up to the owned atoms (k_g_scatter re-zeroes them each evaluation);
    // bounds that do not are replaced by empty bins, so no spread, tap or interpolation kernel
    // indexes past the owned atoms (the scan's total, block-uniform: no read-back of start[nbins]
    // on the critical path)
    if (total != nown) {
        __syncthreads();   // every thread's bounds stores before they are overwritten
        for (int b = threadIdx.x; b <= nbins; b += blockDim.x) start[b] = 0;
        if (threadIdx.x == 0) atomicOr(err, kGuardGridBins);
    }
}

// also re-zeroes the bin counts (consumed by k_g_bin's bounds) for the next evaluation
__global__ void __launch_bounds__(256) k_g_scatter(int nown, const int4* __restrict__ g0u, const int* __restrict__ rank,
                                                   const int* __restrict__ start, int* __restrict__ tmp, int nbins,
                                                   int* __restrict__ cnt, int* __restrict__ err) {
    const int io = blockIdx.x * blockDim.x + threadIdx.x;
    for (int b = io; b < nbins; b += gridDim.x * blockDim.x) cnt[b] = 0;
    if (io >= nown) return;
    const int bin = g0u[io].w, s = (unsigned)bin < (unsigned)nbins ? start[bin] + rank[io] : -1;
    if ((unsigned)s >= (unsigned)nown) { atomicOr(err, kGuardGridBins); return; }   // guard
    tmp[s] = io;
}

// taps of every sorted atom in bin-aligned rows: taps[slot][d][p], p in [0, 24), is the
// kernel weight of grid point 8*bin_d + p (tap m = p - (g0_d mod 8); zero outside 0 <= m < W),
// q folded into the x row.  A tile db tiles ahead of the atom's bin then reads the fixed
// window p = 8*db + i, so no per-atom offset is needed to address the taps.
constexpr int kRow = 24;
constexpr int kTapStride = 3 * kRow;
constexpr int kRowF32 = 16;                 // fp32 rows (GridPlan::taps_f32, W <= 9): points 0..15
constexpr int kTapStrideF32 = 3 * kRowF32;  // floats per atom
constexpr int kOtWaves = 4;     // bins per 256-thread block: one wave per bin, no block barriers
constexpr int kOtLds = 128;     // members per bin staged in LDS (denser bins read global memory)
constexpr int kOtChunk = 8;     // atoms whose tap rows are assembled in LDS at a time (16, 24 slower)

// LDS written by some lanes of a wave, then read by others of the same wave
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// one wave per bin (a bin holds ~23 atoms at C3: a 256-thread block per bin left most of its
// lanes idle and serialised two block barriers per bin).  Slot of each member = bin start +
// number of members with a smaller atom index (the order of a stable sort).  The tap rows of
// kOtChunk members at a time: one lane per nonzero tap (atom, axis, tap m) -- exactly W
// evaluations per row, where a lane per 16-B pair of the 24-point row evaluated both points
// whenever either was nonzero -- written into a zeroed LDS copy of the rows, which the wave
// then stores to the bin's contiguous slot range in consecutive 16 B per lane.
// WT > 0: the kernel width as a compile-time constant (the tap index divisions become
// multiplies; 14 = the fp64 default, 8 = mixed precision); WT = 0: W at run time.  F32: the taps
// evaluated in fp32 (mixed precision, es_val_f) and, when W <= 9 (GridPlan::taps_f32), stored as
// fp32 rows of 16 points (taps then holds floats: [slot][3][16])
template <int WT, bool F32 = false>
__global__ void __launch_bounds__(256) k_g_order_taps(int nbins, const int* __restrict__ start,
                                                      const int* __restrict__ tmp, int* __restrict__ order, int Wr,
                                                      double beta, int3 ng, const double4* __restrict__ srec,
                                                      const int4* __restrict__ g0u, double* __restrict__ taps,
                                                      int4* __restrict__ g0s, int nown, int* __restrict__ err) {
    __shared__ int mem[kOtWaves][kOtLds];
    __shared__ int srt[kOtWaves][kOtLds];
    __shared__ double4 srl[kOtWaves][64];   // sorted members' srec / g0u (bins of <= 64 members)
    __shared__ int4 gl[kOtWaves][64];
    __shared__ __attribute__((aligned(16))) double rows[kOtWaves][kOtChunk * kTapStride];
    constexpr int kPairs = kTapStride / 2;   // 36
    const int W = WT > 0 ? WT : Wr;
    const int w = wave_id(), lane = threadIdx.x & 63;
    const int b = blockIdx.x * kOtWaves + w;
    if (b >= nbins) return;   // wave-uniform
    const int b0 = start[b], m = start[b + 1] - b0;
    if (m == 0) return;
    if (b0 < 0 || m < 0 || b0 + m > nown) {   // guard (k_g_bin's bounds hold by construction)
        if (lane == 0) atomicOr(err, kGuardGridBins);
        return;
    }
    const int* src = tmp + b0;
    const bool fast = m <= 64, in_lds = m <= kOtLds;
    if (fast) {   // members in registers: rank by wave-uniform lane reads, their srec / g0u
                  // loads in flight meanwhile, then kept in LDS in slot order
        const int v = lane < m ? src[lane] : INT_MAX;
        double4 sr = make_double4(0.0, 0.0, 0.0, 0.0);
        int4 g = make_int4(0, 0, 0, 0);
        if (lane < m) {
            sr = srec[v];
            g = g0u[v];
        }
        int r = 0;
        for (int j = 0; j < m; j++) r += __builtin_amdgcn_readlane(v, j) < v;
        if (lane < m) {
            order[b0 + r] = v;
            srl[w][r] = sr;
            gl[w][r] = g;
            g0s[b0 + r] = make_int4(g.x < 0 ? g.x + ng.x : g.x, g.y < 0 ? g.y + ng.y : g.y,
                                    g.z < 0 ? g.z + ng.z : g.z, v);
        }
    } else {
        if (in_lds) {
            for (int e = lane; e < m; e += 64) mem[w][e] = src[e];
            wave_sync();
            src = mem[w];
        }
        for (int e = lane; e < m; e += 64) {
            const int v = src[e];
            int r = 0;
            for (int j = 0; j < m; j++) r += src[j] < v;
            order[b0 + r] = v;
            if (in_lds) srt[w][r] = v;
        }
        if (!in_lds) __threadfence();   // order[] stores of other lanes, read back below
    }
    wave_sync();
    const int* so = in_lds ? srt[w] : order + b0;
    double* rw = rows[w];
    const int per = 3 * W;
    const double hw_inv = 2.0 / W;
    for (int c0 = 0; c0 < m; c0 += kOtChunk) {
        const int mc = min(kOtChunk, m - c0);
        for (int e = lane; e < mc * kPairs; e += 64) reinterpret_cast<v2d*>(rw)[e] = v2d{0.0, 0.0};
        wave_sync();
        for (int e = lane; e < mc * per; e += 64) {
            const int u = e / per, rem = e - u * per, d = rem / W, mm = rem - d * W;
            double sd, scale;
            int g0;
            if (fast) {
                const double* sp = reinterpret_cast<const double*>(&srl[w][c0 + u]);
                const int* gp = reinterpret_cast<const int*>(&gl[w][c0 + u]);
                sd = sp[d];
                scale = d == 0 ? sp[3] : 1.0;
                g0 = gp[d];
            } else {
                const int io = so[c0 + u];
                const double* sp = reinterpret_cast<const double*>(srec + io);
                const int* gp = reinterpret_cast<const int*>(g0u + io);
                sd = sp[d];
                scale = d == 0 ? sp[3] : 1.0;
                g0 = gp[d];
            }
            // q folded into the x row; bin-aligned point (g0 mod 8) + m, g0 mod 8 == wrapped
            // g0 mod 8 (ng is a multiple of 8)
            const double t = (double)(g0 + mm) - sd;
            rw[u * kTapStride + d * kRow + (g0 & 7) + mm] = scale * (F32 ? es_val_f(t, hw_inv, beta) : es_val(t, hw_inv, beta));
        }
        wave_sync();
        const size_t s0 = (size_t)b0 + c0;
        if (F32 && W <= 9) {   // fp32 rows of 16 points (kRowF32), 48 floats per atom: 4 floats per lane
            for (int e = lane; e < mc * 12; e += 64) {
                const int ad = e >> 2, qd = e & 3;   // (atom, axis), quarter of the 16 points
                const double* r = rw + (ad / 3) * kTapStride + (ad % 3) * kRow + 4 * qd;
                reinterpret_cast<float4*>(taps)[s0 * 12 + e] = make_float4((float)r[0], (float)r[1], (float)r[2], (float)r[3]);
            }
        } else if (W <= 9) {   // taps end at point (g0 mod 8) + W - 1 <= 15: points 16..23 stay the zeros
                        // written at allocation (cf_create), so a row is 8 pairs of its 12
            for (int e = lane; e < mc * 24; e += 64) {
                const int pr = (e / 8) * 12 + (e & 7);   // (atom, axis) = e / 8
                reinterpret_cast<v2d*>(taps)[s0 * kPairs + pr] = reinterpret_cast<const v2d*>(rw)[pr];
            }
        } else {
            for (int e = lane; e < mc * kPairs; e += 64)
                reinterpret_cast<v2d*>(taps)[s0 * kPairs + e] = reinterpret_cast<const v2d*>(rw)[e];
        }
        if (!fast && lane < mc) {
            const int io = so[c0 + lane];
            const int4 g = g0u[io];
            g0s[s0 + lane] = make_int4(g.x < 0 ? g.x + ng.x : g.x, g.y < 0 ? g.y + ng.y : g.y,
                                       g.z < 0 ? g.z + ng.z : g.z, io);
        }
        wave_sync();   // the rows are re-zeroed for the next chunk
    }
}

// ---------------------------------------------------------------------------------
// 2. spread (a gather per 8^3 grid tile)
// ---------------------------------------------------------------------------------
__device__ __forceinline__ int wrapb(int b, int n) { return b < 0 ? b + n : (b >= n ? b - n : b); }

// One 256-thread workgroup per 8^3 tile.  The tile's source atoms
//     (first tap in one of the NS^3 bins 0..NS-1 tiles behind it) are walked in passes of 64;
//     each pass stages, per atom, only the three 8-tap windows this tile reads (the bin-aligned
//     rows make a window a fixed 64-B piece: 192 B per atom instead of the 576-B row set), and
//     the 4 waves take every 4th atom of the pass: lane (y, z) accumulates the tile's 8 x
//     points of its (y, z) column (1 mul + 8 FMAs per atom; the x window is a broadcast LDS
//     read).  Every wave is busy in every pass (a 2x2x2-tile workgroup, round 1, left the waves
//     whose tile a pass's source column does not reach waiting at the pass barrier), and the
//     small blocks (25 KB LDS, <= 64 VGPRs) keep ~6 per CU resident, so a pass's load latency
//     hides behind other blocks.  The 4 waves' partial tiles are summed in fixed order.
constexpr int kSpWin = 24;         // doubles staged per atom: x, y, z windows of 8
constexpr int kSpMaxSrc = 1024;    // source atoms whose slots are resolved per segment

// acc[i] = fma(x_i, yz, acc[i]), i < 8, where x_i is the value lane i of this lane's 16-lane row
// holds in xv (v_fmac_f64 with a 64-bit DPP row_newbcast:i source; the s_nop gives the DPP
// source the wait states it needs after a VALU write)
__device__ __forceinline__ void fma8_row_bcast(double (&acc)[8], double xv, double yz) {
    asm("s_nop 1\n\t"
        "v_fmac_f64_dpp %0, %8, %9 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %6, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %7, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf"
        : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]),
          "+v"(acc[7])
        : "v"(xv), "v"(yz));
}

// TF: fp32 tap rows (GridPlan::taps_f32, NS = 2): a 16-B piece is half a window (4 floats), widened
// to fp64 as it is staged; the sums stay fp64
template <int NS, int kSpPass, bool TF = false, bool GF = false, bool FA = false>
__global__ void __launch_bounds__(256) CF_LDS_UNPAIRED k_g_spread_tile(int3 ng, int3 nb, const int* __restrict__ start,
                                                       const double* __restrict__ taps, const int4* __restrict__ g0s,
                                                       double* __restrict__ grid, const int* __restrict__ xr, int W) {
    // GF: the grid is fp32 (GridPlan::grid_f32): each point's fp64 sum rounded once as it is stored.
    // FA (mixed precision, with TF and GF): the windows staged as fp32 and the per-wave sums in fp32,
    // eight packed FMAs' worth in four v_pk_fma_f32 per (atom, lane) with the x window read as two
    // broadcast 16-B LDS loads (the fp64 form: eight DPP row-broadcast FMAs); the 4 waves' partial
    // tiles are added in fp64 in a fixed order.  Each grid point sums ~20 contributions at C5:
    // fp32 rounding ~1e-7 relative, under the mixed grid's own error.
    static_assert(!TF || NS == 2, "fp32 rows hold points 0..15: windows db = 0, 1");
    static_assert(!FA || (TF && GF), "fp32 arithmetic on the fp32 rows and grid only");
    constexpr int NB3 = NS * NS * NS;
    static_assert(NS <= 3, "tile offsets are packed in 2 bits per axis");
    constexpr int kStD = 2 * kSpPass * kSpWin > 4 * 8 * 64 ? 2 * kSpPass * kSpWin : 4 * 8 * 64;
    __shared__ __attribute__((aligned(16))) double st[kStD];   // 2 staging buffers; reused by the reduction
    __shared__ int bin_start[NB3], bin_pre[NB3 + 1], bin_db[NB3];
    __shared__ int src[kSpMaxSrc];   // slot << 6 | (dx, dy, dz) 2 bits each, of the segment's atoms that reach this tile
    __shared__ int wcnt[4 * (kSpMaxSrc / 256)];
    // XCD-aware tile order (as in k_g_interp)
    const int nyz = nb.y * nb.z;
    int tile = blockIdx.x;
    if (nyz % 8 == 0) {
        const int per = nyz / 8, i = blockIdx.x / 8;
        tile = (i / per) * nyz + (blockIdx.x % 8) * per + i % per;
    }
    const int tz = tile % nb.z, ty = (tile / nb.z) % nb.y, tx = tile / (nb.z * nb.y);
    if (!x_range_in_slab(8 * tx, 8 * tx + 7, xr, W, ng.x)) return;
    const int t = threadIdx.x;
    if (t < NB3) {
        const int dx = t / (NS * NS), dy = (t / NS) % NS, dz = t % NS;   // tiles behind this one
        const int b = (wrapb(tx - dx, nb.x) * nb.y + wrapb(ty - dy, nb.y)) * nb.z + wrapb(tz - dz, nb.z);
        const int s0 = start[b];
        bin_start[t] = s0;
        bin_pre[t + 1] = start[b + 1] - s0;   // counts, scanned below
        bin_db[t] = (dx << 8) | (dy << 4) | dz;
    }
    __syncthreads();
    if (t == 0) {
        bin_pre[0] = 0;
        for (int i = 0; i < NB3; i++) bin_pre[i + 1] += bin_pre[i];
    }
    __syncthreads();
    const int total = bin_pre[NB3];
    const int lane = t & 63, w = wave_id();
    const int y = lane >> 3;   // this lane's (y, z) column: y = lane >> 3, z = lane & 7
    double acc[8];
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = 0.0;
    v2f accf[4] = {v2f{0.f, 0.f}, v2f{0.f, 0.f}, v2f{0.f, 0.f}, v2f{0.f, 0.f}};   // (FA: x = 2k, 2k + 1)
    for (int seg0 = 0; seg0 < total; seg0 += kSpMaxSrc) {
        const int nall = min(kSpMaxSrc, total - seg0);
        __syncthreads();   // previous segment's passes done with src
        // resolve (slot, bin) of each source atom and keep, in source order, those whose support
        // reaches this tile: a window db tiles ahead ([8 db, 8 db + 8) of the bin-aligned row) is
        // all zero when the taps [r, r + W) end before it (r = first tap mod 8) -- about a third
        // of the (tile, atom) pairs at W = 14
        constexpr int kRounds = kSpMaxSrc / 256;
        int2 sb[kRounds];
        int4 g[kRounds];
#pragma unroll
        for (int k = 0; k < kRounds; k++) {   // every source's slot, then every g0s load in flight at once
            const int u = 256 * k + t;
            sb[k] = make_int2(0, 0);
            if (u < nall) {
                const int a = seg0 + u;
                int lo = 0, hi = NB3;   // bin i with bin_pre[i] <= a < bin_pre[i + 1]
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (bin_pre[mid] <= a) lo = mid; else hi = mid;
                }
                sb[k] = make_int2(bin_start[lo] + (a - bin_pre[lo]), lo);
            }
        }
#pragma unroll
        for (int k = 0; k < kRounds; k++) g[k] = 256 * k + t < nall ? g0s[sb[k].x] : make_int4(0, 0, 0, 0);
        bool keep[kRounds];
        unsigned long long m[kRounds];
        int dbits[kRounds];   // the source bin's tile offsets, 2 bits per axis (NS <= 3)
#pragma unroll
        for (int k = 0; k < kRounds; k++) {
            const int db = bin_db[sb[k].y];
            dbits[k] = ((db >> 4) & 0x30) | ((db >> 2) & 0xC) | (db & 3);
            keep[k] = 256 * k + t < nall && (g[k].x & 7) + W > 8 * (db >> 8) &&
                      (g[k].y & 7) + W > 8 * ((db >> 4) & 15) && (g[k].z & 7) + W > 8 * (db & 15);
            m[k] = __ballot(keep[k]);
            if ((t & 63) == 0) wcnt[4 * k + (t >> 6)] = __popcll(m[k]);
        }
        __syncthreads();
        int nseg = 0;
#pragma unroll
        for (int k = 0; k < kRounds; k++) {   // kept sources in source order: (round, wave, lane)
            int off = nseg;
            for (int q = 0; q < (t >> 6); q++) off += wcnt[4 * k + q];
            if (keep[k]) src[off + __popcll(m[k] & ((1ull << (t & 63)) - 1))] = (sb[k].x << 6) | dbits[k];
            nseg += wcnt[4 * k] + wcnt[4 * k + 1] + wcnt[4 * k + 2] + wcnt[4 * k + 3];
        }
        __syncthreads();
        if (nseg == 0) continue;
        // staging: 16-B piece e of the pass = atom e / 12, axis (e % 12) / 4, quarter e % 4 of the window
        // (TF: atom e / 6, axis (e % 6) / 2, half e % 2 of the window: 4 floats, staged as 4 doubles)
        constexpr int kPP = TF ? kSpWin / 4 : kSpWin / 2;      // pieces per atom
        constexpr int kPieces = kSpPass * kPP;                  // 768 at 64 atoms per pass (TF: 384)
        constexpr int kPer = (kPieces + 255) / 256;             // 3 per thread at 64 (TF: 2)
        using Piece = std::conditional_t<TF, float4, v2d>;
        Piece r[kPer];
        auto fetch = [&](int base, int n) {
#pragma unroll
            for (int q = 0; q < kPer; q++) {
                const int e = min(t + 256 * q, kPieces - 1);
                const int a = e / kPP, c = e - kPP * a;
                const int u = base + min(a, n - 1);
                const int sb = src[u];
                if constexpr (TF) {
                    const int d = c >> 1, h = c & 1;
                    const int db = (sb >> (4 - 2 * d)) & 3;
                    const float* tf = reinterpret_cast<const float*>(taps);
                    r[q] = *reinterpret_cast<const float4*>(tf + (sb >> 6) * kTapStrideF32 + d * kRowF32 + 8 * db + 4 * h);
                    if (a >= n) r[q] = make_float4(0.f, 0.f, 0.f, 0.f);
                } else {
                    const int d = c >> 2, h = c & 3;
                    const int db = (sb >> (4 - 2 * d)) & 3;
                    const int off = (sb >> 6) * kTapStride + d * kRow + 8 * db;
                    r[q] = *reinterpret_cast<const v2d*>(taps + off + 2 * h);
                    // atoms past the pass end are staged as zero windows, so that the compute loop
                    // reads whole groups of four without bounds checks (adds exact zeros)
                    if (a >= n) r[q] = v2d{0.0, 0.0};
                }
            }
        };
        auto stage = [&](double* buf) {
#pragma unroll
            for (int q = 0; q < kPer; q++) {
                const int e = t + 256 * q;
                if (kPieces % 256 == 0 || e < kPieces) {
                    if constexpr (FA) {   // fp32 staging: piece e is floats 4e .. 4e + 3
                        reinterpret_cast<float4*>(buf)[e] = r[q];
                    } else if constexpr (TF) {
                        v2d* o = reinterpret_cast<v2d*>(buf) + 2 * e;
                        o[0] = v2d{(double)r[q].x, (double)r[q].y};
                        o[1] = v2d{(double)r[q].z, (double)r[q].w};
                    } else {
                        reinterpret_cast<v2d*>(buf)[e] = r[q];
                    }
                }
            }
        };
        const int npass = (nseg + kSpPass - 1) / kSpPass;
        // staging buffer p (FA: fp32 windows, half the bytes)
        auto sbuf = [&](int p) { return FA ? (double*)(reinterpret_cast<float*>(st) + (p & 1) * kSpPass * kSpWin)
                                           : st + (p & 1) * kSpPass * kSpWin; };
        fetch(0, min(kSpPass, nseg));
        stage(sbuf(0));
        __syncthreads();
        for (int p = 0; p < npass; p++) {
            const int base = p * kSpPass, n = min(kSpPass, nseg - base);
            if (p + 1 < npass) fetch(base + kSpPass, min(kSpPass, nseg - base - kSpPass));
            const double* buf = sbuf(p);
            if constexpr (FA) {
                static_assert(kSpPass % 16 == 0, "four-atom groups");
                const float* fb = reinterpret_cast<const float*>(buf);
                const int yo = 8 + y, zo = 16 + (lane & 7);
                for (int a = w; a < n; a += 16) {
                    float4 xa[4], xb[4];
                    float yz[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const float* r = fb + (a + 4 * u) * kSpWin;
                        xa[u] = *reinterpret_cast<const float4*>(r);       // x taps 0..3 (a broadcast)
                        xb[u] = *reinterpret_cast<const float4*>(r + 4);   // x taps 4..7
                        yz[u] = r[yo] * r[zo];
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const v2f s2 = v2f{yz[u], yz[u]};
                        accf[0] = v2f{xa[u].x, xa[u].y} * s2 + accf[0];
                        accf[1] = v2f{xa[u].z, xa[u].w} * s2 + accf[1];
                        accf[2] = v2f{xb[u].x, xb[u].y} * s2 + accf[2];
                        accf[3] = v2f{xb[u].z, xb[u].w} * s2 + accf[3];
                    }
                }
            } else {
                // lane l reads x tap (l & 7) of the staged window, so lane i of every 16-lane row
                // holds tap i, and each FMA takes tap i by a row broadcast of its operand
                // (row_newbcast:i, 64-bit DPP): every operand comes from the LDS with 8-B per-lane
                // reads, no scalar-load latency (round 2 read the x window with wave-uniform scalar
                // loads, whose latency every wave waited on).
                // Four atoms per iteration: their twelve reads in flight together, one wait (a
                // branch-free body at fixed offsets; the windows of atoms past the pass end are
                // staged as zeros, kSpPass is a multiple of 16, so every read is in the buffer).
                static_assert(kSpPass % 16 == 0, "four-atom groups");
                const double* rb = buf + (lane & 7);   // x tap; y tap at +8 + y - (lane & 7), z at +16
                const int oy = 8 + y - (lane & 7);
                for (int a = w; a < n; a += 16) {
                    const double* r = rb + a * kSpWin;
                    double xv[4], yv[4], zv[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        xv[u] = r[4 * u * kSpWin]; yv[u] = r[4 * u * kSpWin + oy]; zv[u] = r[4 * u * kSpWin + 16];
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) fma8_row_bcast(acc, xv[u], yv[u] * zv[u]);
                }
            }
            if (p + 1 < npass) stage(sbuf(p + 1));
            __syncthreads();
        }
    }
    // the 4 waves' partial tiles, summed in fixed wave order
    __syncthreads();
    double* red = st;   // [4][8][64]
    if constexpr (FA) {
#pragma unroll
        for (int k = 0; k < 4; k++) { acc[2 * k] = accf[k].x; acc[2 * k + 1] = accf[k].y; }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) red[(w * 8 + i) * 64 + lane] = acc[i];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int pt = t + 256 * h, i = pt >> 6, l = pt & 63;
        const double v = ((red[i * 64 + l] + red[(8 + i) * 64 + l]) + red[(16 + i) * 64 + l]) + red[(24 + i) * 64 + l];
        const size_t o = ((size_t)(8 * tx + i) * ng.y + 8 * ty + (l >> 3)) * ng.z + 8 * tz + (l & 7);
        if constexpr (GF) reinterpret_cast<float*>(grid)[o] = (float)v;
        else grid[o] = v;
    }
}

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Round 4: the spread as an fp64 matrix-core contraction (CF_VARIANT_VECTOR_SPREAD: k_g_spread_tile).
// One 256-thread workgroup per 16 (x) x 8 (y) x 8 (z) tile, whose 1024 points are
//     G[x][(y, z)] = sum_a X_a[x] (Y_a[y] Z_a[z])
// over the tile's source atoms: per group of 4 atoms one v_mfma_f64_16x16x4_f64 per 16 (y, z)
// columns, A = the 4 atoms' x windows (lane l: x = l & 15 of atom l >> 4), B = Y Z products
// (lane l: atom l >> 4, column 16 nb + (l & 15), one multiply per lane), so the FMAs leave the
// VALU (k_g_spread_tile: 1 mul + 8 VALU FMAs per (tile, atom) per lane plus the DPP
// bookkeeping).  The tile is 16 wide in x so that M = 16 is the x axis with no padding; its
// sources are the atoms whose first tap lies in the (NS + 1) x NS x NS sort bins (8^3 each, the
// bins of k_g_bin) that can reach it: x bins 2 tx - dxb, dxb = -1 .. NS - 1, y and z bins as the
// 8^3 tile's.  A source's x window is 16 points of its bin-aligned 24-point row starting at
// 8 dxb (the row is zero outside [0, 24), so the two 8-point halves are row windows dxb and
// dxb + 1, or zeros); y and z windows as before.  Passes of kP atoms staged structure-of-arrays
// (X[kP][16], Y[kP][8], Z[kP][8]: the A reads of a wave are 512 contiguous bytes, the B reads
// broadcast), double-buffered; the 4 waves take every 4th group of 4 atoms and keep the whole
// tile (4 accumulators of 16 x 16 per wave), summed in fixed wave order at the end: every output
// is the same sum in the same order on every run (bitwise reproducible), though not the VALU
// kernel's order (equal to it to ~1e-15 relative).  When ng.x is an odd multiple of 8 (C5: 264)
// the last x tile covers 8 planes: bin 2 tx + 1 wraps to bin 0, whose atoms reach only the
// tile's missing half (rows < 0 are zero), and only the planes x < ng.x are written.
template <int NS>
__global__ void __launch_bounds__(256) k_g_spread_mfma(int3 ng, int3 nb, const int* __restrict__ start,
                                                       const double* __restrict__ taps, const int4* __restrict__ g0s,
                                                       double* __restrict__ grid, const int* __restrict__ xr, int W) {
    constexpr int NBX = NS + 1;              // x bins per tile: dxb = ix - 1, ix < NBX
    constexpr int NSRC = NBX * NS * NS;
    static_assert(NS <= 3 && NSRC <= 64, "bin offsets are packed in 2 bits per axis; one wave scans the bins");
    constexpr int kBA = 16;                  // atoms per wave block (4 groups of 4: 16 MFMAs)
    constexpr int kBufD = kBA * 32;          // X 16 + Y 8 + Z 8 doubles per atom
    __shared__ __attribute__((aligned(16))) double st[4 * kBufD];   // one buffer per wave; [0, 1024) reused by the reduction
    static_assert(4 * kBufD >= 1024, "the reduction buffer fits");
    __shared__ int bin_start[NSRC], bin_pre[NSRC + 1], bin_db[NSRC];
    __shared__ int src[kSpMaxSrc];   // slot << 6 | ix << 4 | dy << 2 | dz of the kept sources
    __shared__ int wcnt[4 * (kSpMaxSrc / 256)];
    const int nyz = nb.y * nb.z;
    int tile = blockIdx.x;
    if (nyz % 8 == 0) {   // XCD-aware order, as k_g_spread_tile
        const int per = nyz / 8, i = blockIdx.x / 8;
        tile = (i / per) * nyz + (blockIdx.x % 8) * per + i % per;
    }
    const int tz = tile % nb.z, ty = (tile / nb.z) % nb.y, tx = tile / nyz;
    const int xlim = min(16, ng.x - 16 * tx);   // 8 for the last tile when ng.x is an odd multiple of 8
    if (!x_range_in_slab(16 * tx, 16 * tx + xlim - 1, xr, W, ng.x)) return;
    const int t = threadIdx.x;
    const int lane = t & 63, w = wave_id();
    if (w == 0) {   // the source bins, their counts scanned across the lanes (was a serial loop)
        int s0 = 0, cnt = 0;
        if (lane < NSRC) {
            const int ix = lane / (NS * NS), dy = (lane / NS) % NS, dz = lane % NS;
            const int b = (wrapb(2 * tx + 1 - ix, nb.x) * nb.y + wrapb(ty - dy, nb.y)) * nb.z + wrapb(tz - dz, nb.z);
            s0 = start[b];
            cnt = start[b + 1] - s0;
            bin_start[lane] = s0;
            bin_db[lane] = (ix << 8) | (dy << 4) | dz;
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(cnt, o);
            if (lane >= o) cnt += v;
        }
        if (lane < NSRC) bin_pre[lane + 1] = cnt;
        if (lane == 0) bin_pre[0] = 0;
    }
    __syncthreads();
    const int total = bin_pre[NSRC];
    const int k = lane >> 4, c = lane & 15;   // MFMA operand lane: atom k of the group, x / column c
    d4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; q++) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
    // staging: piece e = lane & 15 (16 B) of atoms (lane >> 4) + 4 q, q < 4, of a wave block: e < 8
    // x (half e >> 2), 8..11 y, 12..15 z -- per-lane constants: the axis, the source-word bits
    // that pick its window, the window adjustment and the LDS address pattern (selects, no
    // branches); atoms past the end are zero windows (the last group of 4 is read whole)
    const int e = lane & 15, a0 = lane >> 4;
    const int axis = e < 8 ? 0 : (e < 12 ? 1 : 2);
    const int fsh = 4 - 2 * axis;                   // source-word bits of this axis's window
    const int wadj = axis == 0 ? (e >> 2) - 1 : 0;  // x: window dxb + half
    const int poff = kRow * axis + 2 * (e & 3);
    const int dbase = axis == 0 ? 2 * e : (axis == 1 ? 16 * kBA : 24 * kBA) + 2 * (e & 3);
    const int dstr = axis == 0 ? 16 : 8;            // doubles per atom in this piece's array
    double* const wbuf = st + w * kBufD;            // this wave's buffer
    for (int seg0 = 0; seg0 < total; seg0 += kSpMaxSrc) {
        const int nall = min(kSpMaxSrc, total - seg0);
        __syncthreads();   // previous segment's blocks done with src
        constexpr int kRounds = kSpMaxSrc / 256;
        int2 sb[kRounds];
        int4 g[kRounds];
#pragma unroll
        for (int r = 0; r < kRounds; r++) {
            const int u = 256 * r + t;
            sb[r] = make_int2(0, 0);
            if (u < nall) {
                const int a = seg0 + u;
                int lo = 0, hi = NSRC;
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (bin_pre[mid] <= a) lo = mid; else hi = mid;
                }
                sb[r] = make_int2(bin_start[lo] + (a - bin_pre[lo]), lo);
            }
        }
#pragma unroll
        for (int r = 0; r < kRounds; r++) g[r] = 256 * r + t < nall ? g0s[sb[r].x] : make_int4(0, 0, 0, 0);
        bool keep[kRounds];
        unsigned long long m[kRounds];
        int dbits[kRounds];
#pragma unroll
        for (int r = 0; r < kRounds; r++) {
            const int db = bin_db[sb[r].y];
            const int ix = db >> 8, dy = (db >> 4) & 15, dz = db & 15;
            dbits[r] = (ix << 4) | (dy << 2) | dz;
            // the x taps [rx, rx + W) of the row reach the tile's points [8 (ix - 1), 8 (ix - 1) + 16)
            keep[r] = 256 * r + t < nall && (g[r].x & 7) + W > 8 * (ix - 1) && (g[r].y & 7) + W > 8 * dy &&
                      (g[r].z & 7) + W > 8 * dz;
            m[r] = __ballot(keep[r]);
            if ((t & 63) == 0) wcnt[4 * r + (t >> 6)] = __popcll(m[r]);
        }
        __syncthreads();
        int nseg = 0;
#pragma unroll
        for (int r = 0; r < kRounds; r++) {
            int off = nseg;
            for (int q = 0; q < (t >> 6); q++) off += wcnt[4 * r + q];
            if (keep[r]) src[off + __popcll(m[r] & ((1ull << (t & 63)) - 1))] = (sb[r].x << 6) | dbits[r];
            nseg += wcnt[4 * r] + wcnt[4 * r + 1] + wcnt[4 * r + 2] + wcnt[4 * r + 3];
        }
        __syncthreads();
        // Wave w takes the blocks of 16 kept sources w, w + 4, w + 8, ... through its own LDS
        // double buffer, with no block barrier until the segment ends: the waves drift apart, so
        // one wave's MFMAs overlap another's staging (the block-wide passes of 32 or 64 atoms had
        // every wave meet at each pass barrier: 51 of 81 us with the MFMAs removed).  Block bi + 2's
        // tap loads are issued as block bi starts, two blocks (32 MFMAs) before they are staged.
        const int nwb = (nseg + kBA - 1) / kBA;
        const int nb_w = nwb > w ? (nwb - w + 3) / 4 : 0;   // this wave's blocks
        v2d rva[4], rvb[4];
        auto fetch = [&](v2d (&rv)[4], int bi) {
            const int base = (w + 4 * bi) * kBA, n = min(kBA, nseg - base);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int a = a0 + 4 * q;
                const int s = src[base + min(a, n - 1)];
                const int wi = ((s >> fsh) & 3) + wadj;
                const v2d v = *reinterpret_cast<const v2d*>(taps + (size_t)(s >> 6) * kTapStride + poff + 8 * max(wi, 0));
                rv[q] = a < n && (unsigned)wi <= 2u ? v : v2d{0.0, 0.0};
            }
        };
        // one buffer per wave: a wave's LDS accesses execute in order, so block bi + 1 is staged
        // over block bi right after the wave's own reads of it (16 KB per workgroup instead of 32:
        // more workgroups per CU)
        auto stage = [&](const v2d (&rv)[4]) {
#pragma unroll
            for (int q = 0; q < 4; q++) *reinterpret_cast<v2d*>(wbuf + dbase + dstr * (a0 + 4 * q)) = rv[q];
        };
        // block bi: `nxt` holds block bi + 1 (loaded during block bi - 1), `fre` receives bi + 2
        auto block = [&](int bi, v2d (&fre)[4], const v2d (&nxt)[4]) {
            if (bi + 2 < nb_w) fetch(fre, bi + 2);
            const int n = min(kBA, nseg - (w + 4 * bi) * kBA);
            const double* xb = wbuf + c;
            const double* yb = wbuf + 16 * kBA + (c >> 3);
            const double* zb = wbuf + 24 * kBA + (c & 7);
            const int ngr = (n + 3) >> 2;
            for (int gi = 0; gi < ngr; gi++) {
                const int a = 4 * gi + k;
                const double xa = xb[16 * a];
                const double za = zb[8 * a];
                const double* ya = yb + 8 * a;
#pragma unroll
                for (int q = 0; q < 4; q++) acc[q] = mfma64(xa, ya[2 * q] * za, acc[q]);
            }
            wave_sync();   // (keeps the compiler from moving the stores above the reads)
            if (bi + 1 < nb_w) stage(nxt);
            wave_sync();   // this wave's stores before its next block's reads
        };
        if (nb_w > 0) {
            fetch(rva, 0);
            if (nb_w > 1) fetch(rvb, 1);
            stage(rva);
            wave_sync();
            for (int bi = 0; bi < nb_w; bi += 2) {
                block(bi, rva, rvb);
                if (bi + 1 < nb_w) block(bi + 1, rvb, rva);
            }
        }
    }
    // the 4 waves' partial tiles, summed in fixed wave order ((w0 + w1) + w2) + w3 through one
    // 8-KB tile; acc[q][i] of lane l is the point x = (l >> 4) + 4 i, (y, z) column 16 q + (l & 15)
    double* red = st;   // [16 x][64 (y, z)]
    for (int ww = 0; ww < 4; ww++) {
        __syncthreads();
        if (w == ww) {
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    double& r = red[(k + 4 * i) * 64 + 16 * q + c];
                    r = ww == 0 ? acc[q][i] : r + acc[q][i];
                }
        }
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 4; h++) {
        const int pt = t + 256 * h, x = pt >> 6, l = pt & 63;
        if (x < xlim) grid[((size_t)(16 * tx + x) * ng.y + 8 * ty + (l >> 3)) * ng.z + 8 * tz + (l & 7)] = red[pt];
    }
}

// ---------------------------------------------------------------------------------
// 3. pruned DFT stages
// ---------------------------------------------------------------------------------
// Every pruned-DFT stage as one batched complex GEMM on the fp64 matrix cores,
//   C(m, n) = sum_k A(m, k) B(k, n),
//   A(m, k) = A[m sam + k sak]            (complex; real for the forward z stage's grid rows)
//   B(k, n) = B[k sbk + (n / ndiv) sb1 + (n % ndiv) sb0]                       (complex)
//   C(m, n) = C[m scm + (n / ndiv) scn1 + (n % ndiv) scn0]   (complex, or its real part)
// n = (n / ndiv, n % ndiv) folds a batch index into the columns.  A block of 4 waves owns a
// BM x BN output tile (64 x 64, or 32 x 32 when the big tiles would not give every CU a
// block); K is walked in chunks of 16 staged in LDS from coalesced global loads (threads run
// along whichever index of the operand is contiguous in memory), double-buffered: the next
// chunk's loads are in flight in registers while the current chunk's MFMAs issue.  Each wave
// computes a (BM/2) x (BN/2) quadrant as 16x16 v_mfma_f64_16x16x4_f64 tiles: lane l supplies
// A[m0 + (l & 15)][k0 + (l >> 4)] and B[k0 + (l >> 4)][n0 + (l & 15)] (one ds_read_b128 each:
// re and im), complex products as real MFMAs: re += Ar Br + (-Ai) Bi, im += Ar Bi + Ai Br.
// Accumulator register r of lane l is C[(l >> 4) + 4r][l & 15].  Every output is summed by
// one wave in k order: deterministic.
// The former one-tile-per-wave kernel fetched its operands straight from global memory (16
// cache lines per load instruction) and ran 11-23 us per stage at C3.
struct CGemm {
    int M, N, K;
    const void* A; long sam, sak;
    const double2* B; long sbk, sb1, sb0;
    void* C; long scm, scn1, scn0;
    int ndiv;
    // x-slab (multi-rank): which index is the grid x-plane -- 0 none, 1 m / xdiv, 2 n / xdiv,
    // 3 k.  Tiles whose x-planes all lie outside the slab are skipped; along k only the slab's
    // planes are walked (k = kbase + t mod K, t < kcount).
    int xdim = 0, xdiv = 1;
    const int* xr = nullptr;
    int W = 0, ngx = 0;
};

constexpr int kGBK = 16;   // k per LDS chunk (4 MFMA k-steps)

// WM x (4 / WM) waves over the block tile (2 x 2, or 4 x 1 for the 64 x 80 tile that fits
// kmax = 65's 65 output columns with less padding)
template <int BM, int BN, int WM, bool AREAL, bool CREAL>
__global__ void __launch_bounds__(256) k_g_cgemm(CGemm g) {
    constexpr int WN = 4 / WM;
    constexpr int SM = BM / (16 * WM), SN = BN / (16 * WN);   // 16x16 subtiles per wave and axis
    static_assert(SM * 16 * WM == BM && SN * 16 * WN == BN && (BM * kGBK) % 256 == 0 && (BN * kGBK) % 256 == 0,
                  "cgemm tile shape");
    constexpr int AP = BM + 1, BP = BN + 1;              // padded LDS rows (conflict-free transposed stores)
    constexpr int AE = BM * kGBK / 256, BE = BN * kGBK / 256;   // elements per thread per chunk
    __shared__ double2 sA[2][kGBK * AP];
    __shared__ double2 sB[2][kGBK * BP];
    const int tiles_m = (g.M + BM - 1) / BM;
    const int tm = blockIdx.x % tiles_m, tn = blockIdx.x / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    if (g.xdim == 1 && !x_range_in_slab(m0 / g.xdiv, min(m0 + BM - 1, g.M - 1) / g.xdiv, g.xr, g.W, g.ngx)) return;
    if (g.xdim == 2 && !x_range_in_slab(n0 / g.xdiv, min(n0 + BN - 1, g.N - 1) / g.xdiv, g.xr, g.W, g.ngx)) return;
    int kbase = 0, kcount = g.K;
    if (g.xdim == 3 && g.xr) {
        int s0, len;
        slab_of(g.xr, g.W, g.ngx, s0, len);
        if (len < g.K) { kbase = s0; kcount = len; }
    }
    const int t = threadIdx.x;
    const bool a_kfast = g.sak == 1, b_kfast = g.sbk == 1;
    // element e (of AE / BE) of thread t in the chunk: (row, k) of the A tile, (k, col) of B
    auto a_idx = [&](int e, int& mm, int& kk) {
        const int q = t + 256 * e;
        if (a_kfast) { kk = q % kGBK; mm = q / kGBK; } else { mm = q % BM; kk = q / BM; }
    };
    auto b_idx = [&](int e, int& kk, int& nn) {
        const int q = t + 256 * e;
        if (b_kfast) { kk = q % kGBK; nn = q / kGBK; } else { nn = q % BN; kk = q / BN; }
    };
    auto kmap = [&](int kt, bool& ok) {   // chunk-relative k -> operand k (slab walk)
        ok = kt < kcount;
        int k = kbase + kt;
        return k >= g.K ? k - g.K : k;
    };
    double2 ra[AE], rb[BE];
    auto load = [&](int c) {
#pragma unroll
        for (int e = 0; e < AE; e++) {
            int mm, kk;
            a_idx(e, mm, kk);
            bool ok;
            const int k = kmap(c * kGBK + kk, ok);
            const int m = m0 + mm;
            ra[e] = make_double2(0.0, 0.0);
            if (ok && m < g.M) {
                if (AREAL) ra[e].x = reinterpret_cast<const double*>(g.A)[m * g.sam + k * g.sak];
                else ra[e] = reinterpret_cast<const double2*>(g.A)[m * g.sam + k * g.sak];
            }
        }
#pragma unroll
        for (int e = 0; e < BE; e++) {
            int kk, nn;
            b_idx(e, kk, nn);
            bool ok;
            const int k = kmap(c * kGBK + kk, ok);
            const int n = n0 + nn;
            rb[e] = (ok && n < g.N) ? g.B[k * g.sbk + (long)(n / g.ndiv) * g.sb1 + (long)(n % g.ndiv) * g.sb0]
                                    : make_double2(0.0, 0.0);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int e = 0; e < AE; e++) {
            int mm, kk;
            a_idx(e, mm, kk);
            sA[buf][kk * AP + mm] = ra[e];
        }
#pragma unroll
        for (int e = 0; e < BE; e++) {
            int kk, nn;
            b_idx(e, kk, nn);
            sB[buf][kk * BP + nn] = rb[e];
        }
    };
    const int lane = t & 63, w = wave_id();
    const int wm = w / WN, wn = w % WN;
    const int r16 = lane & 15, kq = lane >> 4;
    d4 cre[SM][SN], cim[SM][SN];
#pragma unroll
    for (int i = 0; i < SM; i++)
#pragma unroll
        for (int j = 0; j < SN; j++) {
            cre[i][j] = d4{0.0, 0.0, 0.0, 0.0};
            cim[i][j] = d4{0.0, 0.0, 0.0, 0.0};
        }
    const int nchunks = (kcount + kGBK - 1) / kGBK;
    load(0);
    store(0);
    __syncthreads();
    for (int c = 0; c < nchunks; c++) {
        const int buf = c & 1;
        if (c + 1 < nchunks) load(c + 1);
#pragma unroll
        for (int s = 0; s < kGBK / 4; s++) {
            const int kr = 4 * s + kq;
            double2 af[SM], bf[SN];
#pragma unroll
            for (int i = 0; i < SM; i++) af[i] = sA[buf][kr * AP + (wm * SM + i) * 16 + r16];
#pragma unroll
            for (int j = 0; j < SN; j++) bf[j] = sB[buf][kr * BP + (wn * SN + j) * 16 + r16];
#pragma unroll
            for (int i = 0; i < SM; i++)
#pragma unroll
                for (int j = 0; j < SN; j++) {
                    if (AREAL) {
                        cre[i][j] = mfma64(af[i].x, bf[j].x, cre[i][j]);
                        cim[i][j] = mfma64(af[i].x, bf[j].y, cim[i][j]);
                    } else {
                        cre[i][j] = mfma64(af[i].x, bf[j].x, cre[i][j]);
                        cre[i][j] = mfma64(-af[i].y, bf[j].y, cre[i][j]);
                        if (!CREAL) {
                            cim[i][j] = mfma64(af[i].x, bf[j].y, cim[i][j]);
                            cim[i][j] = mfma64(af[i].y, bf[j].x, cim[i][j]);
                        }
                    }
                }
        }
        if (c + 1 < nchunks) store(buf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < SN; j++) {
        const int n = n0 + (wn * SN + j) * 16 + r16;
        if (n >= g.N) continue;
        const long coff = (long)(n / g.ndiv) * g.scn1 + (long)(n % g.ndiv) * g.scn0;
#pragma unroll
        for (int i = 0; i < SM; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int m = m0 + (wm * SM + i) * 16 + kq + 4 * q;
                if (m >= g.M) continue;
                const long off = (long)m * g.scm + coff;
                if (CREAL) reinterpret_cast<double*>(g.C)[off] = cre[i][j][q];
                else reinterpret_cast<double2*>(g.C)[off] = make_double2(cre[i][j][q], cim[i][j][q]);
            }
    }
}

// ---------------------------------------------------------------------------------
// 3b. pruned DFT stages by the 8 x Q factorization (ng = 8Q, every axis; the default).
//     Each stage maps a batch of sequences between the length side (n < ng, grid points)
//     and the mode side (k = k0 + j, j < J; the reference's mode box), w = e^{i 2pi/ng}:
//       analysis   X[k] = sum_n x[n] w^{nk}        (forward z, y, x stages)
//       synthesis  x[n] = sum_j c[j] w^{n k_j}     (inverse x, y, z stages; z keeps Re)
//     With n = Qa + b (a < 8, b < Q), w^{nk} = e^{i 2pi a (k mod 8)/8} w^{bk}, so
//       analysis:  Y[b][r] = sum_a x[Qa+b] e^{i 2pi a r/8}   (8-point DFT per b: ~70 flops)
//                  X[k]    = sum_b w^{bk} Y[b][k mod 8]      (Q complex MACs per mode)
//       synthesis: Z[b][r] = sum_{k = r mod 8} c_k w^{bk}     (same count), then the 8-point DFT
//                  over r gives x[Qa+b] for every a.
//     Per sequence ~Q (J + 70) complex operations instead of ng J (C5: 8x fewer than the GEMM
//     stages for the x/y stages, 3.6x for z), which makes the stages HBM-bound instead of
//     bound by the matrix pipe.  Layout: a 256-thread block owns 64 sequences, lane = sequence;
//     wave w owns the residue classes r = w and w + 4 (the modes k = r mod 8 of every lane's
//     sequence: mt accumulators per class in registers).  b is walked in chunks of 8: the
//     chunk's 8-point DFTs (threads along whichever index is contiguous in memory) go to LDS
//     [b][r][sequence]; each lane then reads its sequence's Y[b][r] (conflict-free).  The
//     twiddles are factored, w^{b(k_r + 8t)} = w^{b k_r} w_Q^{bt} (k_r the first mode of class
//     r, w_Q = w^8): a [8][Q] twist table and one [Q][mt] table shared by every class (<= 13 KB
//     per axis: it stays in the scalar cache), read with wave-uniform scalar loads and fed to
//     the FMAs as SGPR operands.  (Per-class [r][b][mt] tables of up to 72 KB missed the
//     scalar cache on every b: C5 stages 2-4x slower.)  Every output is one lane's sum in b
//     order: deterministic.  Multi-rank x-slab: blocks whose sequences all lie in x-planes
//     outside the slab exit (z and y stages); the forward x stage reads planes outside the
//     slab as zero (select, not multiply: they are stale).
// ---------------------------------------------------------------------------------
struct Dft8 {
    int nseq, Q, sdiv;
    long s1, s0, sn;     // length side: element (s, n) at (s / sdiv) s1 + (s % sdiv) s0 + n sn
    long c1, c0, cj;     // mode side:   element (s, j) at (s / sdiv) c1 + (s % sdiv) c0 + j cj
    const void* in;
    void* out;
    int rj[8], rc[8];    // j of the first mode of class r, class size
    int xmode, xdiv;     // 1: sequence s lies in x-plane s / xdiv; 2: n is the x-plane (analysis)
    const int* xr;
    int W, ngx;
};

// the coefficient pass (k_g_coeffs) fused into the forward x stage on one rank (COEF): the stage
// writes f = w_z c a conj(S) / phih instead of B, and its blocks' energy partials (round 6: one
// launch and one pass over B fewer on the reciprocal chain's exposed tail)
struct Coef {
    int KX, KY, KZ;
    double3 rec;
    double cst, one_4a2;
    const double *dx, *dy, *dz;
    double* e_part;
};

constexpr int kD8Seq = 64, kD8BC = 8;
constexpr int kDft8Mt[] = {4, 8, 9, 16, 17};   // class-size paddings instantiated (CF_D8_MT)

__device__ __forceinline__ v2d mul_i(v2d v) { return v2d{-v.y, v.x}; }

// y[r] = sum_a x[a] e^{+i 2pi a r/8} (radix-2 in registers)
__device__ __forceinline__ void dft8(const v2d (&x)[8], v2d (&y)[8]) {
    const double c = 0.70710678118654752440;
    const v2d e0 = x[0] + x[4], e1 = x[0] - x[4], e2 = x[2] + x[6], e3 = x[2] - x[6];
    const v2d o0 = x[1] + x[5], o1 = x[1] - x[5], o2 = x[3] + x[7], o3 = x[3] - x[7];
    const v2d E0 = e0 + e2, E2 = e0 - e2, E1 = e1 + mul_i(e3), E3 = e1 - mul_i(e3);
    const v2d O0 = o0 + o2, O2 = o0 - o2, O1 = o1 + mul_i(o3), O3 = o1 - mul_i(o3);
    const v2d wO1 = v2d{c * (O1.x - O1.y), c * (O1.x + O1.y)};      // e^{i pi/4} O1
    const v2d w3O3 = v2d{-c * (O3.x + O3.y), c * (O3.x - O3.y)};    // e^{i 3pi/4} O3
    const v2d iO2 = mul_i(O2);
    y[0] = E0 + O0; y[4] = E0 - O0;
    y[1] = E1 + wO1; y[5] = E1 - wO1;
    y[2] = E2 + iO2; y[6] = E2 - iO2;
    y[3] = E3 + w3O3; y[7] = E3 - w3O3;
}

__device__ __forceinline__ void cmac(v2d& acc, v2d y, double2 t) {
    acc.x = fma(y.x, t.x, acc.x);
    acc.x = fma(-y.y, t.y, acc.x);
    acc.y = fma(y.x, t.y, acc.y);
    acc.y = fma(y.y, t.x, acc.y);
}

// analysis (CIN: complex input; else real input, classes r > 4 from conj Y[b][8 - r]).
// A block owns SEQ sequences (64, or 16 for the stages with few sequences, so the grid still
// fills the chip) and 8 SEQ threads: lane = (sequence, class), 64 / SEQ classes per wave.  Each
// thread does one (sequence, b) 8-point DFT per chunk; the next chunk's 8 inputs are loaded
// into registers before the current chunk's class sums, so the global latency overlaps the
// FMAs.  The twist table (class-dependent) is read from LDS, the [Q][mt] rows as scalar loads.
template <int MT, bool CIN, int SEQ, bool COEF = false>
__global__ void __launch_bounds__(8 * SEQ) k_g_dft8_fwd(Dft8 d, const double2* __restrict__ twist,
                                                        const double2* __restrict__ tq, Coef cf = Coef{}) {
    constexpr int NR = CIN ? 8 : 5, SP = SEQ + 1, NT = 8 * SEQ;
    extern __shared__ v2d sm8[];
    v2d* sY = sm8;                       // [kD8BC][NR][SP]
    v2d* stw = sm8 + kD8BC * NR * SP;    // [8][Q]
    const int s0 = blockIdx.x * SEQ;
    if (d.xmode == 1 && d.xr &&
        !x_range_in_slab(s0 / d.xdiv, min(s0 + SEQ - 1, d.nseq - 1) / d.xdiv, d.xr, d.W, d.ngx))
        return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int sq = lane % SEQ, r = wave_id() * (64 / SEQ) + lane / SEQ;
    for (int e = tid; e < 8 * d.Q; e += NT) stw[e] = reinterpret_cast<const v2d*>(twist)[e];
    // this thread's step-1 item: real input rows are contiguous along n (8 lanes per sequence
    // over b); complex inputs are contiguous along the sequence index (lanes over sequences)
    const int sl = CIN ? (tid % SEQ) : (tid >> 3), bl = CIN ? (tid / SEQ) : (tid & 7);
    const int si = s0 + sl;
    const bool sok = si < d.nseq;
    const long ibase = sok ? (long)(si / d.sdiv) * d.s1 + (long)(si % d.sdiv) * d.s0 : 0;
    v2d xn[8];
    auto load = [&](int bc) {
        const bool ok = sok && bc + bl < d.Q;
#pragma unroll
        for (int a = 0; a < 8; a++) {
            const int n = d.Q * a + bc + bl;
            const bool oka = ok && (d.xmode != 2 || x_in_slab(n, d.xr, d.W, d.ngx));
            if constexpr (CIN) {
                const v2d v = reinterpret_cast<const v2d*>(d.in)[oka ? ibase + n * d.sn : 0];
                xn[a] = oka ? v : v2d{0.0, 0.0};
            } else {
                const double v = reinterpret_cast<const double*>(d.in)[oka ? ibase + n * d.sn : 0];
                xn[a] = v2d{oka ? v : 0.0, 0.0};
            }
        }
    };
    v2d acc[MT];
#pragma unroll
    for (int t = 0; t < MT; t++) acc[t] = v2d{0.0, 0.0};
    const bool cj = !CIN && r > 4;
    const int rr = cj ? 8 - r : r;
    load(0);
    for (int bc = 0; bc < d.Q; bc += kD8BC) {
        const int nb = min(kD8BC, d.Q - bc);
        {
            v2d y[8];
            dft8(xn, y);
#pragma unroll
            for (int q = 0; q < NR; q++) sY[(bl * NR + q) * SP + sl] = y[q];
        }
        __syncthreads();
        if (bc + kD8BC < d.Q) load(bc + kD8BC);
        const v2d* twr = stw + r * d.Q + bc;
        const double2* tqb = tq + (long)bc * MT;
#pragma unroll 2
        for (int b = 0; b < nb; b++) {
            v2d y = sY[(b * NR + rr) * SP + sq];
            if (cj) y.y = -y.y;
            const v2d tw = twr[b];
            v2d yt = v2d{0.0, 0.0};
            cmac(yt, y, make_double2(tw.x, tw.y));   // w^{b k_r} Y[b][r]
#pragma unroll
            for (int t = 0; t < MT; t++) cmac(acc[t], yt, tqb[b * MT + t]);
        }
        __syncthreads();
    }
    const int s = s0 + sq;
    if constexpr (!COEF) {
        if (s >= d.nseq) return;
        const long base = (long)(s / d.sdiv) * d.c1 + (long)(s % d.sdiv) * d.c0;
        const int cnt = d.rc[r], j0 = d.rj[r];
#pragma unroll
        for (int t = 0; t < MT; t++)
            if (t < cnt) reinterpret_cast<v2d*>(d.out)[base + (long)(j0 + 8 * t) * d.cj] = acc[t];
    } else {
        // x stage: sequence s = (ny index, nz), mode j = nx + KX - 1 -- the element k_g_coeffs
        // calls t = (j NY + ny index) KZ + nz; the same coefficient and energy per element
        // (RCK:528, 549-551), the energy summed per block in a fixed order
        __shared__ double red[8 * SEQ / 64];
        double e = 0;
        if (s < d.nseq) {
            const long base = (long)(s / d.sdiv) * d.c1 + (long)(s % d.sdiv) * d.c0;
            const int cnt = d.rc[r], j0 = d.rj[r];
            const int nz = s % cf.KZ, ny = s / cf.KZ - (cf.KY - 1);
            const double ky = ny * cf.rec.y, kz = nz * cf.rec.z;
            const double wz = nz > 0 ? 2.0 : 1.0;
            const double Dyz = cf.dy[abs(ny)] * cf.dz[nz];
#pragma unroll
            for (int t = 0; t < MT; t++) {
                if (t < cnt) {
                    const int j = j0 + 8 * t, nx = j - (cf.KX - 1);
                    const double kx = nx * cf.rec.x;
                    const double k2 = kx * kx + ky * ky + kz * kz;
                    const double a = k2 > 0 ? exp(-k2 * 0.25 * cf.one_4a2) / k2 : 0.0;
                    const double D = cf.dx[abs(nx)] * Dyz;
                    const double sr = acc[t].x * D, si = acc[t].y * D;
                    e += 0.5 * wz * cf.cst * a * (sr * sr + si * si);
                    const double c = wz * cf.cst * a * D;
                    reinterpret_cast<v2d*>(d.out)[base + (long)j * d.cj] = v2d{c * sr, -c * si};
                }
            }
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) e += __shfl_xor(e, m);
        if (lane == 0) red[wave_id()] = e;
        __syncthreads();
        if (tid == 0) {
            double tot = 0;
#pragma unroll
            for (int w = 0; w < 8 * SEQ / 64; w++) tot += red[w];
            cf.e_part[blockIdx.x] = tot;
        }
    }
}

// analysis along z of the real grid rows (contiguous along n): 8 rows per block, NB waves;
// lane = (row, class), wave g = the g-th of NB contiguous b ranges (so the [Q][mt] twiddle rows
// stay wave-uniform scalar loads).  The rows' 8-point DFTs are computed for every b at once from
// loads that run along the row ((row, b) items with lane-consecutive b: each a-slice of a row is
// one contiguous run, every element loaded once); Y[row][b][r <= 4] and the twist table live in
// LDS (21 KB at C5: many blocks per CU).  The b loop is software-pipelined (the next b's LDS and
// scalar loads are issued before the current b's FMAs).  The NB partial sums are added in wave
// order into LDS output rows (deterministic), written as contiguous rows of t1.  (The
// sequence-lane kernel read a row as 8-element pieces per b chunk: 2.9x the grid's bytes
// fetched at C5.)
constexpr int kZR = 8;    // rows per block of the z analysis
constexpr int kZIR = 16;  // rows per block of the z synthesis

template <int MT, int NB, bool GF = false>   // GF: fp32 grid rows (GridPlan::grid_f32)
__global__ void __launch_bounds__(64 * NB) k_g_dft8_zfwd(Dft8 d, const double2* __restrict__ twist,
                                                         const double2* __restrict__ tq) {
    extern __shared__ v2d sm8[];
    constexpr int R = kZR;
    const int Q = d.Q;
    v2d* sY = sm8;                        // [R][Q][5]
    v2d* stw = sm8 + R * Q * 5;           // [8][Q]
    v2d* sO = stw + 8 * Q;                // [R][J] output rows
    const int s0 = blockIdx.x * R;
    if (d.xmode == 1 && d.xr &&
        !x_range_in_slab(s0 / d.xdiv, min(s0 + R - 1, d.nseq - 1) / d.xdiv, d.xr, d.W, d.ngx))
        return;
    const int tid = threadIdx.x;
    for (int e = tid; e < 8 * Q; e += 64 * NB) stw[e] = reinterpret_cast<const v2d*>(twist)[e];
    using GT = std::conditional_t<GF, float, double>;
    const GT* in = reinterpret_cast<const GT*>(d.in);
    for (int it = tid; it < R * Q; it += 64 * NB) {
        const int row = it / Q, b = it - row * Q;
        const int s = s0 + row;
        const bool ok = s < d.nseq;
        const long base = (long)(ok ? s : 0) * d.s1 + b;
        v2d x[8], y[8];
#pragma unroll
        for (int a = 0; a < 8; a++) {
            const double v = (double)in[base + (long)Q * a];
            x[a] = v2d{ok ? v : 0.0, 0.0};
        }
        dft8(x, y);
#pragma unroll
        for (int r = 0; r < 5; r++) sY[(row * Q + b) * 5 + r] = y[r];
    }
    __syncthreads();
    const int lane = tid & 63, g = wave_id();
    const int row = lane & 7, r = lane >> 3;
    const bool cj = r > 4;
    const int rr = cj ? 8 - r : r;
    const int b0 = g * Q / NB, b1 = (g + 1) * Q / NB;
    v2d acc[MT];
#pragma unroll
    for (int t = 0; t < MT; t++) acc[t] = v2d{0.0, 0.0};
    if (b0 < b1) {
        v2d yn = sY[(row * Q + b0) * 5 + rr], twn = stw[r * Q + b0];
        double2 qn[MT];
#pragma unroll
        for (int t = 0; t < MT; t++) qn[t] = tq[b0 * MT + t];
        for (int b = b0; b < b1; b++) {
            v2d y = yn;
            const v2d tw = twn;
            double2 q[MT];
#pragma unroll
            for (int t = 0; t < MT; t++) q[t] = qn[t];
            if (b + 1 < b1) {
                yn = sY[(row * Q + b + 1) * 5 + rr];
                twn = stw[r * Q + b + 1];
#pragma unroll
                for (int t = 0; t < MT; t++) qn[t] = tq[(b + 1) * MT + t];
            }
            if (cj) y.y = -y.y;
            v2d yt = v2d{0.0, 0.0};
            cmac(yt, y, make_double2(tw.x, tw.y));   // w^{b k_r} Y[b][r]
#pragma unroll
            for (int t = 0; t < MT; t++) cmac(acc[t], yt, q[t]);
        }
    }
    const int J = d.rc[0] + d.rc[1] + d.rc[2] + d.rc[3] + d.rc[4] + d.rc[5] + d.rc[6] + d.rc[7];
    const int cnt = d.rc[r], j0 = d.rj[r];
    for (int gg = 0; gg < NB; gg++) {   // partial sums added in wave order
        if (g == gg) {
#pragma unroll
            for (int t = 0; t < MT; t++)
                if (t < cnt) {
                    v2d& o = sO[row * J + j0 + 8 * t];
                    o = gg == 0 ? acc[t] : o + acc[t];
                }
        }
        __syncthreads();
    }
    const int nrow = min(R, d.nseq - s0);
    v2d* out = reinterpret_cast<v2d*>(d.out) + (long)s0 * d.c1;   // rows of J = c1 consecutive modes
    for (int e = tid; e < nrow * J; e += 64 * NB) out[e] = sO[e];
}

// synthesis along z into the real grid rows: 16 rows per block, NB waves; lane = (row, class
// pair) with pairs {0, 4}, {1, 7}, {2, 6}, {3, 5}, wave g = the g-th of NB b ranges.  Only Re x is
// kept, so a pair needs only P_r = Z_r + conj Z_{8-r} (Re(e^{it} Z_r) + Re(e^{-it} Z_{8-r}) =
// Re(e^{it} P_r)) and (Re Z_0, Re Z_4): 4 complex values per (row, b) in LDS for every b at
// once; then the outputs x[Qa + b] are formed per (row, b) item with lane-consecutive b, so each
// a-slice of a row is written as one contiguous run (the sequence-lane kernel wrote 64-byte
// pieces per b chunk: 1.55x the grid's bytes written at C5).
template <int MT, int NB, bool GF = false>   // GF: fp32 grid rows (GridPlan::grid_f32)
__global__ void __launch_bounds__(64 * NB) k_g_dft8_zinv(Dft8 d, const double2* __restrict__ twist,
                                                         const double2* __restrict__ tq) {
    extern __shared__ v2d sm8[];
    constexpr int R = kZIR;
    const int Q = d.Q;
    v2d* sZ = sm8;                 // [R][Q][4]
    v2d* stw = sm8 + R * Q * 4;    // [8][Q]
    const int s0 = blockIdx.x * R;
    if (d.xmode == 1 && d.xr &&
        !x_range_in_slab(s0 / d.xdiv, min(s0 + R - 1, d.nseq - 1) / d.xdiv, d.xr, d.W, d.ngx))
        return;
    const int tid = threadIdx.x;
    for (int e = tid; e < 8 * Q; e += 64 * NB) stw[e] = reinterpret_cast<const v2d*>(twist)[e];
    const int lane = tid & 63, g = wave_id();
    const int row = lane & 15, p = lane >> 4;
    const int r1 = p, r2 = p == 0 ? 4 : 8 - p;
    v2d c1[MT], c2[MT];
    {
        const int s = s0 + row;
        const bool ok = s < d.nseq;
        const v2d* in = reinterpret_cast<const v2d*>(d.in) + (long)(ok ? s : 0) * d.c1;
        const int n1 = d.rc[r1], j1 = d.rj[r1], n2 = d.rc[r2], j2 = d.rj[r2];
#pragma unroll
        for (int t = 0; t < MT; t++) {
            const bool o1 = ok && t < n1, o2 = ok && t < n2;
            const v2d a1 = in[o1 ? j1 + 8 * t : 0], a2 = in[o2 ? j2 + 8 * t : 0];
            c1[t] = o1 ? a1 : v2d{0.0, 0.0};
            c2[t] = o2 ? a2 : v2d{0.0, 0.0};
        }
    }
    __syncthreads();
    const int b0 = g * Q / NB, b1 = (g + 1) * Q / NB;
    if (b0 < b1) {
        double2 qn[MT];
#pragma unroll
        for (int t = 0; t < MT; t++) qn[t] = tq[b0 * MT + t];
        for (int b = b0; b < b1; b++) {
            double2 q[MT];
#pragma unroll
            for (int t = 0; t < MT; t++) q[t] = qn[t];
            if (b + 1 < b1) {
#pragma unroll
                for (int t = 0; t < MT; t++) qn[t] = tq[(b + 1) * MT + t];
            }
            v2d z1 = v2d{0.0, 0.0}, z2 = v2d{0.0, 0.0};
#pragma unroll
            for (int t = 0; t < MT; t++) {
                cmac(z1, c1[t], q[t]);
                cmac(z2, c2[t], q[t]);
            }
            const v2d t1 = stw[r1 * Q + b], t2 = stw[r2 * Q + b];
            v2d y1 = v2d{0.0, 0.0}, y2 = v2d{0.0, 0.0};
            cmac(y1, z1, make_double2(t1.x, t1.y));
            cmac(y2, z2, make_double2(t2.x, t2.y));
            sZ[(row * Q + b) * 4 + p] = p == 0 ? v2d{y1.x, y2.x} : v2d{y1.x + y2.x, y1.y - y2.y};
        }
    }
    __syncthreads();
    const double c = 0.70710678118654752440;
    using GT = std::conditional_t<GF, float, double>;
    GT* out = reinterpret_cast<GT*>(d.out);
    for (int it = tid; it < R * Q; it += 64 * NB) {
        const int rw = it / Q, b = it - rw * Q;
        const int s = s0 + rw;
        if (s >= d.nseq) break;   // rows are in order: every later item is past the end too
        const v2d* z = sZ + (rw * Q + b) * 4;
        const v2d z04 = z[0], P1 = z[1], P2 = z[2], P3 = z[3];
        const double e = z04.x + z04.y, o = z04.x - z04.y;               // a even / odd: Re Z0 +- Re Z4
        const double u1 = c * (P1.x - P1.y), v1 = c * (P1.x + P1.y);     // Re(e^{i pi/4} P1), Re(e^{-i pi/4} P1)
        const double u3 = c * (-P3.x - P3.y), v3 = c * (-P3.x + P3.y);   // Re(e^{i 3pi/4} P3), Re(e^{-i 3pi/4} P3)
        // angle pi a r/4 of class r at output a (mod 2pi): r = 1: a pi/4, r = 2: a pi/2, r = 3: 3a pi/4
        double x[8];
        x[0] = e + P1.x + P2.x + P3.x;
        x[1] = o + u1 - P2.y + u3;
        x[2] = e - P1.y - P2.x + P3.y;
        x[3] = o - v1 + P2.y - v3;
        x[4] = e - P1.x + P2.x - P3.x;
        x[5] = o - u1 - P2.y - u3;
        x[6] = e + P1.y - P2.x - P3.y;
        x[7] = o + v1 + P2.y + v3;
        const long base = (long)s * d.s1 + b;
#pragma unroll
        for (int a = 0; a < 8; a++) out[base + (long)Q * a] = (GT)x[a];
    }
}

// synthesis (ROUT: keep the real part, written as doubles).  A block owns SEQ sequences and
// 8 SEQ threads, lane = (sequence, class) as in the analysis: each lane holds the modes of its
// class and forms Z[b][r] for the chunk; then each thread turns one (sequence, b) into the
// outputs n = Qa + b.  b chunks are independent, so they are also dealt over gridDim.y blocks
// of the same sequences.
// COEF (several ranks, the x stage): the coefficient pass of k_g_coeffs applied as the all-reduced
// B(n) is loaded (f = w_z c a conj(S) / phih, S = B D), with the energy of each element summed by
// the blockIdx.y = 0 blocks (each loads every element of its sequences once) into e_part[blockIdx.x]
// -- the same per-element arithmetic as the forward x stage's COEF form on one rank
template <int MT, bool ROUT, int SEQ, bool COEF = false>
__global__ void __launch_bounds__(8 * SEQ) k_g_dft8_inv(Dft8 d, const double2* __restrict__ twist,
                                                        const double2* __restrict__ tq, Coef cf = Coef{}) {
    constexpr int SP = SEQ + 1, NT = 8 * SEQ;
    extern __shared__ v2d sm8[];
    v2d* sZ = sm8;                      // [kD8BC][8][SP]
    v2d* stw = sm8 + kD8BC * 8 * SP;    // [8][Q]
    // the [Q][mt] rows in LDS (broadcast reads): as wave-uniform scalar loads every b step waited
    // on them, and a scalar load's wait covers the LDS reads too (one counter): C3 inverse stages
    // 28.5 -> 27.0 us, C5 153 -> 146 (r6ai; the same staging in the analysis made it slower,
    // 36.5 -> 40.1 and 151 -> 161: its larger LDS footprint costs blocks per CU)
    v2d* stq = stw + 8 * d.Q;           // [Q][MT]
    const int s0 = blockIdx.x * SEQ;
    if (d.xmode == 1 && d.xr &&
        !x_range_in_slab(s0 / d.xdiv, min(s0 + SEQ - 1, d.nseq - 1) / d.xdiv, d.xr, d.W, d.ngx))
        return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int sq = lane % SEQ, r = wave_id() * (64 / SEQ) + lane / SEQ;
    for (int e = tid; e < 8 * d.Q; e += NT) stw[e] = reinterpret_cast<const v2d*>(twist)[e];
    for (int e = tid; e < d.Q * MT; e += NT) stq[e] = reinterpret_cast<const v2d*>(tq)[e];
    const int s = s0 + sq;
    v2d cv[MT];
    {
        const bool ok = s < d.nseq;
        const long base = ok ? (long)(s / d.sdiv) * d.c1 + (long)(s % d.sdiv) * d.c0 : 0;
        const int cnt = d.rc[r], j0 = d.rj[r];
#pragma unroll
        for (int t = 0; t < MT; t++) {
            const bool okt = ok && t < cnt;
            const v2d v = reinterpret_cast<const v2d*>(d.in)[okt ? base + (long)(j0 + 8 * t) * d.cj : 0];
            cv[t] = okt ? v : v2d{0.0, 0.0};
        }
        if constexpr (COEF) {
            // sequence s = (ny index, nz), mode j = nx + KX - 1, as in k_g_dft8_fwd's COEF form
            // (RCK:528, 549-551)
            __shared__ double red[8 * SEQ / 64];
            double e = 0;
            if (ok) {
                const int nz = s % cf.KZ, ny = s / cf.KZ - (cf.KY - 1);
                const double ky = ny * cf.rec.y, kz = nz * cf.rec.z;
                const double wz = nz > 0 ? 2.0 : 1.0;
                const double Dyz = cf.dy[abs(ny)] * cf.dz[nz];
#pragma unroll
                for (int t = 0; t < MT; t++) {
                    if (t < cnt) {
                        const int j = j0 + 8 * t, nx = j - (cf.KX - 1);
                        const double kx = nx * cf.rec.x;
                        const double k2 = kx * kx + ky * ky + kz * kz;
                        const double a = k2 > 0 ? exp(-k2 * 0.25 * cf.one_4a2) / k2 : 0.0;
                        const double D = cf.dx[abs(nx)] * Dyz;
                        const double sr = cv[t].x * D, si = cv[t].y * D;
                        e += 0.5 * wz * cf.cst * a * (sr * sr + si * si);
                        const double c = wz * cf.cst * a * D;
                        cv[t] = v2d{c * sr, -c * si};
                    }
                }
            }
            if (cf.e_part && blockIdx.y == 0) {   // (block-uniform)
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) e += __shfl_xor(e, m);
                if (lane == 0) red[wave_id()] = e;
                __syncthreads();
                if (tid == 0) {
                    double tot = 0;
#pragma unroll
                    for (int w = 0; w < 8 * SEQ / 64; w++) tot += red[w];
                    cf.e_part[blockIdx.x] = tot;
                }
            }
        }
    }
    const int sl = ROUT ? (tid >> 3) : (tid % SEQ), bl = ROUT ? (tid & 7) : (tid / SEQ);
    const int ss = s0 + sl;
    const long obase = ss < d.nseq ? (long)(ss / d.sdiv) * d.s1 + (long)(ss % d.sdiv) * d.s0 : 0;
    __syncthreads();
    for (int bc = kD8BC * blockIdx.y; bc < d.Q; bc += kD8BC * gridDim.y) {
        const int nb = min(kD8BC, d.Q - bc);
        const v2d* twr = stw + r * d.Q + bc;
        const v2d* tqb = stq + bc * MT;
#pragma unroll 2
        for (int b = 0; b < nb; b++) {
            v2d z = v2d{0.0, 0.0}, zt = v2d{0.0, 0.0};
#pragma unroll
            for (int t = 0; t < MT; t++) {
                const v2d q = tqb[b * MT + t];
                cmac(z, cv[t], make_double2(q.x, q.y));
            }
            const v2d tw = twr[b];
            cmac(zt, z, make_double2(tw.x, tw.y));   // w^{b k_r} sum_t c_t w_Q^{b t}
            sZ[(b * 8 + r) * SP + sq] = zt;
        }
        __syncthreads();
        if (ss < d.nseq && bl < nb) {
            v2d z[8], x[8];
#pragma unroll
            for (int q = 0; q < 8; q++) z[q] = sZ[(bl * 8 + q) * SP + sl];
            dft8(z, x);
#pragma unroll
            for (int a = 0; a < 8; a++) {
                const long o = obase + (long)(d.Q * a + bc + bl) * d.sn;
                if constexpr (ROUT) reinterpret_cast<double*>(d.out)[o] = x[a].x;
                else reinterpret_cast<v2d*>(d.out)[o] = x[a];
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------
// 4. coefficients: S = B/phih, energy c a |S|^2 (x1/2 for the nz = 0 plane, which holds
//    both members of each +-n pair), f = w_z c a conj(S)/phih written in place.
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_g_coeffs(int KX, int KY, int KZ, double3 rec, double cst, double one_4a2,
                                                  const double* __restrict__ dx, const double* __restrict__ dy,
                                                  const double* __restrict__ dz, double2* __restrict__ buf,
                                                  double* __restrict__ e_part, int include_energy) {
    __shared__ double red[256];
    const int NY = 2 * KY - 1;
    const int total = (2 * KX - 1) * NY * KZ;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    double e = 0;
    if (t < total) {
        const int nz = t % KZ, r = t / KZ;
        const int ny = r % NY - (KY - 1), nx = r / NY - (KX - 1);
        const double kx = nx * rec.x, ky = ny * rec.y, kz = nz * rec.z;
        const double k2 = kx * kx + ky * ky + kz * kz;
        const double a = k2 > 0 ? exp(-k2 * 0.25 * one_4a2) / k2 : 0.0;   // RCK:528
        const double D = dx[abs(nx)] * dy[abs(ny)] * dz[nz];
        const double2 B = buf[t];
        const double sr = B.x * D, si = B.y * D;
        const double wz = nz > 0 ? 2.0 : 1.0;
        if (include_energy) e = 0.5 * wz * cst * a * (sr * sr + si * si);   // RCK:549-551
        const double c = wz * cst * a * D;
        buf[t] = make_double2(c * sr, -c * si);
    }
    red[threadIdx.x] = e;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) e_part[blockIdx.x] = red[0];
}

// ---------------------------------------------------------------------------------
// 5. interpolation, one workgroup per 8^3 tile: the potential grid over the tile plus the
//    W-1 halo (R = 7 + W points per axis, wrapped) is staged in LDS, then each wave takes
//    atoms of the tile's bin.  Per atom: lane (d, m) evaluates tap m of axis d and its
//    derivative; lane (jg, k) accumulates t0 = sum_i G X_i and t1 = sum_i G dX_i over its
//    (j = 4jj + jg, k) columns (2 FMAs per LDS read, x taps as wave-uniform scalars), then
//    pot = sum t0 Y Z, grad = (t1 Y Z, t0 dY Z, t0 Y dZ) in a fixed-order wave reduction.
// ---------------------------------------------------------------------------------
constexpr int kInterpThreads = 512;

// A 64-bit value of another lane by two DPP moves (VALU; a __shfl_xor costs two ds_bpermute,
// LDS instructions, per step and value -- the interpolation's LDS issue queue is its bottleneck).
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    int lo, hi;
    if constexpr (ROWS == 0xF) {
        // every lane has a valid source (quad permutations, mirrors): no "old" value, so no
        // zeroed destination register per move (the update form cost one v_mov per DPP move)
        lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, ROWS, 0xF, false);
        hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, ROWS, 0xF, false);
    } else {   // rows outside the mask keep the old value: 0, so that they add nothing
        lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xF, false);
        hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xF, false);
    }
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// v + (the same lane of the partner row / half-wave): gfx950 v_permlane16_swap / 32_swap of two
// copies of v leave row r's and row r ^ 1's values (halves: lanes l and l ^ 32) in the two
// outputs at each lane's own position, so every lane gets the same two-term sum
__device__ __forceinline__ double add_swap16(double v) {
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}

__device__ __forceinline__ double add_swap32(double v) {
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}

// Wave sums of four values at once, halving the values carried per lane at every exchange:
// quad xor 1 (even lanes keep pv / px, odd lanes py / pz), quad xor 2 (one value per lane: lane
// l holds quantity (pv, py, px, pz)[l & 3] over its quad), row rotations by 4 and 8 (the row's
// four quads, same l & 3), then the partner row and the other half-wave.  13 exchanges instead
// of 4 x 6 DPP reductions.  Lane l < 4 (every lane, for its l & 3) ends with the wave total of
// quantity (pv, py, px, pz)[l & 3]; one fixed order per lane: deterministic.
__device__ __forceinline__ double wave_sum4(double pv, double px, double py, double pz, int lane) {
    const bool odd = lane & 1, hi = lane & 2;
    const double a = (odd ? py : pv) + dpp_f64<0xB1, 0xF>(odd ? pv : py);    // quad_perm [1,0,3,2]
    const double b = (odd ? pz : px) + dpp_f64<0xB1, 0xF>(odd ? px : pz);
    double c = (hi ? b : a) + dpp_f64<0x4E, 0xF>(hi ? a : b);                // quad_perm [2,3,0,1]
    c += dpp_f64<0x124, 0xF>(c);   // row_ror:4
    c += dpp_f64<0x128, 0xF>(c);   // row_ror:8
    c = add_swap16(c);
    return add_swap32(c);
}

// the potential grid over tile (tx, ty, tz) plus the W - 1 halo, wrapped, into sg[R][R][R]:
// rows of R consecutive z; thread t covers column c = t % R of rows t / R, t / R + RPP, ...
// The same halo, 16 B per load: thread t takes the z pair (2 c, 2 c + 1), c = t % ceil(R / 2), of
// rows t / ceil(R / 2), + RPP, ... (an even z and an even ng.z keep every pair inside one wrapped
// row and 16-B aligned; the odd R's last pair reads one point past the halo, not stored).  Half
// the loads and address computations of interp_stage (its VALU work was a third of
// k_g_interp2's, profiles/r04i_*)
// x-plane stride of k_g_interp2's halo (doubles): the smallest >= R^2 that is W..32-W modulo 32,
// so that the two 16-lane rows of a half-wave -- x rows 2ii and 2ii + 1, W z points each --
// fall on disjoint LDS banks (a ds_read_b64 group is 32 lanes over 64 four-byte banks, i.e.
// 32 doubles: the rows' residues b..b+W-1 and b+SX..b+SX+W-1 mod 32 must not meet)
template <int W>
constexpr int interp_plane_stride() {
    int s = (7 + W) * (7 + W);
    while (s % 32 < W || s % 32 > 32 - W) s++;
    return s;
}

template <int W, int SX = (7 + W) * (7 + W), bool GF = false>   // GF: an fp32 grid, widened as staged
__device__ __forceinline__ void interp_stage16(int3 ng, const double* __restrict__ G, int tx, int ty, int tz,
                                               double* __restrict__ sg) {
    constexpr int R = 7 + W;
    constexpr int RC = (R + 1) / 2;            // z pairs per row
    constexpr int RPP = kInterpThreads / RC;   // rows per pass
    const int c = threadIdx.x % RC, r0 = threadIdx.x / RC;
    int z = 8 * tz + 2 * c;
    z -= z >= ng.z ? ng.z : 0;
    constexpr int kRows = (R * R + RPP - 1) / RPP;
    constexpr int kDA = RPP / R, kDB = RPP % R;
    if (r0 < RPP) {
        v2d gv[kRows];
        int so[kRows];   // LDS row offset a * SX + b * R of halo row (a, b) = (x, y)
        int a = r0 / R, b = r0 - (r0 / R) * R;
        const int zy = ng.y * ng.z;
#pragma unroll
        for (int q = 0; q < kRows; q++) {
            const bool in = r0 + q * RPP < R * R;
            so[q] = a * SX + b * R;
            int x = 8 * tx + (in ? a : 0), y = 8 * ty + (in ? b : 0);
            x -= x >= ng.x ? ng.x : 0;
            y -= y >= ng.y ? ng.y : 0;
            const unsigned idx = (unsigned)(x * zy + y * ng.z + z);
            if constexpr (GF) {
                const float2 f = reinterpret_cast<const float2*>(G)[idx >> 1];   // (z even: 8-B aligned)
                gv[q] = v2d{(double)f.x, (double)f.y};
            } else {
                gv[q] = *reinterpret_cast<const v2d*>(reinterpret_cast<const char*>(G) + idx * 8u);
            }
            a += kDA; b += kDB;
            if (b >= R) { b -= R; a += 1; }
        }
#pragma unroll
        for (int q = 0; q < kRows; q++) {
            const int row = r0 + q * RPP;
            if (row < R * R) {
                sg[so[q] + 2 * c] = gv[q].x;
                if (2 * c + 1 < R) sg[so[q] + 2 * c + 1] = gv[q].y;
            }
        }
    }
}

// interp_stage16 with the work per thread fixed across x planes: thread t takes the z pair c and
// the y row b of item t mod (R RC) and every second x plane from t / (R RC) (2 R RC <= threads);
// its y / z wrap, grid row offset and LDS offset are computed once, each plane costs a row add, an
// x wrap and the load (round 4's row-by-row form recomputed both wraps and both offsets per row:
// 194 VALU per thread, a fifth of k_g_interp2's VALU instructions at C3)
template <int W, int SX>
__device__ __forceinline__ void interp_stage16p(int3 ng, const double* __restrict__ G, int tx, int ty, int tz,
                                                double* __restrict__ sg) {
    constexpr int R = 7 + W;
    constexpr int RC = (R + 1) / 2;   // z pairs per row
    constexpr int NIT = R * RC;       // (row, pair) items per plane
    constexpr int NP = (R + 1) / 2;   // planes of parity 0 (parity 1: R / 2)
    const int t = threadIdx.x;
    if (t >= 2 * NIT) return;
    const int par = t >= NIT ? 1 : 0, it = t - par * NIT;
    const int b = it / RC, c = it - b * RC;
    int y = 8 * ty + b, z = 8 * tz + 2 * c;
    y -= y >= ng.y ? ng.y : 0;
    z -= z >= ng.z ? ng.z : 0;
    const int yz = y * ng.z + z, zy = ng.y * ng.z;
    const int x0 = 8 * tx + par;
    v2d gv[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) {
        if (k < NP - 1 || par + 2 * k < R) {
            int x = x0 + 2 * k;
            x -= x >= ng.x ? ng.x : 0;
            const unsigned off = (unsigned)(x * zy + yz) * 8u;
            gv[k] = *reinterpret_cast<const v2d*>(reinterpret_cast<const char*>(G) + off);
        }
    }
    double* d = sg + par * SX + b * R + 2 * c;
    const bool two = 2 * c + 1 < R;   // the odd R's last pair: one point past the row
#pragma unroll
    for (int k = 0; k < NP; k++) {
        if (k < NP - 1 || par + 2 * k < R) {
            d[2 * k * SX] = gv[k].x;
            if (two) d[2 * k * SX + 1] = gv[k].y;
        }
    }
}

template <int W>
__device__ __forceinline__ void interp_stage(int3 ng, const double* __restrict__ G, int tx, int ty, int tz,
                                             double* __restrict__ sg) {
    constexpr int R = 7 + W;
    constexpr int RPP = kInterpThreads / R;   // rows per pass
    const int c = threadIdx.x % R, r0 = threadIdx.x / R;
    int z = 8 * tz + c;
    z -= z >= ng.z ? ng.z : 0;
    // every load of the staging issued before the first LDS store (one memory latency per
    // block instead of one per group of 4 rows): the block's halo comes from L2 / MALL.  Row
    // (a, b) = (x, y) halo offsets stepped incrementally by RPP rows (no divisions per row) and
    // 32-bit element offsets (ng^3 < 2^31) from the grid base
    constexpr int kRows = (R * R + RPP - 1) / RPP;
    constexpr int kDA = RPP / R, kDB = RPP % R;
    if (r0 < RPP) {
        double gv[kRows];
        int a = r0 / R, b = r0 - (r0 / R) * R;
        const int zy = ng.y * ng.z;
#pragma unroll
        for (int q = 0; q < kRows; q++) {
            const bool in = r0 + q * RPP < R * R;   // rows past the halo re-read row 0 (not stored)
            int x = 8 * tx + (in ? a : 0), y = 8 * ty + (in ? b : 0);
            x -= x >= ng.x ? ng.x : 0;
            y -= y >= ng.y ? ng.y : 0;
            // 32-bit byte offset from the uniform base: one global_load with an SGPR base
            const unsigned off = (unsigned)(x * zy + y * ng.z + z) * 8u;
            gv[q] = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(G) + off);
            a += kDA; b += kDB;
            if (b >= R) { b -= R; a += 1; }
        }
#pragma unroll
        for (int q = 0; q < kRows; q++) {
            const int row = r0 + q * RPP;
            if (row < R * R) sg[row * R + c] = gv[q];
        }
    }
}

template <int W>
__global__ void __launch_bounds__(kInterpThreads) k_g_interp(int3 ng, int3 nb, const int* __restrict__ start,
                                                             const int4* __restrict__ g0s,
                                                             const double4* __restrict__ srec, double beta,
                                                             double3 gscale, const double* __restrict__ G, int lo,
                                                             double* __restrict__ dedq, double* __restrict__ f_part,
                                                             int store) {
    constexpr int R = 7 + W;
    constexpr int NJ = (W + 3) / 4;
    extern __shared__ double sg[];   // [R][R][R]
    __shared__ double2 tp[kInterpThreads / 64][3][16];   // per wave: the current atom's taps (v, dv) per axis
    // XCD-aware tile order (as in k_g_spread): XCD blockIdx % 8 takes a contiguous 1/8 of the
    // (y, z) tile plane over every x, so neighbouring tiles' potential halos share its L2
    const int nyz = nb.y * nb.z;
    int tile = blockIdx.x;
    if (nyz % 8 == 0) {
        const int per = nyz / 8, i = blockIdx.x / 8;
        tile = (i / per) * nyz + (blockIdx.x % 8) * per + i % per;
    }
    const int s0 = start[tile], s1 = start[tile + 1];
    if (s0 == s1) return;
    const int tz = tile % nb.z, ty = (tile / nb.z) % nb.y, tx = tile / (nb.z * nb.y);
    interp_stage<W>(ng, G, tx, ty, tz, sg);
    __syncthreads();
    const int lane = threadIdx.x & 63, w = wave_id();
    const int d = lane >> 4, m = lane & 15;
    const int k = lane & 15, jg = lane >> 4;
    // the next atom's bin entry and coordinates are loaded while this one is evaluated (the
    // two dependent loads are otherwise the head of every atom's latency chain)
    int4 g_n = s0 + w < s1 ? g0s[s0 + w] : make_int4(0, 0, 0, 0);
    double4 sr_n = srec[g_n.w];
    for (int s = s0 + w; s < s1; s += kInterpThreads / 64) {
        const int4 g = g_n;
        const double4 sr = sr_n;
        if (s + kInterpThreads / 64 < s1) {
            g_n = g0s[s + kInterpThreads / 64];
            sr_n = srec[g_n.w];
        }
        // taps: lane (d, m)
        // tap m at t = g0 + m - s, g0 = ceil(s - W/2) (the unwrapped first tap of k_g_bin)
        const double sd = d == 0 ? sr.x : (d == 1 ? sr.y : sr.z);
        double v = 0, dv = 0;
        if (d < 3 && m < W) es_tap(ceil(sd - 0.5 * W) + m - sd, 2.0 / W, beta, v, dv);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // previous atom's reads of tp done
        __builtin_amdgcn_wave_barrier();
        if (d < 3) tp[w][d][m] = make_double2(v, dv);   // zero beyond W
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int rx = g.x & 7, ry = g.y & 7, rz = g.z & 7;
        const double2 zv = tp[w][2][k];
        const double zt = zv.x, dzt = zv.y;
        double t0[NJ], t1[NJ];
#pragma unroll
        for (int jj = 0; jj < NJ; jj++) { t0[jj] = 0; t1[jj] = 0; }
        const int kk = k < W ? k : 0;
        const double* base = sg + (rx * R + ry) * R + rz + kk;
#pragma unroll
        for (int i = 0; i < W; i++) {
            const double2 xv = tp[w][0][i];   // broadcast LDS read (was 4 v_readlane per i)
            const double xi = xv.x, dxi = xv.y;
#pragma unroll
            for (int jj = 0; jj < NJ; jj++) {
                const int j = 4 * jj + jg;
                const double gv = base[(i * R + (j < W ? j : 0)) * R];
                t0[jj] += gv * xi;
                t1[jj] += gv * dxi;
            }
        }
        double pv = 0, px = 0, py = 0, pz = 0;
#pragma unroll
        for (int jj = 0; jj < NJ; jj++) {
            const int j = 4 * jj + jg;
            const double2 yv = tp[w][1][j < 16 ? j : 15];   // 4 addresses per wave (one per row)
            const double yt = j < W ? yv.x : 0.0, dyt = j < W ? yv.y : 0.0;
            pv += t0[jj] * yt;
            px += t1[jj] * yt;
            py += t0[jj] * dyt;
        }
        pz = pv * dzt;
        pv *= zt; px *= zt; py *= zt;
        // lane l < 4 ends with the wave total of quantity (pv, py, px, pz)[l]
        const double tot = wave_sum4(pv, px, py, pz, lane);
        if (lane < 4) {   // each owned atom is in exactly one bin: no other writer
            const int i = lo + g.w;
            const int c = lane == 2 ? 0 : (lane == 1 ? 1 : 2);   // force component of lanes 1..3
            if (store) {   // the reciprocal chain on its own stream: dedq_rec, f_rec = (p, -q) per atom,
                           // which k_assemble_energy folds in as the fused adds below
                if (lane == 0) {
                    dedq[i] = tot;
                    f_part[4 * i + 3] = -sr.w;
                } else {
                    f_part[4 * i + c] = tot;
                }
            } else if (lane == 0) {
                dedq[i] += tot;
            } else {
                const double gs = c == 0 ? gscale.x : (c == 1 ? gscale.y : gscale.z);
                f_part[3 * i + c] = fma(-sr.w * gs, tot, f_part[3 * i + c]);
            }
        }
    }
}

// ---------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------
// acc += x_I * y, x_I = the value lane I of this lane's 16-lane row holds in x (v_fmac_f64 with
// a 64-bit DPP row_newbcast:I source).  NOP: an s_nop 1 ahead of it, for a DPP source written
// by a VALU instruction just before (2 wait states; the compiler does not see inside the asm).
template <int I, bool NOP = false>
__device__ __forceinline__ void fmac_row_bcast(double& acc, double x, double y) {
    if constexpr (NOP)
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
            : "+v"(acc) : "v"(x), "v"(y), "i"(I));
    else
        asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(x), "v"(y), "i"(I));
}

// x_0 of this lane's 16-lane row (v_mov_b64 with a 64-bit DPP row_newbcast:0 source; the source
// must be fenced by dpp_ready after its last VALU write)
__device__ __forceinline__ double row_bcast0(double x) {
    double r;
    asm("v_mov_b64_dpp %0, %1 row_newbcast:0 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(x));
    return r;
}

// v_permlane16_swap of two copies of v: `even` = v of the even row of this lane's row pair
// (rows 0, 2), `odd` = v of the odd row (rows 1, 3), at this lane's position in the row
__device__ __forceinline__ void rows_even_odd(double v, double& even, double& odd) {
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    even = __longlong_as_double(((long long)hi[0] << 32) | lo[0]);
    odd = __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}

// a VALU-written value made safe as a DPP source: every reader comes after this s_nop
__device__ __forceinline__ double dpp_ready(double v) {
    asm("s_nop 1" : "+v"(v));
    return v;
}

template <int... Is, class F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, Is...>, F&& f) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) { static_for_impl(std::make_integer_sequence<int, N>{}, f); }

// Sums of four values over each 32-lane half of the wave (wave_sum4 without the half-wave
// exchange): lane l with (l & 31) < 4 holds its half's total of (pv, py, px, pz)[l & 3].
__device__ __forceinline__ double half_sum4(double pv, double px, double py, double pz, int lane) {
    const bool odd = lane & 1, hi = lane & 2;
    const double a = (odd ? py : pv) + dpp_f64<0xB1, 0xF>(odd ? pv : py);
    const double b = (odd ? pz : px) + dpp_f64<0xB1, 0xF>(odd ? px : pz);
    double c = (hi ? b : a) + dpp_f64<0x4E, 0xF>(hi ? a : b);
    c += dpp_f64<0x124, 0xF>(c);   // row_ror:4
    c += dpp_f64<0x128, 0xF>(c);   // row_ror:8
    return add_swap16(c);
}

// Two atoms per wave, one per 32-lane half h.  Lane (h, jg, k): z column k of the tile's halo,
// x rows i = 2ii + jg (ii < NX2 = ceil(W/2)), every y row j < W, taken in two halves of NJH rows
// (the accumulators of one half stay in registers).  Every tap lives in a register: each lane
// evaluates x tap 2k + jg (k < NX2), y tap k and z tap k of its half's atom, and the contractions
// take the x and y taps they need from the lane that holds them by DPP row broadcast (x tap 2ii +
// jg in lane ii of row jg, y tap j in lane j of both rows), so the LDS serves only the potential
// halo (49 reads per atom at W = 14).  A halo read of the two rows of a half hits x planes 2ii and
// 2ii + 1, whose z runs lie on disjoint LDS banks with the plane stride SX (interp_plane_stride;
// round 4 split the rows by y parity, 21 doubles apart: 3 of the 14 banks pairs met, 1.69
// conflict cycles per LDS instruction).  t0 = sum_i G X_i, t1 = sum_i G dX_i per (j, k) over the
// lane's x rows, then pot / gradient by y and z as in k_g_interp; the four sums of a half over
// its 32 lanes (both x parities) reduced in a fixed order; lanes (h, 0..3) store.
template <int W>
__global__ void __launch_bounds__(kInterpThreads) CF_LDS_UNPAIRED k_g_interp2(int3 ng, int3 nb, const int* __restrict__ start,
                                                              const int4* __restrict__ g0s,
                                                              const double4* __restrict__ srec, double beta,
                                                              double3 gscale, const double* __restrict__ G, int lo,
                                                              double* __restrict__ dedq, double* __restrict__ f_part,
                                                              int store) {
    constexpr int R = 7 + W;
    constexpr int SX = interp_plane_stride<W>();
    constexpr int NX2 = (W + 1) / 2;              // x rows per lane (the lane's parity)
    constexpr int NJH = (W + 1) / 2;              // y rows per half
    constexpr int NQ = 2 * NX2;                   // (y half, x row) steps
    constexpr int NW = kInterpThreads / 64;
    static_assert(W <= 16, "row broadcast reaches lanes 0..15");
    extern __shared__ double sg[];   // [R][SX]: x planes of R rows of R z points
    const int nyz = nb.y * nb.z;
    int tile = blockIdx.x;
    if (nyz % 8 == 0) {
        const int per = nyz / 8, i = blockIdx.x / 8;
        tile = (i / per) * nyz + (blockIdx.x % 8) * per + i % per;
    }
    const int s0 = start[tile], s1 = start[tile + 1];
    if (s0 == s1) return;
    const int tz = tile % nb.z, ty = (tile / nb.z) % nb.y, tx = tile / (nb.z * nb.y);
    if constexpr (2 * R * ((R + 1) / 2) <= kInterpThreads) interp_stage16p<W, SX>(ng, G, tx, ty, tz, sg);
    else interp_stage16<W, SX>(ng, G, tx, ty, tz, sg);
    __syncthreads();
    const int lane = threadIdx.x & 63, w = wave_id();
    const int h = lane >> 5, jg = (lane >> 4) & 1, k = lane & 15;
    const double hw_inv = 2.0 / W;
    // this half's next atom (bin entry, coordinates) loaded while the current one is evaluated
    int4 g_n = make_int4(0, 0, 0, 0);
    if (s0 + 2 * w + h < s1) g_n = g0s[s0 + 2 * w + h];
    double4 sr_n = srec[g_n.w];
    for (int sb = s0 + 2 * w; sb < s1; sb += 2 * NW) {   // wave-uniform
        const bool valid = sb + h < s1;
        const int4 g = g_n;
        const double4 sr = sr_n;
        if (sb + 2 * NW + h < s1) {
            g_n = g0s[sb + 2 * NW + h];
            sr_n = srec[g_n.w];
        }
        // taps (t = g0 + m - s, g0 = ceil(s - W/2)): y tap k, z tap k, x tap 2k + jg; zero
        // beyond the support
        // (one pass for y and z: row jg = 0 of each half evaluates y tap k, row 1 z tap k, and a
        // v_permlane16_swap copies each row's values into the other, so every lane ends with both)
        double xv = 0, xd = 0, yv = 0, yd = 0, zv = 0, zd = 0;
        {
            const double sd = jg ? sr.z : sr.y;
            double v = 0, dv = 0;
            if (k < W) es_tap(ceil(sd - 0.5 * W) + k - sd, hw_inv, beta, v, dv);
            rows_even_odd(v, yv, zv);
            rows_even_odd(dv, yd, zd);
        }
        if (k < NX2 && 2 * k + jg < W) es_tap(ceil(sr.x - 0.5 * W) + (2 * k + jg) - sr.x, hw_inv, beta, xv, xd);
        xv = dpp_ready(xv); xd = dpp_ready(xd); yv = dpp_ready(yv); yd = dpp_ready(yd);
        const int rx = g.x & 7, ry = g.y & 7, rz = g.z & 7;
        const double* base = sg + (rx + jg) * SX + ry * R + rz + (k < W ? k : 0);
        double t0[NJH], t1[NJH];   // the first x row of a y half initialises them (products)
        double pv = 0, px = 0, py = 0;
        // steps q = (y half, x row ii) in order; the NJH halo reads of step q + 1 are issued
        // before step q's FMAs (the scheduling barriers keep them there: the compiler otherwise
        // sinks each read to its first use, behind the inline asm, one LDS latency per read)
        double gv[2][NJH];
        // odd W: x row W of the jg = 1 lanes lies past the halo (its tap is zero); they re-read row
        // W - 1 of the jg = 0 lanes (the same addresses: a broadcast)
        const int xlast = (W % 2 == 1 && jg) ? -SX : 0;
        auto load_step = [&](int q, double (&gq)[NJH]) {
            const int yh = q / NX2, ii = q % NX2;
            const int xo = 2 * ii * SX + (ii == NX2 - 1 ? xlast : 0);
#pragma unroll
            for (int jj = 0; jj < NJH; jj++) {
                const int j = yh * NJH + jj;
                gq[jj] = base[xo + (j < W ? j : 0) * R];
            }
        };
        load_step(0, gv[0]);
        static_for<NQ>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            constexpr int yh = q / NX2, ii = q % NX2;
            if constexpr (q + 1 < NQ) load_step(q + 1, gv[(q + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ii == 0) {
                const double x0 = row_bcast0(xv), d0 = row_bcast0(xd);
#pragma unroll
                for (int jj = 0; jj < NJH; jj++) {
                    t0[jj] = x0 * gv[q & 1][jj];
                    t1[jj] = d0 * gv[q & 1][jj];
                }
            } else {
#pragma unroll
                for (int jj = 0; jj < NJH; jj++) {
                    fmac_row_bcast<ii>(t0[jj], xv, gv[q & 1][jj]);
                    fmac_row_bcast<ii>(t1[jj], xd, gv[q & 1][jj]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ii == NX2 - 1) {   // this y half done: contract with its y taps
                static_for<NJH>([&](auto J) {
                    constexpr int jj = decltype(J)::value;
                    constexpr int j = yh * NJH + jj;
                    if constexpr (j < W) {
                        fmac_row_bcast<j>(pv, yv, t0[jj]);
                        fmac_row_bcast<j>(px, yv, t1[jj]);
                        fmac_row_bcast<j>(py, yd, t0[jj]);
                    }
                });
            }
        });
        const double pz = pv * zd;
        pv *= zv; px *= zv; py *= zv;
        const double tot = half_sum4(pv, px, py, pz, lane);
        const int hl = lane & 31;
        if (hl < 4 && valid) {   // each owned atom is in exactly one bin: no other writer
            const int i = lo + g.w;
            const int c = hl == 2 ? 0 : (hl == 1 ? 1 : 2);   // force component of lanes 1..3
            if (store) {
                if (hl == 0) {
                    dedq[i] = tot;
                    f_part[4 * i + 3] = -sr.w;
                } else {
                    f_part[4 * i + c] = tot;
                }
            } else if (hl == 0) {
                dedq[i] += tot;
            } else {
                const double gs = c == 0 ? gscale.x : (c == 1 ? gscale.y : gscale.z);
                f_part[3 * i + c] = fma(-sr.w * gs, tot, f_part[3 * i + c]);
            }
        }
    }
}

// acc += x_I * y on the lanes of banks BANKS of every row (row_newbcast:I, bank_mask): the
// other lanes keep acc
template <int I, int BANKS>
__device__ __forceinline__ void fmac_row_bcast_banks(double& acc, double x, double y) {
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:%4" : "+v"(acc) : "v"(x), "v"(y), "i"(I),
        "i"(BANKS));
}

// 64-bit row rotation by 8 lanes (lane l of a row gets lane (l - 8) mod 16's value)
__device__ __forceinline__ double row_ror8(double v) { return dpp_f64<0x128, 0xF>(v); }

// Sums of four values over each 16-lane row (rows are atoms here): lane l with (l & 15) < 4 holds
// its row's total of (pv, py, px, pz)[l & 3]
__device__ __forceinline__ double row_sum4(double pv, double px, double py, double pz, int lane) {
    const bool odd = lane & 1, hi = lane & 2;
    const double a = (odd ? py : pv) + dpp_f64<0xB1, 0xF>(odd ? pv : py);
    const double b = (odd ? pz : px) + dpp_f64<0xB1, 0xF>(odd ? px : pz);
    double c = (hi ? b : a) + dpp_f64<0x4E, 0xF>(hi ? a : b);
    c += dpp_f64<0x124, 0xF>(c);   // row_ror:4
    c += dpp_f64<0x128, 0xF>(c);   // row_ror:8
    return c;
}

// W <= 8 (the mixed-precision grid): four atoms per wave, one per 16-lane row.  Lane (jg, k) of a
// row (jg = bit 3, k = bits 0-2) owns z column k and rows j = 2jj + jg (jj < ceil(W/2)), so every
// lane of the wave does useful work (k_g_interp2 leaves lanes k >= W of its 16-lane columns idle
// at W <= 8).  Taps: lanes jg = 0 evaluate x tap k, lanes jg = 1 z tap k (one pass; a row rotation
// by 8 gives the jg = 0 lanes their z tap); y taps 2n + jg in lane (jg, n < NJ), broadcast to the
// lanes of each half-row by row_newbcast with a bank mask.  Otherwise as k_g_interp2.
template <int W, bool F32 = false, bool GF = false>   // F32: fp32 taps; GF: fp32 grid (GridPlan::grid_f32)
__global__ void __launch_bounds__(kInterpThreads) CF_LDS_UNPAIRED k_g_interp4(int3 ng, int3 nb, const int* __restrict__ start,
                                                              const int4* __restrict__ g0s,
                                                              const double4* __restrict__ srec, double beta,
                                                              double3 gscale, const double* __restrict__ G, int lo,
                                                              double* __restrict__ dedq, double* __restrict__ f_part,
                                                              int store) {
    static_assert(W <= 8, "one 8-lane half-row per z column");
    constexpr int R = 7 + W;
    constexpr int NJ = (W + 1) / 2;
    constexpr int NW = kInterpThreads / 64;
    extern __shared__ double sg[];   // [R][R][R]
    const int nyz = nb.y * nb.z;
    int tile = blockIdx.x;
    if (nyz % 8 == 0) {
        const int per = nyz / 8, i = blockIdx.x / 8;
        tile = (i / per) * nyz + (blockIdx.x % 8) * per + i % per;
    }
    const int s0 = start[tile], s1 = start[tile + 1];
    if (s0 == s1) return;
    const int tz = tile % nb.z, ty = (tile / nb.z) % nb.y, tx = tile / (nb.z * nb.y);
    interp_stage16<W, (7 + W) * (7 + W), GF>(ng, G, tx, ty, tz, sg);
    __syncthreads();
    const int lane = threadIdx.x & 63, w = wave_id();
    const int q = lane >> 4, jg = (lane >> 3) & 1, k = lane & 7;
    const double hw_inv = 2.0 / W;
    int4 g_n = make_int4(0, 0, 0, 0);
    if (s0 + 4 * w + q < s1) g_n = g0s[s0 + 4 * w + q];
    double4 sr_n = srec[g_n.w];
    for (int sb = s0 + 4 * w; sb < s1; sb += 4 * NW) {   // wave-uniform
        const bool valid = sb + q < s1;
        const int4 g = g_n;
        const double4 sr = sr_n;
        if (sb + 4 * NW + q < s1) {
            g_n = g0s[sb + 4 * NW + q];
            sr_n = srec[g_n.w];
        }
        double xv, xd, yv = 0, yd = 0, zv, zd;
        {
            const double sd = jg ? sr.z : sr.x;
            double v = 0, dv = 0;
            if (k < W) {
                if constexpr (F32) es_tap_f(ceil(sd - 0.5 * W) + k - sd, hw_inv, beta, v, dv);
                else es_tap(ceil(sd - 0.5 * W) + k - sd, hw_inv, beta, v, dv);
            }
            xv = v; xd = dv;                              // lanes jg = 0: x tap k (the DPP sources)
            const double rv = row_ror8(v), rdv = row_ror8(dv);   // lane (0, k) <- lane (1, k)
            zv = jg ? v : rv; zd = jg ? dv : rdv;
        }
        if (k < NJ && 2 * k + jg < W) {
            if constexpr (F32) es_tap_f(ceil(sr.y - 0.5 * W) + (2 * k + jg) - sr.y, hw_inv, beta, yv, yd);
            else es_tap(ceil(sr.y - 0.5 * W) + (2 * k + jg) - sr.y, hw_inv, beta, yv, yd);
        }
        xv = dpp_ready(xv); xd = dpp_ready(xd); yv = dpp_ready(yv); yd = dpp_ready(yd);
        const int rx = g.x & 7, ry = g.y & 7, rz = g.z & 7;
        double t0[NJ], t1[NJ];   // row 0 initialises them (products: no zero fill)
        const double* base = sg + (rx * R + ry) * R + rz + (k < W ? k : 0);
        double gv[2][NJ];
        auto load_row = [&](int i, double (&gg)[NJ]) {
#pragma unroll
            for (int jj = 0; jj < NJ; jj++) {
                const int j = 2 * jj + jg;
                gg[jj] = base[(i * R + (j < W ? j : 0)) * R];
            }
        };
        load_row(0, gv[0]);
        static_for<W>([&](auto I) {
            constexpr int i = decltype(I)::value;
            if constexpr (i + 1 < W) load_row(i + 1, gv[(i + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (i == 0) {
                const double x0 = row_bcast0(xv), d0 = row_bcast0(xd);
#pragma unroll
                for (int jj = 0; jj < NJ; jj++) {
                    t0[jj] = x0 * gv[0][jj];
                    t1[jj] = d0 * gv[0][jj];
                }
            } else {
#pragma unroll
                for (int jj = 0; jj < NJ; jj++) {
                    fmac_row_bcast<i>(t0[jj], xv, gv[i & 1][jj]);
                    fmac_row_bcast<i>(t1[jj], xd, gv[i & 1][jj]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        });
        // y: lanes jg = 0 (banks 0, 1) take y tap 2jj from lane jj, lanes jg = 1 (banks 2, 3) tap
        // 2jj + 1 from lane 8 + jj
        double pv = 0, px = 0, py = 0;
        static_for<NJ>([&](auto J) {
            constexpr int jj = decltype(J)::value;
            fmac_row_bcast_banks<jj, 0x3>(pv, yv, t0[jj]);
            fmac_row_bcast_banks<8 + jj, 0xC>(pv, yv, t0[jj]);
            fmac_row_bcast_banks<jj, 0x3>(px, yv, t1[jj]);
            fmac_row_bcast_banks<8 + jj, 0xC>(px, yv, t1[jj]);
            fmac_row_bcast_banks<jj, 0x3>(py, yd, t0[jj]);
            fmac_row_bcast_banks<8 + jj, 0xC>(py, yd, t0[jj]);
        });
        const double pz = pv * zd;
        pv *= zv; px *= zv; py *= zv;
        const double tot = row_sum4(pv, px, py, pz, lane);
        const int rl = lane & 15;
        if (rl < 4 && valid) {   // each owned atom is in exactly one bin: no other writer
            const int i = lo + g.w;
            const int c = rl == 2 ? 0 : (rl == 1 ? 1 : 2);   // force component of lanes 1..3
            if (store) {
                if (rl == 0) {
                    dedq[i] = tot;
                    f_part[4 * i + 3] = -sr.w;
                } else {
                    f_part[4 * i + c] = tot;
                }
            } else if (rl == 0) {
                dedq[i] += tot;
            } else {
                const double gs = c == 0 ? gscale.x : (c == 1 ? gscale.y : gscale.z);
                f_part[3 * i + c] = fma(-sr.w * gs, tot, f_part[3 * i + c]);
            }
        }
    }
}

static double es_host(double t, int W, double beta) {
    double z = 2.0 * t / W, u = 1.0 - z * z;
    return u > 0 ? std::exp(beta * (std::sqrt(u) - 1.0)) : 0.0;
}

// Gauss-Legendre nodes/weights on [-1, 1] (Newton on P_n)
static void gauss_legendre(int n, std::vector<double>& x, std::vector<double>& w) {
    x.assign(n, 0.0);
    w.assign(n, 0.0);
    for (int i = 0; i < (n + 1) / 2; i++) {
        double z = std::cos(kPi * (i + 0.75) / (n + 0.5)), pp = 0;
        for (int it = 0; it < 100; it++) {
            double p1 = 1, p2 = 0;
            for (int j = 1; j <= n; j++) {
                double p3 = p2;
                p2 = p1;
                p1 = ((2.0 * j - 1) * z * p2 - (j - 1.0) * p3) / j;
            }
            pp = n * (z * p1 - p2) / (z * z - 1);
            double dz = p1 / pp;
            z -= dz;
            if (std::fabs(dz) < 1e-16) break;
        }
        x[i] = -z; x[n - 1 - i] = z;
        w[i] = w[n - 1 - i] = 2.0 / ((1 - z * z) * pp * pp);
    }
}

static int round8(int v) { return (v + 7) / 8 * 8; }

void grid_plan(Handle& h, int width, double sigma) {
    GridPlan& p = h.gp;
    p.W = width > 0 ? width : 14;
    if (p.W < 4 || p.W > 16) throw std::invalid_argument("grid kernel width must be in [4, 16]");
    if (!(sigma > 1.0)) sigma = 2.0;
    double sig_eff = 1e30;
    for (int d = 0; d < 3; d++) {
        const int K = h.kmax[d];
        int n = round8((int)std::ceil(sigma * (2 * K - 1)));
        n = std::max(n, std::max(24, round8(p.W + 8)));
        p.ng[d] = n;
        p.nb[d] = n / 8;
        sig_eff = std::min(sig_eff, (double)n / (2 * K - 1));
    }
    p.sigma = sig_eff;
    p.beta = 0.97 * kPi * (1.0 - 0.5 / sig_eff) * p.W;   // ES shape for this oversampling
    p.nbins = p.nb[0] * p.nb[1] * p.nb[2];
    p.KX = h.kmax[0]; p.KY = h.kmax[1]; p.KZ = h.kmax[2];
    p.NX = 2 * p.KX - 1; p.NY = 2 * p.KY - 1;
    // factorized stages: mode set k0 + j, j < J per axis (x, y: |n| < K; z: 0 <= nz < K)
    // alternative kernels of the same sums (cf_options.variants, A/B verification)
    p.dft8 = !(h.variants & CF_VARIANT_GEMM_DFT);
    p.spread_mfma = !(h.variants & CF_VARIANT_VECTOR_SPREAD);
    p.spread_mfma_all = (h.variants & CF_VARIANT_MFMA_SPREAD) != 0;
    p.interp2 = !(h.variants & CF_VARIANT_INTERP1);
    p.interp4 = !(h.variants & CF_VARIANT_INTERP2);
    // mixed precision on the vector spread (W <= 9): fp32 tap rows of 16 points (k_g_order_taps F32,
    // k_g_spread_tile TF): half the row bytes written and a third of the window bytes read
    p.taps_f32 = h.mixed && p.W <= 9 && !p.spread_mfma_all;
    for (int d = 0; d < 3; d++) {
        const int K = h.kmax[d], J = d == 2 ? K : 2 * K - 1, k0 = d == 2 ? 0 : -(K - 1);
        int mx = 0;
        for (int r = 0; r < 8; r++) {
            const int j0 = ((r - k0) % 8 + 8) % 8;
            p.rj[d][r] = j0;
            p.rc[d][r] = j0 < J ? (J - 1 - j0) / 8 + 1 : 0;
            mx = std::max(mx, p.rc[d][r]);
        }
        p.mt[d] = 0;
        for (int m : kDft8Mt)
            if (mx <= m) { p.mt[d] = m; break; }
        if (p.mt[d] == 0) p.dft8 = false;
    }
    // the fp32 real grid (mixed precision): every kernel that touches it has an fp32 form -- the
    // vector spread's store, the z row stages (k_g_dft8_zfwd / zinv, when their LDS fits: d8_fwd /
    // d8_inv) and k_g_interp4's halo staging; the sums stay fp64.  Half the grid's bytes written
    // by the spread and the synthesis and read by the analysis and the interpolation's halos.
    {
        const int Q = p.ng[2] / 8;
        int J = 0;
        for (int r = 0; r < 8; r++) J += p.rc[2][r];
        const bool zrow = (size_t)(kZR * Q * 5 + 8 * Q + kZR * J) * 16 <= 64 * 1024 &&
                          (size_t)(kZIR * Q * 4 + 8 * Q) * 16 <= 64 * 1024;
        p.grid_f32 = p.taps_f32 && p.W <= 8 && p.dft8 && zrow && p.interp2 && p.interp4;
    }
}

void grid_tables(const Handle& h, std::vector<double2> tw[3], std::vector<double2> tw8[3], std::vector<double> deconv[3]) {
    const GridPlan& p = h.gp;
    std::vector<double> gx, gw;
    gauss_legendre(200, gx, gw);
    for (int d = 0; d < 3; d++) {
        const int ng = p.ng[d], K = h.kmax[d];
        tw[d].resize((size_t)(2 * K - 1) * ng);
        for (int ni = 0; ni < 2 * K - 1; ni++) {
            const long n = ni - (K - 1);
            for (int g = 0; g < ng; g++) {
                long r = (n * g) % ng;
                if (r < 0) r += ng;
                const double th = 2.0 * kPi * (double)r / ng;
                tw[d][(size_t)ni * ng + g] = make_double2(std::cos(th), std::sin(th));
            }
        }
        deconv[d].resize(K);
        for (int n = 0; n < K; n++) {
            const double xi = (double)n / ng;
            double s = 0;
            for (size_t q = 0; q < gx.size(); q++) {
                const double t = 0.5 * p.W * gx[q];
                s += 0.5 * p.W * gw[q] * es_host(t, p.W, p.beta) * std::cos(2.0 * kPi * xi * t);
            }
            deconv[d][n] = 1.0 / s;
        }
    }
    // factorized stages: tw8[d] = twist [8 r][Q b] = w^{b k_r} (k_r = k0 + rj[r], the first mode
    // of class r), then [Q b][mt t] = w^{8bt}; exact angles (b k mod ng) like the tables above
    for (int d = 0; d < 3; d++) {
        if (!p.dft8) break;
        const int ng = p.ng[d], Q = ng / 8, K = h.kmax[d], mt = p.mt[d];
        const int k0 = d == 2 ? 0 : -(K - 1);
        auto w = [&](long e) {
            long m = e % ng;
            if (m < 0) m += ng;
            const double th = 2.0 * kPi * (double)m / ng;
            return make_double2(std::cos(th), std::sin(th));
        };
        tw8[d].resize((size_t)8 * Q + (size_t)Q * mt);
        for (int r = 0; r < 8; r++)
            for (int b = 0; b < Q; b++) tw8[d][(size_t)r * Q + b] = w((long)b * (k0 + p.rj[d][r]));
        for (int b = 0; b < Q; b++)
            for (int t = 0; t < mt; t++) tw8[d][(size_t)8 * Q + (size_t)b * mt + t] = w(8L * b * t);
    }
}

static double3 recip_vec(const Handle& h) {
    return make_double3(2 * kPi / h.box_L[0], 2 * kPi / h.box_L[1], 2 * kPi / h.box_L[2]);
}

void launch_grid_sort(Handle& h, const double* pos) {
    const GridPlan& p = h.gp;
    const int nown = h.hi - h.lo;
    const int3 ng = make_int3(p.ng[0], p.ng[1], p.ng[2]), nb = make_int3(p.nb[0], p.nb[1], p.nb[2]);
    const double3 L = make_double3(h.box_L[0], h.box_L[1], h.box_L[2]);
    // g_cnt is zero here: cleared at cf_create and by k_g_scatter of the previous evaluation
    // at least ~512 blocks of 256 atoms each round; up to 8 rounds per block (C5: 5, C3: 1)
    const int per = h.block_rounds() > 0 ? std::min(8, h.block_rounds()) : std::max(1, std::min(8, nown / (256 * 512)));
    hipLaunchKernelGGL(k_g_bin, dim3(nblk(nown, 256 * per)), dim3(256), 0, h.stream, h.lo, nown, pos, h.q, L, ng, p.W,
                       nb, h.g_srec, h.g_g0u, h.g_rank, h.g_cnt, h.g_xrange, h.e_ticket + kTicketGrid, h.g_start, per,
                       h.err_dev);
    hipLaunchKernelGGL(k_g_scatter, dim3(nblk(nown, 256)), dim3(256), 0, h.stream, nown, h.g_g0u, h.g_rank, h.g_start,
                       h.g_tmp, p.nbins, h.g_cnt, h.err_dev);
#define CF_OT(WT_, F_) hipLaunchKernelGGL((k_g_order_taps<WT_, F_>), dim3(nblk(p.nbins, kOtWaves)), dim3(256), 0, h.stream, \
                                          p.nbins, h.g_start, h.g_tmp, h.g_order, p.W, p.beta, ng, h.g_srec, h.g_g0u,  \
                                          h.g_taps, h.g_g0s, nown, h.err_dev)
    if (p.taps_f32) {   // fp32 taps (es_val_f), stored as fp32 rows: the mixed grid's vector spread
        if (p.W == 8) CF_OT(8, true);
        else CF_OT(0, true);
    } else if (p.W == 14) CF_OT(14, false);
    else if (p.W == 13) CF_OT(13, false);
    else if (p.W == 12) CF_OT(12, false);
    else if (p.W == 8) CF_OT(8, false);
    else CF_OT(0, false);
#undef CF_OT
}

#define CF_GRID_W_DISPATCH(W_, CALL) \
    switch (W_) {                    \
        case 4: CALL(4); break;      \
        case 5: CALL(5); break;      \
        case 6: CALL(6); break;      \
        case 7: CALL(7); break;      \
        case 8: CALL(8); break;      \
        case 9: CALL(9); break;      \
        case 10: CALL(10); break;    \
        case 11: CALL(11); break;    \
        case 12: CALL(12); break;    \
        case 13: CALL(13); break;    \
        case 14: CALL(14); break;    \
        case 15: CALL(15); break;    \
        default: CALL(16); break;    \
    }

void launch_grid_spread(Handle& h) {
    const GridPlan& p = h.gp;
    const int3 ng = make_int3(p.ng[0], p.ng[1], p.ng[2]), nb = make_int3(p.nb[0], p.nb[1], p.nb[2]);
#define CF_SPT(NS_, P_, TF_, GF_, FA_) hipLaunchKernelGGL((k_g_spread_tile<NS_, P_, TF_, GF_, FA_>), dim3(p.nbins), dim3(256), 0, \
                                                    h.stream, ng, nb, h.g_start, h.g_taps, h.g_g0s, h.g_grid, h.g_xrange, p.W)
    // the matrix-core form (16 x 8 x 8 tiles, 4 distinct x bins) for W > 9; at W <= 9 (the mixed
    // C5 grid) the vector form with its 8^3 tiles and 8 source bins measured faster (322 against
    // 330 us at C5: the 16-wide x tile doubles the zero-tap share of a narrow kernel)
    // (CF_VARIANT_MFMA_SPREAD selects the matrix form at any width, CF_VARIANT_VECTOR_SPREAD never)
    if (p.spread_mfma && nb.x >= 4 && (p.W > 9 || p.spread_mfma_all)) {
        const dim3 g((unsigned)((ng.x + 15) / 16 * nb.y * nb.z));
        if (p.W <= 9)
            hipLaunchKernelGGL((k_g_spread_mfma<2>), g, dim3(256), 0, h.stream, ng, nb, h.g_start, h.g_taps, h.g_g0s,
                               h.g_grid, h.g_xrange, p.W);
        else
            hipLaunchKernelGGL((k_g_spread_mfma<3>), g, dim3(256), 0, h.stream, ng, nb, h.g_start, h.g_taps, h.g_g0s,
                               h.g_grid, h.g_xrange, p.W);
        return;
    }
    // a first tap in bin B reaches tiles B .. B + NS - 1: NS = 2 when W <= 9 (8 source bins per
    // tile instead of 27).  Passes of 32 atoms at W = 14 (64 / 128 measured slower at C3)
    if (p.grid_f32) CF_SPT(2, 64, true, true, true);
    else if (p.taps_f32) CF_SPT(2, 64, true, false, false);
    else if (p.W <= 9) CF_SPT(2, 64, false, false, false);
    else CF_SPT(3, 32, false, false, false);
#undef CF_SPT
}

template <bool AREAL, bool CREAL>
static void cgemm(Handle& h, CGemm g, int xdim = 0, int xdiv = 1) {
    // multi-rank: tiles outside the rank's x-slab exit at once, so only about the slab's share
    // of the blocks (its owned fraction of the planes plus the W - 1 halo) counts as work
    double active = 1.0;
    if (h.g_xrange && xdim) {
        g.xdim = xdim; g.xdiv = xdiv; g.xr = h.g_xrange; g.W = h.gp.W; g.ngx = h.gp.ng[0];
        if (xdim != 3 && h.n > 0)
            active = std::min(1.0, (double)(h.hi - h.lo) / h.n + (double)(h.gp.W - 1) / h.gp.ng[0]);
    }
    // block tile: the least padded work among the shapes below (kmax = 31 or 65 pads a 64-wide
    // tile to twice its width; 80 fits 65 closely) among the shapes that give every CU a block,
    // or the shape with the most blocks when none does.  (A 48 x 64 tile of 1 x 4 waves for the
    // 129-row stages: less padding than 32 x 32 but slower, 100 against 92 us at C5.)
    constexpr int kShapes = 5;
    const int bms[kShapes] = {64, 64, 32, 32, 64}, bns[kShapes] = {64, 32, 64, 32, 80};
    int best = -1;
    long best_work = 0, best_blocks = 0;
    for (int c = 0; c < kShapes; c++) {
        const long tm = (g.M + bms[c] - 1) / bms[c], tn = (g.N + bns[c] - 1) / bns[c];
        const long blocks = tm * tn, work = tm * bms[c] * tn * bns[c];
        const bool ok = blocks * active >= 256, best_ok = best >= 0 && best_blocks * active >= 256;
        if (best < 0 || (ok && !best_ok) || (ok && best_ok && work < best_work) ||
            (!ok && !best_ok && blocks > best_blocks)) {
            best = c; best_work = work; best_blocks = blocks;
        }
    }
    const dim3 grid((unsigned)best_blocks);
    switch (best) {
        case 0: hipLaunchKernelGGL((k_g_cgemm<64, 64, 2, AREAL, CREAL>), grid, dim3(256), 0, h.stream, g); break;
        case 1: hipLaunchKernelGGL((k_g_cgemm<64, 32, 2, AREAL, CREAL>), grid, dim3(256), 0, h.stream, g); break;
        case 2: hipLaunchKernelGGL((k_g_cgemm<32, 64, 2, AREAL, CREAL>), grid, dim3(256), 0, h.stream, g); break;
        case 3: hipLaunchKernelGGL((k_g_cgemm<32, 32, 2, AREAL, CREAL>), grid, dim3(256), 0, h.stream, g); break;
        default: hipLaunchKernelGGL((k_g_cgemm<64, 80, 4, AREAL, CREAL>), grid, dim3(256), 0, h.stream, g); break;
    }
}

// stage geometry (the same for analysis and synthesis along an axis)
static Dft8 d8_stage(const Handle& h, int axis) {
    const GridPlan& p = h.gp;
    const int ngx = p.ng[0], ngy = p.ng[1], ngz = p.ng[2], KZ = p.KZ, NY = p.NY;
    const long NYKZ = (long)NY * KZ;
    Dft8 d{};
    d.Q = p.ng[axis] / 8;
    for (int r = 0; r < 8; r++) { d.rj[r] = p.rj[axis][r]; d.rc[r] = p.rc[axis][r]; }
    d.xr = h.g_xrange; d.W = p.W; d.ngx = ngx;
    if (axis == 2) {          // rows (x, y): grid[row][z] <-> t1[row][nz]
        d.nseq = ngx * ngy; d.sdiv = 1;
        d.s1 = ngz; d.s0 = 0; d.sn = 1;
        d.c1 = KZ; d.c0 = 0; d.cj = 1;
        d.xmode = 1; d.xdiv = ngy;
    } else if (axis == 1) {   // (x, nz): t1[x][y][nz] <-> t2[x][ny][nz]
        d.nseq = ngx * KZ; d.sdiv = KZ;
        d.s1 = (long)ngy * KZ; d.s0 = 1; d.sn = KZ;
        d.c1 = NYKZ; d.c0 = 1; d.cj = KZ;
        d.xmode = 1; d.xdiv = KZ;
    } else {                  // r = (ny, nz): t2[x][r] <-> b[nx][r]
        d.nseq = (int)NYKZ; d.sdiv = (int)NYKZ;
        d.s1 = 0; d.s0 = 1; d.sn = NYKZ;
        d.c1 = 0; d.c0 = 1; d.cj = NYKZ;
        d.xmode = 2; d.xdiv = 1;
    }
    return d;
}

#define CF_D8_MT(MT_, CALL) \
    switch (MT_) {          \
        case 4: CALL(4); break;   \
        case 8: CALL(8); break;   \
        case 9: CALL(9); break;   \
        case 16: CALL(16); break; \
        default: CALL(17); break; \
    }

static void d8_fwd(Handle& h, int axis, const void* in, void* out, const Coef* cf = nullptr) {
    Dft8 d = d8_stage(h, axis);
    d.in = in; d.out = out;
    const int nb = nblk(d.nseq, kD8Seq);
    const double2* twist = h.g_tw8[axis];
    const double2* tq = twist + 8 * d.Q;
    const int J = d.rc[0] + d.rc[1] + d.rc[2] + d.rc[3] + d.rc[4] + d.rc[5] + d.rc[6] + d.rc[7];
    const size_t lds = (size_t)(kZR * d.Q * 5 + 8 * d.Q + kZR * J) * sizeof(double2);
    if (axis == 2 && lds <= 64 * 1024) {   // grid rows: the row kernel (4 waves, each a quarter of b)
        const dim3 g((unsigned)nblk(d.nseq, kZR));
#define CF_D8Z(MT_)                                                                                     \
    if (h.gp.grid_f32) hipLaunchKernelGGL((k_g_dft8_zfwd<MT_, 4, true>), g, dim3(256), lds, h.stream, d, twist, tq); \
    else hipLaunchKernelGGL((k_g_dft8_zfwd<MT_, 4, false>), g, dim3(256), lds, h.stream, d, twist, tq)
        CF_D8_MT(h.gp.mt[axis], CF_D8Z)
#undef CF_D8Z
        return;
    }
    // blocks of 16 sequences x 8 classes for the mid-sized y and x stages (C5: 44.9 -> 35.2 us
    // per stage); at C3's sizes (< 128 blocks of 64) and for the synthesis the 64-sequence
    // blocks measured faster (10.0 against 10.4 us, 6.8 against 7.7 us)
    const bool small = nb >= 128 && nb < 2048;
    const int seq = small ? 16 : 64;
    const dim3 grid((unsigned)nblk(d.nseq, seq));
    const size_t lds2 = (size_t)(kD8BC * (axis == 2 ? 5 : 8) * (seq + 1) + 8 * d.Q) * sizeof(double2);
    if (cf) {   // the x stage with the coefficient pass fused (one rank): its blocks' energy partials
        h.e_rec_nblk = (int)grid.x;
#define CF_D8FC_(MT_, SEQ_) \
    hipLaunchKernelGGL((k_g_dft8_fwd<MT_, true, SEQ_, true>), grid, dim3(8 * SEQ_), lds2, h.stream, d, twist, tq, *cf)
#define CF_D8FC(MT_) if (small) CF_D8FC_(MT_, 16); else CF_D8FC_(MT_, 64);
        CF_D8_MT(h.gp.mt[axis], CF_D8FC)
#undef CF_D8FC
#undef CF_D8FC_
        return;
    }
#define CF_D8F_(MT_, CIN_, SEQ_) \
    hipLaunchKernelGGL((k_g_dft8_fwd<MT_, CIN_, SEQ_>), grid, dim3(8 * SEQ_), lds2, h.stream, d, twist, tq)
#define CF_D8F(MT_)                                         \
    if (axis == 2) { if (small) CF_D8F_(MT_, false, 16); else CF_D8F_(MT_, false, 64); } \
    else { if (small) CF_D8F_(MT_, true, 16); else CF_D8F_(MT_, true, 64); }
    CF_D8_MT(h.gp.mt[axis], CF_D8F)
#undef CF_D8F
#undef CF_D8F_
}

static void d8_inv(Handle& h, int axis, const void* in, void* out, const Coef* cf = nullptr) {
    Dft8 d = d8_stage(h, axis);
    d.in = in; d.out = out;
    if (axis == 0) d.xmode = 0;   // synthesis along x: every plane is written (inputs are complete)
    const size_t lds = (size_t)(kZIR * d.Q * 4 + 8 * d.Q) * sizeof(double2);
    if (axis == 2 && lds <= 64 * 1024) {   // grid rows: the row kernel (2 waves, each half of b)
        const double2* tw0 = h.g_tw8[axis];
        const double2* tq0 = tw0 + 8 * d.Q;
        const dim3 g((unsigned)nblk(d.nseq, kZIR));
#define CF_D8ZI(MT_)                                                                                    \
    if (h.gp.grid_f32) hipLaunchKernelGGL((k_g_dft8_zinv<MT_, 2, true>), g, dim3(128), lds, h.stream, d, tw0, tq0); \
    else hipLaunchKernelGGL((k_g_dft8_zinv<MT_, 2, false>), g, dim3(128), lds, h.stream, d, tw0, tq0)
        CF_D8_MT(h.gp.mt[axis], CF_D8ZI)
#undef CF_D8ZI
        return;
    }
    // 64-sequence blocks (16-sequence blocks measured slower for the synthesis: 7.7 against 6.8 us
    // per y stage at C3, 40.5 against 36.4 at C5)
    const int nb = nblk(d.nseq, kD8Seq), nchunks = (d.Q + kD8BC - 1) / kD8BC;
    const dim3 grid((unsigned)nb, (unsigned)std::max(1, std::min(nchunks, 2048 / nb)));
    const double2* twist = h.g_tw8[axis];
    const double2* tq = twist + 8 * d.Q;
    const size_t lds2 = (size_t)(kD8BC * 8 * (kD8Seq + 1) + 8 * d.Q + d.Q * h.gp.mt[axis]) * sizeof(double2);
    if (cf) {   // the x stage with the coefficient pass (several ranks): its x-blocks' energy partials
        h.e_rec_nblk = (int)grid.x;
#define CF_D8IC(MT_) \
    hipLaunchKernelGGL((k_g_dft8_inv<MT_, false, kD8Seq, true>), grid, dim3(8 * kD8Seq), lds2, h.stream, d, twist, tq, *cf)
        CF_D8_MT(h.gp.mt[axis], CF_D8IC)
#undef CF_D8IC
        return;
    }
#define CF_D8I(MT_)                                                                                            \
    if (axis == 2) hipLaunchKernelGGL((k_g_dft8_inv<MT_, true, kD8Seq>), grid, dim3(8 * kD8Seq), lds2, h.stream, d, twist, tq); \
    else hipLaunchKernelGGL((k_g_dft8_inv<MT_, false, kD8Seq>), grid, dim3(8 * kD8Seq), lds2, h.stream, d, twist, tq)
    CF_D8_MT(h.gp.mt[axis], CF_D8I)
#undef CF_D8I
}

// one rank with the factorized stages: the coefficient pass rides on the forward x stage (there
// is no all-reduce of B(n) between them); several ranks reduce B(n) first (launch_grid_coeffs)
static bool coef_fused(const Handle& h) { return h.gp.dft8 && h.world == 1; }

static Coef coef_args(const Handle& h) {
    const GridPlan& p = h.gp;
    const double V = h.box_L[0] * h.box_L[1] * h.box_L[2];
    return Coef{p.KX, p.KY, p.KZ, recip_vec(h), 4.0 / V * kPi * h.ke, 1.0 / (h.alpha * h.alpha), h.g_deconv[0],
                h.g_deconv[1], h.g_deconv[2], h.e_rec_part};
}

void launch_grid_dft_fwd(Handle& h) {
    const GridPlan& p = h.gp;
    if (p.dft8) {
        d8_fwd(h, 2, h.g_grid, h.g_t1);
        d8_fwd(h, 1, h.g_t1, h.g_t2);
        if (coef_fused(h)) {
            const Coef cf = coef_args(h);
            d8_fwd(h, 0, h.g_t2, h.g_b, &cf);
        } else {
            d8_fwd(h, 0, h.g_t2, h.g_b);
        }
        return;
    }
    const int ngx = p.ng[0], ngy = p.ng[1], ngz = p.ng[2], KZ = p.KZ, NY = p.NY, NX = p.NX;
    const long NYKZ = (long)NY * KZ;
    const double2* tzh = h.g_tw[2] + (size_t)(KZ - 1) * ngz;   // e^{i th nz z}, nz >= 0: tzh[nz * ngz + z]
    // z (real rows -> half spectrum): t1[row][nz] = sum_z grid[row][z] Tz[nz][z], row = (x, y)
    cgemm<true, false>(h, CGemm{ngx * ngy, KZ, ngz, h.g_grid, ngz, 1, tzh, 1, 0, ngz, h.g_t1, KZ, 0, 1, KZ}, 1, ngy);
    // y: t2[x][ny][nz] = sum_y Ty[ny][y] t1[x][y][nz], columns n = (x, nz)
    cgemm<false, false>(h, CGemm{NY, ngx * KZ, ngy, h.g_tw[1], ngy, 1, h.g_t1, KZ, (long)ngy * KZ, 1, h.g_t2, KZ, NYKZ,
                                 1, KZ}, 2, KZ);
    // x: b[nx][r] = sum_x Tx[nx][x] t2[x][r], r = (ny, nz)
    cgemm<false, false>(h, CGemm{NX, (int)NYKZ, ngx, h.g_tw[0], ngx, 1, h.g_t2, NYKZ, 0, 1, h.g_b, NYKZ, 0, 1,
                                 (int)NYKZ}, 3);
}

double* grid_reduce_buffer(Handle& h, int64_t* count) {
    *count = (int64_t)2 * h.gp.NX * h.gp.NY * h.gp.KZ;
    return reinterpret_cast<double*>(h.g_b);
}

void launch_grid_coeffs(Handle& h, int include_energy, bool inverse_follows) {
    h.coef_inv = 0;
    if (coef_fused(h)) return;   // done by the forward x stage (launch_grid_dft_fwd)
    if (h.gp.dft8 && inverse_follows) {   // several ranks: done by the inverse x stage (launch_grid_dft_inv)
        h.coef_inv = include_energy ? 2 : 1;
        return;
    }
    const GridPlan& p = h.gp;
    const double V = h.box_L[0] * h.box_L[1] * h.box_L[2];
    const double cst = 4.0 / V * kPi * h.ke;   // RCK:517
    const int total = p.NX * p.NY * p.KZ;
    h.e_rec_nblk = nblk(total, 256);
    hipLaunchKernelGGL(k_g_coeffs, dim3(h.e_rec_nblk), dim3(256), 0, h.stream, p.KX, p.KY, p.KZ, recip_vec(h), cst,
                       1.0 / (h.alpha * h.alpha), h.g_deconv[0], h.g_deconv[1], h.g_deconv[2], h.g_b, h.e_rec_part,
                       include_energy);
}

void launch_grid_dft_inv(Handle& h) {
    const GridPlan& p = h.gp;
    if (p.dft8) {
        if (h.coef_inv) {   // the coefficient pass on the all-reduced B(n), as the x stage loads it
            Coef cf = coef_args(h);
            if (h.coef_inv == 1) cf.e_part = nullptr;
            h.coef_inv = 0;
            d8_inv(h, 0, h.g_b, h.g_t2, &cf);
        } else {
            d8_inv(h, 0, h.g_b, h.g_t2);
        }
        d8_inv(h, 1, h.g_t2, h.g_t1);
        d8_inv(h, 2, h.g_t1, h.g_grid);
        return;
    }
    const int ngx = p.ng[0], ngy = p.ng[1], ngz = p.ng[2], KZ = p.KZ, NY = p.NY, NX = p.NX;
    const long NYKZ = (long)NY * KZ;
    const double2* tzh = h.g_tw[2] + (size_t)(KZ - 1) * ngz;
    // x: t2[x][r] = sum_nx Tx[nx][x] f[nx][r]
    cgemm<false, false>(h, CGemm{ngx, (int)NYKZ, NX, h.g_tw[0], 1, ngx, h.g_b, NYKZ, 0, 1, h.g_t2, NYKZ, 0, 1,
                                 (int)NYKZ}, 1, 1);
    // y: t1[x][y][nz] = sum_ny Ty[ny][y] t2[x][ny][nz], columns n = (x, nz)
    cgemm<false, false>(h, CGemm{ngy, ngx * KZ, NY, h.g_tw[1], 1, ngy, h.g_t2, KZ, NYKZ, 1, h.g_t1, KZ,
                                 (long)ngy * KZ, 1, KZ}, 2, KZ);
    // z (half spectrum -> real rows): grid[row][z] = Re sum_nz t1[row][nz] Tz[nz][z], row = (x, y)
    cgemm<false, true>(h, CGemm{ngx * ngy, ngz, KZ, h.g_t1, KZ, 1, tzh, ngz, 0, 1, h.g_grid, ngz, 0, 1, ngz}, 1, ngy);
}

void launch_grid_interp(Handle& h, bool split) {
    const GridPlan& p = h.gp;
    const int3 ng = make_int3(p.ng[0], p.ng[1], p.ng[2]), nb = make_int3(p.nb[0], p.nb[1], p.nb[2]);
    const double3 gs = make_double3(p.ng[0] / h.box_L[0], p.ng[1] / h.box_L[1], p.ng[2] / h.box_L[2]);
    const size_t R = 7 + p.W;
    // W <= 8: four atoms per wave (k_g_interp4; fp32 taps in mixed precision); else two (k_g_interp2);
    // CF_VARIANT_INTERP1: one (k_g_interp)
#define CF_INTERP(W_)                                                                                               \
    hipLaunchKernelGGL(!p.interp2 ? k_g_interp<W_>                                                                 \
                       : (W_ <= 8 && p.interp4) ? (p.grid_f32 ? k_g_interp4<(W_ <= 8 ? W_ : 8), true, true>            \
                                                   : h.mixed ? k_g_interp4<(W_ <= 8 ? W_ : 8), true, false>            \
                                                             : k_g_interp4<(W_ <= 8 ? W_ : 8), false, false>)          \
                                                : k_g_interp2<W_>,                                                     \
                       dim3(p.nbins), dim3(kInterpThreads),                                                         \
                       (!p.interp2 || (W_ <= 8 && p.interp4) ? R * R : (size_t)interp_plane_stride<W_>()) * R *     \
                           sizeof(double),                                                                          \
                       h.stream, ng, nb, h.g_start, h.g_g0s, h.g_srec, p.beta, gs, h.g_grid, h.lo,                   \
                       split ? h.dedq_rec : h.dedq, split ? h.f_rec : h.f_part, split ? 1 : 0)
    CF_GRID_W_DISPATCH(p.W, CF_INTERP)
#undef CF_INTERP
}

}  // namespace cf
