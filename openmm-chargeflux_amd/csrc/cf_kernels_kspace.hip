// cf_kernels_kspace.hip — reciprocal-space Ewald sum on fp64 MFMA (gfx950).
//
// Reference: the half-space triple loop of ReferenceCoulKernels.cpp:513-556 (RCK),
// O(N*K) with two cos/sin passes per (atom, k).  Here the same sums are evaluated in a
// separable form:
//
//   e^{i k.r} = X[nx] * Y[ny] * Z[nz]  with X = e^{i nx gx x}, Y = e^{i ny gy y},
//   Z[+-nz] = c_nz +- i s_nz.
//
//   structure factor  S(nx,ny,+-nz) = SC +- i SS,
//        SC = sum_i (q X Y)_i c_nz(i),  SS = sum_i (q X Y)_i s_nz(i)
//      -> a real GEMM  D[(combo,re|im)][(nz,c|s)] = sum_atoms w * cs   (k_sfac)
//   potential/force   T_i = sum_(nx,ny) X Y [ sum_nz P c + Q s ]  (P,Q from S^)
//      -> a real GEMM  D[(combo,part)][atom]      = sum_(nz,c|s) coef * cs (k_force)
//
// Both GEMMs run on v_mfma_f64_16x16x4_f64 (fp64 in, fp64 accumulate — the same
// precision as the reference's serial double loop).  The VALU builds the operands
// (complex products, phase recurrences) beside the matrix pipe.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <stdexcept>

#include "cf_internal.h"

namespace cf {

typedef double d4 __attribute__((ext_vector_type(4)));
// native 2-vector for staging registers (HIP's double2 struct copies lower to memcpy
// through a private alloca, i.e. scratch memory, when the source address is a select)
typedef double v2d __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

static inline int nblk(int64_t n, int b) { return (int)((n + b - 1) / b); }

// ---------------------------------------------------------------------------------
// per-atom phase tables (owned atoms, rows padded to a multiple of the S-pass tile):
//   XQ[ia][nx]  = q e^{i nx gx x}                      [npad][KX]   double2
//   Y [ia][iy]  = e^{i ny gy y}, ny = iy-(KY-1)         [npad][NYP]  double2
//   CS[nb][ia][jj] = (cos, sin)(nz gz z), j = 2nz+cs = 64nb+jj   [NB][npad][CSW] double
// One lane per (atom, table entry).
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_tables(int lo, int nown, int npad, KGeom g, double3 rec,
                                                const double* __restrict__ pos, const double* __restrict__ q,
                                                double2* __restrict__ xq, double2* __restrict__ ty,
                                                double* __restrict__ cs) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    int ncs2 = g.NB * g.CSW / 2;
    int ncol = g.KX + g.NYP + ncs2;
    if (t >= nown * ncol) return;
    int ia = t / ncol, c = t % ncol;
    int i = lo + ia;
    if (c < g.KX) {
        double s, co;
        sincos((c * rec.x) * pos[3 * i], &s, &co);
        double qi = q[i];
        xq[(size_t)ia * g.KX + c] = make_double2(qi * co, qi * s);
    } else if (c < g.KX + g.NYP) {
        int iy = c - g.KX;
        double2 v = make_double2(0, 0);
        if (iy < g.NY) {
            double s, co;
            sincos(((iy - (g.KY - 1)) * rec.y) * pos[3 * i + 1], &s, &co);
            v = make_double2(co, s);
        }
        ty[(size_t)ia * g.NYP + iy] = v;
    } else {
        int nz = c - g.KX - g.NYP;  // column pair j = 2nz
        double2 v = make_double2(0, 0);
        if (nz < g.KZ) {
            double s, co;
            sincos((nz * rec.z) * pos[3 * i + 2], &s, &co);
            v = make_double2(co, s);
        }
        int j = 2 * nz, nb = j / g.CSW, jj = j % g.CSW;
        *reinterpret_cast<double2*>(cs + ((size_t)nb * npad + ia) * g.CSW + jj) = v;
    }
}

// ---------------------------------------------------------------------------------
// S-pass: structure-factor GEMM over an atom chunk.
//   workgroup = 8 waves; wave w owns combo groups g0+2w, g0+2w+1 (16 combos each,
//   re & im m-tiles) x NT column tiles (<=64 columns) -> 16 accumulator tiles.
//   Atom tiles (TA atoms) of CS / Y / XQ are staged in LDS, double-buffered through
//   registers (load next tile before the MFMAs, write it to LDS after).  The three
//   table slices of a tile are contiguous in HBM, so staging is a linear copy.
// ---------------------------------------------------------------------------------
constexpr int kSWaves = 8;
constexpr int kSThreads = kSWaves * 64;
constexpr int kSMaxV = 8;   // staged double2 per lane per tile

__host__ __device__ inline int cs_lds_stride(int csw) {
    // row stride (doubles) == 16 mod 32: rows a and a+1 land on opposite bank halves
    return csw + ((16 - csw % 32) + 32) % 32;
}

struct SArgs {
    KGeom g;
    int nown, npad, chunk_atoms, wg_groups, nbk0;
    const double* cs; const double2* ty; const double2* xq;
    double* slab;
};

// NT column tiles (16 columns each) of column block nbk0 + blockIdx.x / wg_groups; TA
// atoms per LDS tile.  Both compile-time so the k-step loop is straight-line code and
// the scheduler can issue the next k-step's LDS operands under the current MFMAs.
template <int NT, int TA>
__global__ void __launch_bounds__(kSThreads) k_sfac(SArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const KGeom g = a.g;
    const int wgx = blockIdx.x % a.wg_groups;
    const int nbk = a.nbk0 + blockIdx.x / a.wg_groups;
    const int chunk = blockIdx.y;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int r = lane & 15, kq = lane >> 4;

    const int ngroups = g.ngroups();
    const int g0 = wgx * 16;
    const int col0 = nbk * 64;
    const int a_begin = chunk * a.chunk_atoms;                 // owned index, multiple of TA
    const int a_end = min(a.nown, a_begin + a.chunk_atoms);
    if (a_begin >= a_end) return;  // whole workgroup uniform

    // LDS carve (per buffer): CS [TA][csl] | Y [TA][NYP] (double2) | XQ [TA][KX] (double2)
    const int csl = cs_lds_stride(g.CSW);
    const int cs_d = TA * csl;
    const int y_d = TA * g.NYP * 2;
    const int xq_d = TA * g.KX * 2;
    const int buf_d = cs_d + y_d + xq_d;
    const int half = g.CSW / 2;
    const int ncs2 = TA * half, ny2 = TA * g.NYP, nxq2 = TA * g.KX;

    const int n_el = ncs2 + ny2 + nxq2;
    // branch-free staging: every lane loads a valid address (elements past the tile
    // re-read the last XQ entry and are never stored), so the loads issue back to back
#define CF_STAGE_LOAD(tile_a0, h)                                                                           \
    {                                                                                                       \
        const double2* csb = reinterpret_cast<const double2*>(a.cs + ((size_t)nbk * a.npad + (tile_a0)) * g.CSW); \
        const double2* yb = a.ty + (size_t)(tile_a0) * g.NYP;                                               \
        const double2* xb = a.xq + (size_t)(tile_a0) * g.KX;                                                \
        _Pragma("unroll") for (int u = 0; u < kSMaxV / 2; u++) {                                            \
            int e = threadIdx.x + ((h) * (kSMaxV / 2) + u) * kSThreads;                                     \
            const double2* src = e < ncs2 ? csb + e                                                         \
                               : (e < ncs2 + ny2 ? yb + (e - ncs2) : xb + min(e - ncs2 - ny2, nxq2 - 1));   \
            reg[u] = *reinterpret_cast<const v2d*>(src);                                                    \
        }                                                                                                   \
    }
#define CF_STAGE_STORE(buf, h)                                                                              \
    {                                                                                                       \
        double* base = lds + (buf) * buf_d;                                                                 \
        _Pragma("unroll") for (int u = 0; u < kSMaxV / 2; u++) {                                            \
            int e = threadIdx.x + ((h) * (kSMaxV / 2) + u) * kSThreads;                                     \
            int at = e / half;                                                                              \
            int dst = e < ncs2 ? at * csl + 2 * (e - at * half) : cs_d + 2 * (e - ncs2);                    \
            if (e < n_el) *reinterpret_cast<v2d*>(base + dst) = reg[u];                                     \
        }                                                                                                   \
    }

    // wave's combo groups; a group past ngroups reads row 0 and contributes zero weight
    int gq[2], gnx[2], giy[2];
    double gm[2];
#pragma unroll
    for (int gi = 0; gi < 2; gi++) {
        gq[gi] = g0 + 2 * wave + gi;
        bool v = gq[gi] < ngroups;
        gm[gi] = v ? 1.0 : 0.0;
        gnx[gi] = v ? gq[gi] / g.NYB : 0;
        giy[gi] = v ? (gq[gi] % g.NYB) * 16 + r : 0;
    }

    d4 acc[2][2][NT];
#pragma unroll
    for (int gi = 0; gi < 2; gi++)
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int nt = 0; nt < NT; nt++) acc[gi][p][nt] = (d4){0, 0, 0, 0};

    const int ntiles = (a_end - a_begin + TA - 1) / TA;
    // staging of the next tile runs in two halves, each loaded before and stored after
    // half of the current tile's k-steps (16 staging VGPRs instead of 32)
    v2d reg[kSMaxV / 2];
    CF_STAGE_LOAD(a_begin, 0);
    CF_STAGE_STORE(0, 0);
    CF_STAGE_LOAD(a_begin, 1);
    CF_STAGE_STORE(0, 1);
    __syncthreads();
    constexpr int KSTEPS = TA / 4;
    for (int tt = 0; tt < ntiles; tt++) {
        const int buf = tt & 1;
        const bool more = tt + 1 < ntiles;
        const int next_a0 = a_begin + (tt + 1) * TA;
        const double* cs_l = lds + buf * buf_d;
        const double2* y_l = reinterpret_cast<const double2*>(cs_l + cs_d);
        const double2* xq_l = reinterpret_cast<const double2*>(cs_l + cs_d + y_d);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if (more) CF_STAGE_LOAD(next_a0, h);
#pragma unroll
            for (int t = h * (KSTEPS / 2); t < (h ? KSTEPS : KSTEPS / 2); t++) {
                const int at = 4 * t + kq;
                double b[NT];
#pragma unroll
                for (int nt = 0; nt < NT; nt++) b[nt] = cs_l[at * csl + nt * 16 + r];
#pragma unroll
                for (int gi = 0; gi < 2; gi++) {
                    double2 x = xq_l[at * g.KX + gnx[gi]];
                    double2 y = y_l[at * g.NYP + giy[gi]];
                    double wr = (x.x * y.x - x.y * y.y) * gm[gi];
                    double wi = (x.x * y.y + x.y * y.x) * gm[gi];
#pragma unroll
                    for (int nt = 0; nt < NT; nt++) {
                        acc[gi][0][nt] = mfma64(wr, b[nt], acc[gi][0][nt]);
                        acc[gi][1][nt] = mfma64(wi, b[nt], acc[gi][1][nt]);
                    }
                }
            }
            if (more) CF_STAGE_STORE(buf ^ 1, h);
        }
        __syncthreads();
    }

    // write partial slab: slab[chunk][part][slot][NZP]
    const int nslots = g.nslots();
#pragma unroll
    for (int gi = 0; gi < 2; gi++) {
        if (gq[gi] >= ngroups) continue;
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int nt = 0; nt < NT; nt++) {
#pragma unroll
                for (int v = 0; v < 4; v++) {
                    int row = kq + 4 * v;
                    int slot = gq[gi] * 16 + row;
                    size_t off = (((size_t)chunk * 2 + p) * nslots + slot) * g.NZP + col0 + nt * 16 + r;
                    a.slab[off] = acc[gi][p][nt][v];
                }
            }
    }
}

#undef CF_STAGE_LOAD
#undef CF_STAGE_STORE

__global__ void __launch_bounds__(256) k_sfac_reduce(int64_t count, int nchunks, const double* __restrict__ slab,
                                                     double* __restrict__ out) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= count) return;
    double s = 0;
    for (int c = 0; c < nchunks; c++) s += slab[(size_t)c * count + e];
    out[e] = s;
}

// ---------------------------------------------------------------------------------
// coefficients: for every (nx, ny, nz>=0) form S(+-nz), the reference's half-space
// weights w = 2*c*exp(-k^2/4a^2)/k^2 (RCK:517,528), the energy c*eak*|S|^2
// (RCK:549-551) and the force-pass MFMA A-fragments (P, Q, Pz, Qz).
// ---------------------------------------------------------------------------------
// coefficient element (m-tile mt, k-step ks, A-lane l) in the k_coeffs output
__host__ __device__ inline size_t coef_index(int mt, int ks, int l, int KS) {
    // k-step pair p = ks/2 of m-tile mt is the 64-lane double2 block (mt*KS/2 + p)
    return (((size_t)mt * KS + (ks & ~1)) * 32 + l) * 2 + (ks & 1);
}

__device__ __forceinline__ bool in_half_space(int nx, int ny, int nz) {
    // RCK:519-556: nx=0 -> ny>=0, and ny=0 -> nz>=1
    if (nx > 0) return true;
    if (ny > 0) return true;
    if (ny < 0) return false;
    return nz > 0;
}

__global__ void __launch_bounds__(256) k_coeffs(KGeom g, double3 rec, double cst, double one_4a2,
                                                const double* __restrict__ sred, double* __restrict__ coef,
                                                double* __restrict__ e_part, int include_energy) {
    __shared__ double red[256];
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    int total = g.KX * g.NY * g.KZ;
    double e = 0;
    if (t < total) {
        int nz = t % g.KZ;
        int iy = (t / g.KZ) % g.NY;
        int nx = t / (g.KZ * g.NY);
        int ny = iy - (g.KY - 1);
        int nslots = g.nslots();
        int slot = nx * g.NYP + iy;
        double scr = sred[(size_t)slot * g.NZP + 2 * nz], ssr = sred[(size_t)slot * g.NZP + 2 * nz + 1];
        double sci = sred[((size_t)nslots + slot) * g.NZP + 2 * nz];
        double ssi = sred[((size_t)nslots + slot) * g.NZP + 2 * nz + 1];
        double kx = nx * rec.x, ky = ny * rec.y, kz = nz * rec.z;
        double k2 = kx * kx + ky * ky + kz * kz;
        double w = 0.0;
        if (k2 > 0) w = 2.0 * cst * exp(-k2 * 0.25 * one_4a2) / k2;
        // S(+nz) and S(-nz)
        double pr = scr - ssi, pim = sci + ssr;   // S+
        double mr = scr + ssi, mim = sci - ssr;   // S-
        double hp_r = 0, hp_i = 0, hm_r = 0, hm_i = 0;  // S^ = w conj(S), zero outside the half space
        if (in_half_space(nx, ny, nz)) {
            hp_r = w * pr; hp_i = -w * pim;
            if (include_energy) e += 0.5 * w * (pr * pr + pim * pim);
        }
        if (nz > 0 && in_half_space(nx, ny, -nz)) {
            hm_r = w * mr; hm_i = -w * mim;
            if (include_energy) e += 0.5 * w * (mr * mr + mim * mim);
        }
        double Pr, Pi, Dr, Di;
        if (nz > 0) { Pr = hp_r + hm_r; Pi = hp_i + hm_i; Dr = hp_r - hm_r; Di = hp_i - hm_i; }
        else { Pr = hp_r; Pi = hp_i; Dr = 0; Di = 0; }
        double Qr = -Di, Qi = Dr;                 // Q  = i D
        double Pzr = nz * Dr, Pzi = nz * Di;      // Pz = nz D
        double Qzr = -nz * Pi, Qzi = nz * Pr;     // Qz = i nz P
        // A fragment: combos flattened c = nx*NY + iy, m-tile mt = c/4, row = (c%4) + 4*part, k = j
        // (k-step pairs interleaved per lane, coef_index)
        int cflat = nx * g.NY + iy;
        int mt = cflat / 4, qrow = cflat % 4;
        int KS = g.nksteps();
        double vc[4] = {Pr, Pi, Pzr, Pzi}, vs[4] = {Qr, Qi, Qzr, Qzi};
#pragma unroll
        for (int part = 0; part < 4; part++) {
            int row = qrow + 4 * part;
            int jc = 2 * nz, js = 2 * nz + 1;
            coef[coef_index(mt, jc / 4, (jc % 4) * 16 + row, KS)] = vc[part];
            coef[coef_index(mt, js / 4, (js % 4) * 16 + row, KS)] = vs[part];
        }
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
// force pass: per atom, T0 = Re sum S^ e^{ik.r} (-> dE/dq_recip) and
// Ta = Im sum S^ n_a e^{ik.r} (-> F_a = q g_a Ta), RCK:538-547.
//   workgroup = 8 waves; wave owns NA 16-atom tiles; B operand (CS columns of its
//   atoms) lives in registers for the whole kernel; the A operand (coefficients) is
//   streamed through an LDS double buffer shared by the 8 waves (kFMB m-tiles per
//   stage), and each wave prefetches the next m-tile's A fragments into registers
//   while the MFMAs of the current one run (no LDS latency on the MFMA chain).
//   Coefficients hold k-step pairs interleaved per lane -> one ds_read_b128 feeds
//   two k-steps.  Accumulator lane (qg, atom) receives the 4 parts (U0r,U0i,Uzr,Uzi)
//   of combo 4*mt+qg -> epilogue multiplies by X Y in registers.
// ---------------------------------------------------------------------------------
constexpr int kFMB = 4;                   // m-tiles per LDS stage (must be even)
constexpr int kFStageD2 = kFMB * 8 * 64;  // double2 per stage

struct FArgs {
    KGeom g;
    double3 rec;
    int lo, nown, npad, msplit;
    const double* cs; const double* coef; const double* pos; const double* q;
    double* t_part;
};

// WAVES waves per workgroup (8: 2 per SIMD, 256 registers each; 4: 1 per SIMD, 512),
// NA 16-atom tiles per wave (independent MFMA accumulator chains).
template <int NA, int WAVES>
__global__ void __launch_bounds__(WAVES * 64) k_force(FArgs a) {
    constexpr int kFThreads = WAVES * 64;
    constexpr int kFStageV = kFStageD2 / kFThreads;
    __shared__ __attribute__((aligned(16))) double2 alds[2][kFStageD2];
    const KGeom g = a.g;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 15, qg = lane >> 4;
    const int kc = blockIdx.y / a.msplit, ms = blockIdx.y % a.msplit;
    const int KS = g.nksteps();
    const int ks0 = kc * 16;
    const int NKS = min(16, KS - ks0);    // k-steps past NKS carry zero A and B
    const int M = g.nmtiles();
    const int m_lo = (int)((int64_t)M * ms / a.msplit), m_hi = (int)((int64_t)M * (ms + 1) / a.msplit);
    const int part = blockIdx.y;

    // atoms and B operand
    double b[NA][16];
    double px[NA], py[NA], qa[NA];
    int atom[NA];
#pragma unroll
    for (int at = 0; at < NA; at++) {
        int ia = ((blockIdx.x * WAVES + wave) * NA + at) * 16 + col;  // owned index
        atom[at] = ia;
        bool ok = ia < a.nown;
        int i = a.lo + (ok ? ia : 0);
        px[at] = ok ? a.pos[3 * i] : 0.0;
        py[at] = ok ? a.pos[3 * i + 1] : 0.0;
        qa[at] = ok ? a.q[i] : 0.0;
#pragma unroll
        for (int t = 0; t < 16; t++)
            b[at][t] = (ok && t < NKS) ? a.cs[((size_t)kc * a.npad + ia) * g.CSW + 4 * t + qg] : 0.0;
    }

    // This lane group's combo walks c = 4 mt + qg -> (nx, ny), one m-tile at a time.  The
    // phase w = e^{i(nx gx x + ny gy y)} follows by recurrence: x e^{i 4 gy y} per m-tile,
    // and x e^{i(gx x - NY gy y)} per row wrap (ny past KY-1): sincos only here, once.
    int nx, ny;
    {
        const int c0 = 4 * m_lo + qg;
        nx = c0 / g.NY;
        ny = c0 - nx * g.NY - (g.KY - 1);
    }
    double T0[NA], Tx[NA], Ty[NA], Tz[NA];
    double wr[NA], wi[NA], sr[NA], si[NA], rr[NA], ri[NA];
#pragma unroll
    for (int at = 0; at < NA; at++) {
        T0[at] = Tx[at] = Ty[at] = Tz[at] = 0;
        double s, c;
        sincos((4.0 * a.rec.y) * py[at], &s, &c);  // step e^{i 4 gy y}
        sr[at] = c; si[at] = s;
        sincos(a.rec.x * px[at] - (g.NY * a.rec.y) * py[at], &s, &c);  // row wrap
        rr[at] = c; ri[at] = s;
        sincos((nx * a.rec.x) * px[at] + (ny * a.rec.y) * py[at], &s, &c);
        wr[at] = c; wi[at] = s;
    }

    // stage = kFMB m-tiles x 8 k-step pairs x 64 lanes (double2), a linear copy of 8 KB
    // per m-tile; k-step pairs past NKS and m-tiles past m_hi are zero-filled.
    auto load_stage = [&](int m0, double2 (&reg)[kFStageV]) {
#pragma unroll
        for (int v = 0; v < kFStageV; v++) {
            int e = threadIdx.x + v * kFThreads;
            int mloc = e >> 9, rem = e & 511;  // rem = tp*64 + lane
            int mt = m0 + mloc;
            bool ok = mt < m_hi && 2 * (rem >> 6) < NKS;
            // unconditional load from a clamped address, then select (no branch per load)
            double2 val = reinterpret_cast<const double2*>(a.coef)[ok ? ((size_t)mt * KS + ks0) * 32 + rem : 0];
            reg[v] = ok ? val : make_double2(0, 0);
        }
    };
    auto store_stage = [&](int buf, const double2 (&reg)[kFStageV]) {
#pragma unroll
        for (int v = 0; v < kFStageV; v++) alds[buf][threadIdx.x + v * kFThreads] = reg[v];
    };
    auto read_a = [&](int buf, int mloc, double2 (&av)[8]) {
#pragma unroll
        for (int tp = 0; tp < 8; tp++) av[tp] = alds[buf][mloc * 512 + tp * 64 + lane];
    };

    auto mtile = [&](int mt, const double2 (&av)[8]) {
        if (mt >= m_hi) return;  // wave-uniform
        d4 acc[NA];
#pragma unroll
        for (int at = 0; at < NA; at++) acc[at] = (d4){0, 0, 0, 0};
#pragma unroll
        for (int tp = 0; tp < 8; tp++) {
#pragma unroll
            for (int at = 0; at < NA; at++) acc[at] = mfma64(av[tp].x, b[at][2 * tp], acc[at]);
#pragma unroll
            for (int at = 0; at < NA; at++) acc[at] = mfma64(av[tp].y, b[at][2 * tp + 1], acc[at]);
        }
        // padding combos past KX*NY have zero coefficients
        const double nxd = nx, nyd = ny;
#pragma unroll
        for (int at = 0; at < NA; at++) {
            double re0 = wr[at] * acc[at][0] - wi[at] * acc[at][1];
            double im0 = wr[at] * acc[at][1] + wi[at] * acc[at][0];
            double imz = wr[at] * acc[at][3] + wi[at] * acc[at][2];
            T0[at] += re0;
            Tx[at] += nxd * im0;
            Ty[at] += nyd * im0;
            Tz[at] += imz;
        }
        // advance to combo c + 4
        ny += 4;
#pragma unroll
        for (int at = 0; at < NA; at++) {
            double nr = wr[at] * sr[at] - wi[at] * si[at];
            double ni = wr[at] * si[at] + wi[at] * sr[at];
            wr[at] = nr; wi[at] = ni;
        }
        while (ny > g.KY - 1) {  // at most once per m-tile when NY >= 4
            ny -= g.NY;
            nx += 1;
#pragma unroll
            for (int at = 0; at < NA; at++) {
                double nr = wr[at] * rr[at] - wi[at] * ri[at];
                double ni = wr[at] * ri[at] + wi[at] * rr[at];
                wr[at] = nr; wi[at] = ni;
            }
        }
    };

    const int nstages = (m_hi - m_lo + kFMB - 1) / kFMB;
    double2 reg[kFStageV];
    if (nstages > 0) {
        load_stage(m_lo, reg);
        store_stage(0, reg);
    }
    __syncthreads();
    for (int st = 0; st < nstages; st++) {
        const int buf = st & 1;
        const int m0 = m_lo + st * kFMB;
        if (st + 1 < nstages) load_stage(m0 + kFMB, reg);
        double2 aA[8], aB[8];
        read_a(buf, 0, aA);
#pragma unroll
        for (int mloc = 0; mloc < kFMB; mloc += 2) {
            read_a(buf, mloc + 1, aB);
            mtile(m0 + mloc, aA);
            if (mloc + 2 < kFMB) read_a(buf, mloc + 2, aA);
            mtile(m0 + mloc + 1, aB);
        }
        if (st + 1 < nstages) store_stage(buf ^ 1, reg);
        __syncthreads();
    }

    // reduce over the 4 combo lanes (qg) sharing an atom, write partial
#pragma unroll
    for (int at = 0; at < NA; at++) {
        double v0 = T0[at], v1 = Tx[at], v2 = Ty[at], v3 = Tz[at];
        v0 += __shfl_xor(v0, 16); v1 += __shfl_xor(v1, 16); v2 += __shfl_xor(v2, 16); v3 += __shfl_xor(v3, 16);
        v0 += __shfl_xor(v0, 32); v1 += __shfl_xor(v1, 32); v2 += __shfl_xor(v2, 32); v3 += __shfl_xor(v3, 32);
        if (qg == 0 && atom[at] < a.nown) {
            double* o = a.t_part + ((size_t)part * a.nown + atom[at]) * 4;
            double qi = qa[at];
            o[0] = v0;
            o[1] = qi * a.rec.x * v1;
            o[2] = qi * a.rec.y * v2;
            o[3] = qi * a.rec.z * v3;
        }
    }
}

// ---------------------------------------------------------------------------------
// plan + launchers
// ---------------------------------------------------------------------------------
typedef void (*SfacKernel)(SArgs);

template <int NT>
static SfacKernel sfac_kernel_nt(int ta) {
    switch (ta) {
        case 32: return k_sfac<NT, 32>;
        case 16: return k_sfac<NT, 16>;
        case 8: return k_sfac<NT, 8>;
        default: return k_sfac<NT, 4>;
    }
}

static SfacKernel sfac_kernel(int nt, int ta) {
    switch (nt) {
        case 4: return sfac_kernel_nt<4>(ta);
        case 3: return sfac_kernel_nt<3>(ta);
        case 2: return sfac_kernel_nt<2>(ta);
        default: return sfac_kernel_nt<1>(ta);
    }
}

void kspace_plan(Handle& h) {
    KGeom& g = h.kg;
    g.KX = h.kmax[0]; g.KY = h.kmax[1]; g.KZ = h.kmax[2];
    g.NY = 2 * g.KY - 1;
    g.NYB = (g.NY + 15) / 16;
    g.NYP = 16 * g.NYB;
    g.NYB4 = (g.NY + 3) / 4;
    g.NMT = (g.KX * g.NY + 3) / 4;
    g.NZP = ((2 * g.KZ + 15) / 16) * 16;
    g.NB = (g.NZP + 63) / 64;
    g.CSW = std::min(64, g.NZP);
    int nown = h.hi - h.lo;
    // ---- S-pass
    SPassPlan& sp = h.sp;
    sp.wg_groups = (g.ngroups() + 15) / 16;
    const int csl = cs_lds_stride(g.CSW);
    auto tile_bytes = [&](int TA) { return (size_t)TA * (csl * 8 + g.NYP * 16 + g.KX * 16); };
    auto tile_fits = [&](int TA) {
        int elems = TA * (g.CSW / 2 + g.NYP + g.KX);
        return 2 * tile_bytes(TA) <= 150 * 1024 && elems <= kSMaxV * kSThreads;
    };
    if (!tile_fits(4))
        throw std::invalid_argument("reciprocal-space grid too large for the S-pass LDS tile (kmax)");
    sp.tile_atoms = tile_fits(32) ? 32 : (tile_fits(16) ? 16 : (tile_fits(8) ? 8 : 4));
    sp.lds_bytes = 2 * tile_bytes(sp.tile_atoms);
    // dynamic-LDS permission (a limit, not an allocation) for the S-pass variants used
    for (int nt : {4, (g.NZP % 64) / 16}) {
        if (nt == 0) continue;
        check_hip(hipFuncSetAttribute((const void*)sfac_kernel(nt, sp.tile_atoms),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
                  "k_sfac LDS attribute");
    }
    h.npad = ((nown + sp.tile_atoms - 1) / sp.tile_atoms) * sp.tile_atoms;
    int wg_per_chunk = sp.wg_groups * g.NB;
    int target = std::max(1, (256 + wg_per_chunk - 1) / wg_per_chunk);  // ~one workgroup per CU
    int max_chunks = std::max(1, nown / (2 * sp.tile_atoms));
    sp.nchunks = std::min(target, max_chunks);
    int ca = std::max(1, (nown + sp.nchunks - 1) / sp.nchunks);
    sp.chunk_atoms = ((ca + sp.tile_atoms - 1) / sp.tile_atoms) * sp.tile_atoms;
    sp.nchunks = std::max(1, (nown + sp.chunk_atoms - 1) / sp.chunk_atoms);
    // ---- force pass
    FPassPlan& fp = h.fp;
    // (NA, waves) = (2, 8): 16-atom tiles per wave, waves per workgroup ((4, 4) and (2, 4) measured slower)
    fp.na = 2;
    fp.waves = 8;
    int atoms_per_wg = fp.na * 16 * fp.waves;
    fp.natom_groups = std::max(1, (nown + atoms_per_wg - 1) / atoms_per_wg);
    fp.kchunks = g.NB;
    // split the m-tile range so the number of workgroups is close to a multiple of the CU count
    int best = 1; double best_eff = 0;
    for (int ms = 1; ms <= 8; ms++) {
        int units = fp.natom_groups * fp.kchunks * ms;
        if (ms > 1 && g.nmtiles() / ms < 8) break;
        double rounds = std::ceil(units / 256.0);
        double eff = units / (rounds * 256.0);
        if (eff > best_eff + 0.02) { best_eff = eff; best = ms; }
    }
    fp.msplit = best;
}

size_t kspace_alloc_bytes(const Handle& h) {
    const KGeom& g = h.kg;
    size_t np = h.npad;
    size_t b = 0;
    b += np * g.KX * 16 + np * g.NYP * 16 + (size_t)g.NB * np * g.CSW * 8;
    b += (size_t)h.sp.nchunks * 2 * g.nslots() * g.NZP * 8;
    b += (size_t)2 * g.nslots() * g.NZP * 8;
    b += (size_t)g.nmtiles() * g.nksteps() * 64 * 8;
    b += (size_t)h.fp.nparts() * (h.hi - h.lo) * 4 * 8;
    return b;
}

static double3 recip_vec(const Handle& h) {
    return make_double3(2 * kPi / h.box_L[0], 2 * kPi / h.box_L[1], 2 * kPi / h.box_L[2]);
}

void launch_kspace_tables(Handle& h, const double* pos) {
    const KGeom& g = h.kg;
    int nown = h.hi - h.lo;
    int ncol = g.KX + g.NYP + g.NB * g.CSW / 2;
    int64_t total = (int64_t)nown * ncol;
    hipLaunchKernelGGL(k_tables, dim3(nblk(total, 256)), dim3(256), 0, h.stream, h.lo, nown, h.npad, g,
                       recip_vec(h), pos, h.q, h.tab_xq, h.tab_y, h.tab_cs);
}

void launch_kspace_sfac(Handle& h) {
    const KGeom& g = h.kg;
    SArgs a;
    a.g = g; a.nown = h.hi - h.lo; a.npad = h.npad;
    a.chunk_atoms = h.sp.chunk_atoms;
    a.wg_groups = h.sp.wg_groups;
    a.cs = h.tab_cs; a.ty = h.tab_y; a.xq = h.tab_xq; a.slab = h.s_slab;
    // column blocks 0..NB-1 hold 64 columns except the last (NZP % 64 if nonzero):
    // full blocks in one launch, the ragged one in a second with fewer column tiles
    const int nfull = g.NZP / 64;
    const int rem_nt = (g.NZP % 64) / 16;
    struct L { int nt, nbk0, nblocks; } launches[2] = {{4, 0, nfull}, {rem_nt, nfull, rem_nt > 0 ? 1 : 0}};
    for (const L& l : launches) {
        if (l.nblocks == 0) continue;
        SfacKernel k = sfac_kernel(l.nt, h.sp.tile_atoms);
        a.nbk0 = l.nbk0;
        dim3 grid(h.sp.wg_groups * l.nblocks, h.sp.nchunks);
        hipLaunchKernelGGL(k, grid, dim3(kSThreads), h.sp.lds_bytes, h.stream, a);
    }
    int64_t count = (int64_t)2 * g.nslots() * g.NZP;
    hipLaunchKernelGGL(k_sfac_reduce, dim3(nblk(count, 256)), dim3(256), 0, h.stream, count, h.sp.nchunks, h.s_slab,
                       h.s_red);
}

double* kspace_reduce_buffer(Handle& h, int64_t* count) {
    if (h.kspace_algo == 2) return grid_reduce_buffer(h, count);
    if (h.kspace_algo == 1) {
        *count = 2 * h.khalf;
        return h.sk_red;
    }
    *count = (int64_t)2 * h.kg.nslots() * h.kg.NZP;
    return h.s_red;
}

void launch_kspace_coeffs(Handle& h, int include_energy) {
    const KGeom& g = h.kg;
    double V = h.box_L[0] * h.box_L[1] * h.box_L[2];
    double cst = 4.0 / V * kPi * h.ke;   // RCK:517
    int total = g.KX * g.NY * g.KZ;
    h.e_rec_nblk = nblk(total, 256);
    hipLaunchKernelGGL(k_coeffs, dim3(h.e_rec_nblk), dim3(256), 0, h.stream, g, recip_vec(h), cst,
                       1.0 / (h.alpha * h.alpha), h.s_red, h.coef_a, h.e_rec_part, include_energy);
}

void launch_kspace_force(Handle& h, const double* pos) {
    FArgs a;
    a.g = h.kg; a.rec = recip_vec(h);
    a.lo = h.lo; a.nown = h.hi - h.lo; a.npad = h.npad; a.msplit = h.fp.msplit;
    a.cs = h.tab_cs; a.coef = h.coef_a; a.pos = pos; a.q = h.q; a.t_part = h.t_part;
    dim3 grid(h.fp.natom_groups, h.fp.kchunks * h.fp.msplit);
    hipLaunchKernelGGL((k_force<2, 8>), grid, dim3(512), 0, h.stream, a);
}

// =================================================================================
// direct VALU path (kspace_algo = 1): one lane per k-vector / per atom with explicit
// sincos, exactly the reference's visiting set.  Slow; kept as an independent check
// of the MFMA path and for tiny systems.
// =================================================================================
__global__ void __launch_bounds__(256) k_kvec(int64_t K, KGeom g, double3 rec, double cst, double one_4a2,
                                              double4* __restrict__ kv) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= K) return;
    // enumerate the reference's half-space order RCK:519-556
    int64_t a0 = g.KZ - 1;                       // nx=0, ny=0, nz=1..KZ-1
    int64_t a1 = a0 + (int64_t)(g.KY - 1) * (2 * g.KZ - 1);  // nx=0, ny>=1
    int nx, ny, nz;
    if (t < a0) { nx = 0; ny = 0; nz = (int)t + 1; }
    else if (t < a1) { int64_t u = t - a0; nx = 0; ny = 1 + (int)(u / (2 * g.KZ - 1)); nz = (int)(u % (2 * g.KZ - 1)) - (g.KZ - 1); }
    else {
        int64_t u = t - a1; int64_t per = (int64_t)(2 * g.KY - 1) * (2 * g.KZ - 1);
        nx = 1 + (int)(u / per); int64_t v = u % per;
        ny = (int)(v / (2 * g.KZ - 1)) - (g.KY - 1); nz = (int)(v % (2 * g.KZ - 1)) - (g.KZ - 1);
    }
    double kx = nx * rec.x, ky = ny * rec.y, kz = nz * rec.z;
    double k2 = kx * kx + ky * ky + kz * kz;
    kv[t] = make_double4(kx, ky, kz, 2.0 * cst * exp(-k2 * 0.25 * one_4a2) / k2);
}

__global__ void __launch_bounds__(256) k_dsfac(int64_t K, int lo, int nown, int chunk, const double4* __restrict__ kv,
                                               const double* __restrict__ pos, const double* __restrict__ q,
                                               double* __restrict__ slab) {
    __shared__ double4 sp[256];
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double4 k = t < K ? kv[t] : make_double4(0, 0, 0, 0);
    int a0 = blockIdx.y * chunk, a1 = min(nown, a0 + chunk);
    double cs = 0, ss = 0;
    for (int base = a0; base < a1; base += 256) {
        __syncthreads();
        int ia = base + threadIdx.x;
        if (ia < a1) { int i = lo + ia; sp[threadIdx.x] = make_double4(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2], q[i]); }
        __syncthreads();
        int m = min(256, a1 - base);
        for (int u = 0; u < m; u++) {
            double4 p = sp[u];
            double s, c;
            sincos(k.x * p.x + k.y * p.y + k.z * p.z, &s, &c);
            cs += p.w * c; ss += p.w * s;
        }
    }
    if (t < K) { slab[((size_t)blockIdx.y * 2) * K + t] = cs; slab[((size_t)blockIdx.y * 2 + 1) * K + t] = ss; }
}

__global__ void __launch_bounds__(256) k_dcoeffs(int64_t K, const double4* __restrict__ kv, double* __restrict__ sk,
                                                 double* __restrict__ e_part, int include_energy) {
    __shared__ double red[256];
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double e = 0;
    if (t < K) {
        double cs = sk[t], ss = sk[K + t];
        if (include_energy) e = 0.5 * kv[t].w * (cs * cs + ss * ss);
    }
    red[threadIdx.x] = e;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) e_part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) k_dforce(int64_t K, int lo, int nown, const double4* __restrict__ kv,
                                                const double* __restrict__ sk, const double* __restrict__ pos,
                                                const double* __restrict__ q, double* __restrict__ t_part) {
    __shared__ double4 sk4[256];
    __shared__ double2 ss2[256];
    int ia = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = ia < nown;
    int i = lo + (ok ? ia : 0);
    double x = pos[3 * i], y = pos[3 * i + 1], z = pos[3 * i + 2];
    double t0 = 0, fx = 0, fy = 0, fz = 0;
    for (int64_t base = 0; base < K; base += 256) {
        __syncthreads();
        int64_t kk = base + threadIdx.x;
        if (kk < K) { sk4[threadIdx.x] = kv[kk]; ss2[threadIdx.x] = make_double2(sk[kk], sk[K + kk]); }
        __syncthreads();
        int m = (int)min((int64_t)256, K - base);
        for (int u = 0; u < m; u++) {
            double4 k = sk4[u];
            double2 S = ss2[u];
            double s, c;
            sincos(k.x * x + k.y * y + k.z * z, &s, &c);
            t0 += k.w * (S.x * c + S.y * s);
            double g = k.w * (S.x * s - S.y * c);
            fx += g * k.x; fy += g * k.y; fz += g * k.z;
        }
    }
    if (ok) {
        double qi = q[i];
        double* o = t_part + (size_t)ia * 4;
        o[0] = t0; o[1] = qi * fx; o[2] = qi * fy; o[3] = qi * fz;
    }
}

void launch_kspace_kvec(Handle& h) {
    double V = h.box_L[0] * h.box_L[1] * h.box_L[2];
    double cst = 4.0 / V * kPi * h.ke;
    hipLaunchKernelGGL(k_kvec, dim3(nblk(h.khalf, 256)), dim3(256), 0, h.stream, h.khalf, h.kg, recip_vec(h), cst,
                       1.0 / (h.alpha * h.alpha), h.kvec);
}

void launch_kspace_direct_sfac(Handle& h, const double* pos) {
    launch_kspace_kvec(h);
    int nown = h.hi - h.lo;
    int chunk = (nown + h.sk_nchunk - 1) / h.sk_nchunk;
    hipLaunchKernelGGL(k_dsfac, dim3(nblk(h.khalf, 256), h.sk_nchunk), dim3(256), 0, h.stream, h.khalf, h.lo, nown,
                       chunk, h.kvec, pos, h.q, h.sk_slab);
    int64_t count = 2 * h.khalf;
    hipLaunchKernelGGL(k_sfac_reduce, dim3(nblk(count, 256)), dim3(256), 0, h.stream, count, h.sk_nchunk, h.sk_slab,
                       h.sk_red);
}

void launch_kspace_direct_coeffs(Handle& h, int include_energy) {
    h.e_rec_nblk = nblk(h.khalf, 256);
    hipLaunchKernelGGL(k_dcoeffs, dim3(h.e_rec_nblk), dim3(256), 0, h.stream, h.khalf, h.kvec, h.sk_red, h.e_rec_part,
                       include_energy);
}

void launch_kspace_direct_force(Handle& h, const double* pos) {
    int nown = h.hi - h.lo;
    hipLaunchKernelGGL(k_dforce, dim3(nblk(nown, 256)), dim3(256), 0, h.stream, h.khalf, h.lo, nown, h.kvec, h.sk_red,
                       pos, h.q, h.t_part);
}

}  // namespace cf
