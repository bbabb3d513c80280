// cf_pair.h -- device helpers shared by the direct-space kernels (cf_kernels_core.hip: cell list,
// per-atom lists, k_pairs*, k_excl; cf_kernels_cluster.hip: the cluster-pair list and k_pairs_cq):
// box geometry, the pair-kernel argument block, the erfc table evaluation and the 64-bit fixed
// point of the half lists' partner-side sums.  Reference semantics: ReferenceCoulKernels.cpp (RCK).
#pragma once

#include "cf_internal.h"

namespace cf {

// OpenMM ReferenceForce::getDeltaR[Periodic]: d = J - I, minimum image by the box vectors c,
// b, a in that order via floor(d/L + 0.5) (used by RCK:53-55, 567, 601).  Boxes are in OpenMM's
// reduced form a = (Lx,0,0), b = (bx,Ly,0), c = (cx,cy,Lz); T = (bx, cx, cy), zero for an
// orthorhombic box (the per-axis form, the same bits).
__device__ __forceinline__ double3 delta_r(double3 pi, double3 pj, double3 L, int pbc,
                                           double3 T = make_double3(0.0, 0.0, 0.0)) {
    double3 d = make_double3(pj.x - pi.x, pj.y - pi.y, pj.z - pi.z);
    if (pbc) {
        if (T.x != 0.0 || T.y != 0.0 || T.z != 0.0) {
            const double sc = floor(d.z / L.z + 0.5);
            d.x -= sc * T.y; d.y -= sc * T.z; d.z -= sc * L.z;
            const double sb = floor(d.y / L.y + 0.5);
            d.x -= sb * T.x; d.y -= sb * L.y;
            d.x -= L.x * floor(d.x / L.x + 0.5);
        } else {
            d.z -= L.z * floor(d.z / L.z + 0.5);
            d.y -= L.y * floor(d.y / L.y + 0.5);
            d.x -= L.x * floor(d.x / L.x + 0.5);
        }
    }
    return d;
}

__device__ __forceinline__ double3 ld3(const double* p, int i) {
    return make_double3(p[3 * i], p[3 * i + 1], p[3 * i + 2]);
}

// The periodic lattice of OpenMM's reduced box: a = (L.x,0,0), b = (T.x,L.y,0), c = (T.y,T.z,L.z)
// (T = (bx, cx, cy); all zero for an orthorhombic box, where every helper below reduces to the
// per-axis form with the same bits: the T terms subtract exact zeros).
// ka a + kb b + kc c
__device__ __forceinline__ double3 lattice(double3 L, double3 T, double ka, double kb, double kc) {
    return make_double3(ka * L.x + kb * T.x + kc * T.y, kb * L.y + kc * T.z, kc * L.z);
}
// fractional coordinates: x = s_a a + s_b b + s_c c
__device__ __forceinline__ double3 fractional(double3 x, double3 L, double3 T) {
    const double sc = x.z / L.z;
    const double sb = (x.y - sc * T.z) / L.y;
    const double sa = (x.x - sb * T.x - sc * T.y) / L.x;
    return make_double3(sa, sb, sc);
}
// x moved by the lattice translation -(fl.x a + fl.y b + fl.z c); with fl = floor(fractional(x))
// the result lies in the unit cell (fractional coordinates in [0, 1))
__device__ __forceinline__ double3 wrap_by(double3 x, double3 fl, double3 L, double3 T) {
    return make_double3(x.x - fl.x * L.x - fl.y * T.x - fl.z * T.y, x.y - fl.y * L.y - fl.z * T.z, x.z - fl.z * L.z);
}
__device__ __forceinline__ double3 floor3(double3 v) { return make_double3(floor(v.x), floor(v.y), floor(v.z)); }

constexpr int kMaxRegExcl = 8;
constexpr int kErfcDeg = 7;      // erfcx polynomial degree per interval (fp64): relative error 3.6e-16
constexpr int kErfcMaxM = 129;   // fp64 intervals of width 1/16: x = alpha r up to 8 (erfc(8) = 1e-29)
constexpr int kErfcDegF = 6;     // the same in fp32 (mixed precision): relative error ~1e-7
constexpr int kErfcMaxMF = 32;   // fp32 intervals of width 0.375: x = alpha r up to 11.6
constexpr int kMaxLjTypes = 64;  // LJ types carried in the 6 high bits of a list entry
constexpr int kSeg = 4;          // neighbour sub-lists per atom (one per scanning wave / pair lane)
constexpr int kShiftBits = 26;
constexpr int kJMask = (1 << kShiftBits) - 1;   // atom / slot index bits of a packed entry
constexpr int kBruteShift = 31;  // shift code: minimum image by floor (brute-force path)
// Half neighbour list, split by x (a half-space rule): the pair (i, j) is
// kept by the atom of the lower x cell when their cells differ in x, and otherwise by the
// atom with the smaller wrapped x (rounded to fp32, a per-atom key that both sides see
// identically; ties: the lower sorted slot).  Every atom so keeps about half of its partners
// wherever it sits in its cell (a cell-index rule -- own cell "later" partners plus 13
// forward cells -- gives the first rows of a cell ~2x the partners of the last ones and skews
// the sub-lists, ~0.66 lane efficiency against ~0.84).  A row's partners lie in the 18 cells
// at x offset 0 or +1: the row cell's window.  Entry = sorted slot of j | k << 21 (window
// cell k = ox*9 + (oy+1)*3 + (oz+1)) | LJ type << 26: the partner's address needs no table
// lookup (the gather is not queued behind LDS work).
constexpr int kHalfWin = 18;          // window cells per block: x offsets 0 and +1
constexpr int kHalfBlock = 1024;      // threads per k_pairs_half block (one cell; 4 lanes per row)
constexpr int kHalfOwn = 4;           // the row cell's own window index (0, 0, 0)
constexpr int kHalfMaxWin = 4096;     // window atoms per block (LDS accumulators: 128 KB)
constexpr int kHalfSlotBits = 21;     // sorted slots < 2^21 (cf_api.hip enables half lists below)
constexpr int kHalfSlotMask = (1 << kHalfSlotBits) - 1;
static_assert(kHalfSlotBits + 5 <= kShiftBits, "window cell bits overlap the LJ type bits");
// j-side sums in 64-bit fixed point (integer adds: exact, so any order gives the same bits):
// v -> round(v 2^34) via the 1.5 * 2^52 magic add (exact for |v 2^34| < 2^51); a contribution
// with |v| >= 2^16 flags the evaluation for the fp64 rescan fallback
constexpr double kFixScale = 17179869184.0;            // 2^34
constexpr double kFixInv = 1.0 / 17179869184.0;
constexpr double kFixMagic = 6755399441055744.0;       // 1.5 * 2^52
constexpr long long kFixMagicBits = 0x4338000000000000LL;
constexpr double kFixMax = 65536.0;
// mixed precision on the cluster-pair list (DirectArgs::win32): the partner-side sums in 32-bit fixed
// point, 2^-13 kJ/mol/nm (1.2e-4: below the fp32 pair terms' own rounding at |F| ~ 1e3, against the
// C5 bar of 1e-4 RMS relative), range +-2^18 per window slot; half the LDS window (64 KB) and half
// of win_out's bytes written by the pair kernel and read back by k_excl
constexpr float kFix32Scale = 8192.0f;   // 2^13
constexpr double kFix32Inv = 1.0 / 8192.0;
__device__ __forceinline__ unsigned to_fix32(float v) { return (unsigned)__float2int_rn(v * kFix32Scale); }
// an already scaled value (v * 2^13) to the 32-bit fixed point: floor(vs + 0.5) in one instruction
// (v_cvt_rpi_i32_f32; round-to-nearest but for exact ties, which round up instead of to even)
__device__ __forceinline__ unsigned scaled_to_fix32(float vs) {
    int r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(vs));
    return (unsigned)r;
}
// why half_flag was raised (bits; cf_get_fallback_stats reports their union)
constexpr int kHalfWindowFull = 1;     // a cell's 18-cell window holds more than kHalfMaxWin atoms
constexpr int kHalfListOverflow = 2;   // a row's sub-list overflowed, or the builder could not place it
constexpr int kHalfFixedRange = 4;     // a partner-side term beyond the fixed-point range

struct DirectArgs {
    int n, lo, hi, include_forces;
    double3 L; double3 invL; int3 nc; int brute;
    double3 T; int tric;        // reduced triclinic box: off-diagonals (bx, cx, cy); tric = any nonzero
    double rc2, alpha;
    double rc;                  // cutoff (the half list's fixed-point range bound)
    double ke;                  // Coulomb constant ONE_4PI_EPS0 (Handle::ke)
    const double* erfc_tab;     // [kErfcDeg+1][kErfcMaxM] erfcx(x) on intervals of width 1/erfc_scale
    const float* erfc_tab_f;    // [erfc_m_f][kErfcDegF+1] fp32 (mixed precision), width 1/erfc_scale_f
    double erfc_scale; int erfc_m;
    double erfc_scale_f; int erfc_m_f;
    double rl2;                 // list radius^2: (rc + list skin)^2
    int nb_cap;                 // capacity of ONE of the kSeg sub-lists
    int nlr;                    // list rows = owned atoms; row c <-> sorted slot own_slot(c)
    const int* own_s;           // [nlr] cell-sorted slots of the owned atoms (null: identity)
    const int* own_start;       // [ncell + 1] owned atoms per cell, scanned (null on one rank)
    const int* flag;            // rebuild flag (list kernels exit when 0)
    const int* atom_sorted; const int* key_sorted;
    const int* cstart; const int* cend;
    const double4* pos4s; const double2* ljs;
    const int* typ_s;           // [N] LJ type per sorted slot (null: > kMaxLjTypes distinct types)
    const double2* lj_tab; int lj_ntypes;   // per-type (sigma/2, 2 sqrt(eps))
    const double* pos; const double* q;
    const int* ex_start; const int* ex_list;
    const double* dedq_self;
    int* nl; int* nl_cnt;
    double* dedq; double* f_part; double* e_atom;
    // half list (single rank, fp64): pairs once, j-side summed in fixed point (k_pairs_half)
    int half;
    int* half_flag;             // device: 1 = the half-list evaluation cannot be used (k_excl rescans)
    unsigned long long* win_out;// [ncell][kHalfMaxWin][4] per-cell window partials (fixed point)
    int* win_woff;              // [ncell][kHalfWin] window offsets of the 18 window cells
    const int* key_s;           // cell key per sorted slot
    long long* fallback;        // [3] diagnostics (Handle::n_fallback_dev)
    // cluster-pair half list (cf_kernels_cluster.hip)
    const int* cl_start;        // [ncell + 1] first cluster of each cell
    const int2* cl_info;        // [clusters] (first sorted slot, count)
    const uint2* cpl;           // [clusters][cpl_cap] (first slot of j | window cell << 21, pair mask)
    const int* cpl_cnt;         // [clusters]
    int cpl_cap;
    const float4* pos4f;        // [N] fp32 (x, y, z, LJ type bits)
    const int* slot_of;         // [N] atom -> sorted slot
    float rcm2f;                // prefilter radius^2: rc with a margin above the fp32 rounding of |d|
    int ncl_cap;                // clusters cl_info / cpl_cnt / cpl hold
    int win32;                  // win_out holds 32-bit fixed-point sums (uint4 per slot): mixed precision, cluster list
    int* err;                   // [1] device index guards (kGuard* bits, cf_internal.h)
};

__device__ __forceinline__ int own_slot(const DirectArgs& a, int c) { return a.own_s ? a.own_s[c] : c; }

// minimum image of a pair vector d = pos_i - pos_j: per axis d - L rint(d/L) (getDeltaRPeriodic's
// floor(d/L + 0.5) up to exact half-box ties, which lie beyond the cutoff); a reduced triclinic
// box subtracts c, b, a in that order (kernel-uniform branch)
__device__ __forceinline__ void min_image(const DirectArgs& a, double& dx, double& dy, double& dz) {
    // one branch-free sequence for both box kinds: with the off-diagonals T = 0 the shear
    // terms subtract exact zeros, so an orthorhombic box gets the bits of the per-axis form
    // (the two-branch version kept dx, dy, dz in scratch memory: 40 B per lane in k_pairs)
    const double sc = rint(dz * a.invL.z);
    dx -= sc * a.T.y; dy -= sc * a.T.z; dz -= sc * a.L.z;
    const double sb = rint(dy * a.invL.y);
    dx -= sb * a.T.x; dy -= sb * a.L.y;
    dx -= a.L.x * rint(dx * a.invL.x);
}


struct PairAcc {
    double fx = 0, fy = 0, fz = 0, dq = 0, e = 0;
};

struct PairAccF {   // mixed precision: fp32 forces / dE/dq, fp64 energy
    float fx = 0, fy = 0, fz = 0, dq = 0;
    double e = 0;
};

// erfc(x) = e^{-x^2} erfcx(x): erfcx from a piecewise degree-7 polynomial (interval table
// in LDS, fitted at cf_create in long double, relative error ~4e-16 over [0, alpha*rc]),
// and e^{-x^2} is shared with the force term -> one exp per pair instead of erfc + exp.
// The table is coefficient-major, tab[j * kErfcMaxM + interval]: the 64 lanes of a read
// fetch coefficient j of their (random) intervals from one contiguous run of doubles, so they
// spread over the LDS banks.  (Interval-major rows of 8 doubles put every lane's read on one
// of 4 bank groups: 6.8 conflict cycles per LDS instruction in the round-1 PMC pass.)
__device__ __forceinline__ double erfc_exp(double x, const double* __restrict__ tab, double scale, double& e2) {
    const double y = x * scale;
    const int i = (int)y;
    const double u = 2.0 * (y - (double)i) - 1.0;
    const double* c = tab + i;
    // Estrin's scheme (the 8 coefficient reads are independent, so they issue back to back and
    // wait once; Horner's chain interleaved each LDS read with the FMA that needed it: 8 LDS
    // latencies per pair)
    static_assert(kErfcDeg == 7, "Estrin pairing below is written for degree 7");
    double cc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) cc[j] = c[j * kErfcMaxM];
    const double u2 = u * u;
    const double p01 = fma(cc[1], u, cc[0]), p23 = fma(cc[3], u, cc[2]);
    const double p45 = fma(cc[5], u, cc[4]), p67 = fma(cc[7], u, cc[6]);
    const double p03 = fma(p23, u2, p01), p47 = fma(p67, u2, p45);
    const double p = fma(p47, u2 * u2, p03);
    e2 = exp_nonpos(-x * x);
    return e2 * p;
}

__device__ __forceinline__ unsigned long long to_fix(double v) {
    return (unsigned long long)(__double_as_longlong(fma(v, kFixScale, kFixMagic)) - kFixMagicBits);
}

// the same for a value already scaled by 2^34: one add (literal operand) + one integer add
__device__ __forceinline__ unsigned long long scaled_to_fix(double vs) {
    return (unsigned long long)(__double_as_longlong(vs + kFixMagic) - kFixMagicBits);
}

__device__ __forceinline__ int3 half_offset(int k) {   // window cell k -> cell offset
    return make_int3(k / 9, (k / 3) % 3 - 1, k % 3 - 1);
}

__device__ __forceinline__ int wrap_cell(int v, int n) { return v < 0 ? v + n : (v >= n ? v - n : v); }

DirectArgs direct_args(Handle& h, const double* pos, int include_forces);

}  // namespace cf
