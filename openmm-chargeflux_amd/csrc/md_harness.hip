// md_harness.hip — the benchmark's MD harness (NOT part of the CoulForce path): velocity
// Verlet for the owned atoms and the flexible-water harmonic restraints (O-H, O-H, H-H),
// fused into two kernels per step so the harness does not dominate small per-rank steps.
// Built into its own library (libcf_mdharness.so) and driven by bench.py.
//
// Step:  md_kick_drift   v += dt/2 f/m ; x += dt v            (owned atoms)
//        <positions replicated, forces zeroed, CoulForce adds its forces>
//        md_restrain_kick f += restraint(x) ; v += dt/2 f/m   (owned atoms)
// bench.py fuses the last kernel of a step with the first of the next (md_restrain_kick_drift):
// one harness launch per step.
// Waters are atoms 3w, 3w+1, 3w+2 (O, H, H) for w < n_waters; every atom recomputes the
// three bonds of its own water, so there are no atomics and the result is deterministic.
#include <hip/hip_runtime.h>

#include <cstdint>

#define MD_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

// v += dt/2 f/m ; x += dt v for the owned atoms, and f = 0 (its last reader this step: the
// next force evaluation adds into it, so the step needs no separate zeroing launch)
__global__ void __launch_bounds__(256) k_kick_drift(int lo, int hi, double dt, double* __restrict__ x,
                                                    double* __restrict__ v, double* __restrict__ f,
                                                    const double* __restrict__ inv_m) {
    int i = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hi) return;
    double h = 0.5 * dt * inv_m[i];
#pragma unroll
    for (int d = 0; d < 3; d++) {
        double vv = v[3 * i + d] + h * f[3 * i + d];
        v[3 * i + d] = vv;
        x[3 * i + d] += dt * vv;
        f[3 * i + d] = 0.0;
    }
}

__device__ __forceinline__ void bond(const double* x, int a, int b, double k, double r0, double g[3]) {
    double d[3] = {x[3 * b] - x[3 * a], x[3 * b + 1] - x[3 * a + 1], x[3 * b + 2] - x[3 * a + 2]};
    double r = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    double c = k * (r - r0) / r;
    g[0] = c * d[0]; g[1] = c * d[1]; g[2] = c * d[2];  // force on a; -g on b
}

__global__ void __launch_bounds__(256) k_restrain_kick(int lo, int hi, int n_waters, double k_oh, double r_oh,
                                                       double k_hh, double r_hh, double dt,
                                                       const double* __restrict__ x, double* __restrict__ v,
                                                       double* __restrict__ f, const double* __restrict__ inv_m) {
    int i = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hi) return;
    double fi[3] = {f[3 * i], f[3 * i + 1], f[3 * i + 2]};
    if (i < 3 * n_waters) {
        int o = 3 * (i / 3), r = i - o;
        double g1[3], g2[3], g3[3];
        bond(x, o, o + 1, k_oh, r_oh, g1);
        bond(x, o, o + 2, k_oh, r_oh, g2);
        bond(x, o + 1, o + 2, k_hh, r_hh, g3);
#pragma unroll
        for (int d = 0; d < 3; d++) {
            double add = r == 0 ? g1[d] + g2[d] : (r == 1 ? -g1[d] + g3[d] : -g2[d] - g3[d]);
            fi[d] += add;
        }
    }
    double h = 0.5 * dt * inv_m[i];
#pragma unroll
    for (int d = 0; d < 3; d++) {
        f[3 * i + d] = fi[d];
        v[3 * i + d] += h * fi[d];
    }
}

// The end of step n and the start of step n + 1 in one launch: f += restraint(x) ; v += dt/2 f/m
// (the second half kick; skipped on the first call, where x, v are the initial state) ; v += dt/2
// f/m ; x += dt v ; f = 0.  One thread per water (its three atoms: every restraint is evaluated
// from positions no thread has drifted yet) or per other atom.
__global__ void __launch_bounds__(256) k_restrain_kick_drift(int lo, int hi, int n_waters, double k_oh, double r_oh,
                                                             double k_hh, double r_hh, double dt, int first,
                                                             double* __restrict__ x, double* __restrict__ v,
                                                             double* __restrict__ f,
                                                             const double* __restrict__ inv_m) {
    const int wend = min(hi, 3 * n_waters);                 // owned water atoms [lo, wend): whole waters
    const int nwu = wend > lo ? (wend - lo) / 3 : 0;
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    int a0, na;
    if (u < nwu) { a0 = lo + 3 * u; na = 3; }
    else { a0 = max(lo, wend) + (u - nwu); na = 1; if (a0 >= hi) return; }
    double fr[3][3] = {};
    if (na == 3) {
        double g1[3], g2[3], g3[3];
        bond(x, a0, a0 + 1, k_oh, r_oh, g1);
        bond(x, a0, a0 + 2, k_oh, r_oh, g2);
        bond(x, a0 + 1, a0 + 2, k_hh, r_hh, g3);
#pragma unroll
        for (int d = 0; d < 3; d++) {
            fr[0][d] = g1[d] + g2[d];
            fr[1][d] = -g1[d] + g3[d];
            fr[2][d] = -g2[d] - g3[d];
        }
    }
    for (int q = 0; q < na; q++) {
        const int i = a0 + q;
        const double h = 0.5 * dt * inv_m[i];
#pragma unroll
        for (int d = 0; d < 3; d++) {
            const double fi = f[3 * i + d] + fr[q][d];
            double vv = v[3 * i + d];
            if (!first) vv += h * fi;   // second half kick of the previous step
            vv += h * fi;               // first half kick of this step
            v[3 * i + d] = vv;
            x[3 * i + d] += dt * vv;
            f[3 * i + d] = 0.0;
        }
    }
}

inline int nblk(int n) { return (n + 255) / 256; }

}  // namespace

MD_EXPORT int md_kick_drift(int lo, int hi, double dt, double* x, double* v, double* f, const double* inv_m,
                            void* stream) {
    if (hi <= lo) return 0;
    hipLaunchKernelGGL(k_kick_drift, dim3(nblk(hi - lo)), dim3(256), 0, (hipStream_t)stream, lo, hi, dt, x, v, f,
                       inv_m);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

MD_EXPORT int md_restrain_kick(int lo, int hi, int n_waters, double k_oh, double r_oh, double k_hh, double r_hh,
                               double dt, const double* x, double* v, double* f, const double* inv_m, void* stream) {
    if (hi <= lo) return 0;
    hipLaunchKernelGGL(k_restrain_kick, dim3(nblk(hi - lo)), dim3(256), 0, (hipStream_t)stream, lo, hi, n_waters,
                       k_oh, r_oh, k_hh, r_hh, dt, x, v, f, inv_m);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

MD_EXPORT int md_restrain_kick_drift(int lo, int hi, int n_waters, double k_oh, double r_oh, double k_hh, double r_hh,
                                     double dt, int first, double* x, double* v, double* f, const double* inv_m,
                                     void* stream) {
    if (hi <= lo) return 0;
    hipLaunchKernelGGL(k_restrain_kick_drift, dim3(nblk(hi - lo)), dim3(256), 0, (hipStream_t)stream, lo, hi,
                       n_waters, k_oh, r_oh, k_hh, r_hh, dt, first, x, v, f, inv_m);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
