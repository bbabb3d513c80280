// cf_kernels_openmm.hip -- OpenMM GPU-platform buffer conventions at the C ABI (cf_compute_openmm).
//
// The reference's CUDA platform binds its kernels to the platform's own device buffers
// (platforms/cuda/src/CudaCoulKernels.cpp:523-600): positions and charges as posq (real4) in the
// platform's sorted atom order with atomIndex (sorted slot -> atom), forces accumulated into
// forceBuffers -- 64-bit fixed point in 2^32 units, x | y | z planes of paddedNumAtoms entries,
// indexed by sorted slot -- and the energy into energyBuffer.  These two kernels put that layout
// in front of the evaluator: a gather into the handle's atom-order fp64 positions and a scatter of
// its atom-order forces into the fixed-point planes.  posq.w is only read, never written (the
// reference's computeNonbonded / copy kernels overwrite it with the flux charges).
#include "cf_pair.h"

namespace cf {

// posq[s] -> pos[atom_index[s]] (fp64); mixed precision adds posqCorrection in fp64, the way the
// platform reconstructs its fp64 positions (x = posq.x + posqCorrection.x)
template <bool F4>
__global__ void __launch_bounds__(256) k_om_gather(int n, const void* __restrict__ posq, const float4* __restrict__ corr,
                                                   const int* __restrict__ atom_index, double* __restrict__ pos,
                                                   int* __restrict__ err) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const int a = atom_index[s];
    if ((unsigned)a >= (unsigned)n) { atomicOr(err, kGuardAtomIndex); return; }   // guard
    double x, y, z;
    if constexpr (F4) {
        const float4 p = static_cast<const float4*>(posq)[s];
        x = p.x; y = p.y; z = p.z;
        if (corr) {
            const float4 c = corr[s];
            x += c.x; y += c.y; z += c.z;
        }
    } else {
        const double4 p = static_cast<const double4*>(posq)[s];
        x = p.x; y = p.y; z = p.z;
    }
    pos[3 * a] = x; pos[3 * a + 1] = y; pos[3 * a + 2] = z;
}

// forces of atom atom_index[s] -> fixed point at slot s of the three planes (OpenMM's conversion:
// (unsigned long long)(long long)(f * 2^32), added with 64-bit integer atomics as the platform's
// own kernels add theirs), and the energy into the energy-buffer slot
template <bool EF>
__global__ void __launch_bounds__(256) k_om_scatter(int n, const int* __restrict__ atom_index,
                                                    const double* __restrict__ frc, int padded,
                                                    unsigned long long* __restrict__ fbuf,
                                                    const double* __restrict__ ene, void* __restrict__ ebuf) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s == 0 && ebuf) {
        if constexpr (EF) atomicAdd(static_cast<float*>(ebuf), (float)*ene);
        else atomicAdd(static_cast<double*>(ebuf), *ene);
    }
    if (s >= n || !fbuf) return;
    const int a = atom_index[s];
    if ((unsigned)a >= (unsigned)n) return;   // (flagged by k_om_gather)
    constexpr double kScale = 4294967296.0;
#pragma unroll
    for (int d = 0; d < 3; d++) {
        const double f = frc[3 * a + d];
        if (f != 0.0) atomicAdd(fbuf + (size_t)d * padded + s, (unsigned long long)(long long)(f * kScale));
    }
}

static inline int nblk_om(int n) { return (n + 255) / 256; }

void launch_om_gather(Handle& h, const void* posq, const void* corr, int posq_kind, const int* atom_index,
                      double* pos) {
    if (posq_kind == CF_POSQ_FLOAT4)
        hipLaunchKernelGGL(k_om_gather<true>, dim3(nblk_om(h.n)), dim3(256), 0, h.stream, h.n, posq,
                           static_cast<const float4*>(corr), atom_index, pos, h.err_dev);
    else
        hipLaunchKernelGGL(k_om_gather<false>, dim3(nblk_om(h.n)), dim3(256), 0, h.stream, h.n, posq, nullptr,
                           atom_index, pos, h.err_dev);
}

void launch_om_scatter(Handle& h, const int* atom_index, const double* frc, int padded, long long* fbuf,
                       const double* ene, void* ebuf, int energy_kind) {
    auto* fb = reinterpret_cast<unsigned long long*>(fbuf);
    if (energy_kind == CF_ENERGY_FLOAT)
        hipLaunchKernelGGL(k_om_scatter<true>, dim3(nblk_om(h.n)), dim3(256), 0, h.stream, h.n, atom_index, frc, padded,
                           fb, ene, ebuf);
    else
        hipLaunchKernelGGL(k_om_scatter<false>, dim3(nblk_om(h.n)), dim3(256), 0, h.stream, h.n, atom_index, frc,
                           padded, fb, ene, ebuf);
}

}  // namespace cf
