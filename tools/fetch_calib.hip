// fetch_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths this library's hot kernels use (MI355X_MICROARCH.md: only 16-B/lane coalesced
// streaming reads are calibrated, at exactly 1/2).  Each kernel moves a known number of bytes,
// every byte once, from a 1 GiB buffer (no L2 reuse), in one access pattern:
//   c_stream16   16 B per lane, coalesced                     (guide case: FETCH = bytes / 2)
//   c_seg64      4 lanes x 16 B = one 64-B piece, pieces at permuted 64-B offsets
//                (k_g_spread_tile's window staging, k_g_interp's halo rows)
//   c_gather32   32 B per lane (two 16-B loads), permuted 32-B records
//                (k_pairs_half's partner gathers, each record once here)
//   c_gather8    8 B per lane, permuted 8-B words
//   c_scalar64   wave-uniform 64 B (s_load_dwordx16), permuted 64-B pieces (spread's x window)
//   c_rows168    runs of 21 doubles (168 B, 8-B aligned) per 21 lanes at permuted row starts
//                (k_g_interp's halo rows: lane t reads z = t % 21 of row t / 21)
//   w_stream16   16 B per lane coalesced stores
//   w_seg64      64-B pieces (8 doubles) at permuted offsets (spread's grid tile rows)
// Run: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib ; rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
// (the program prints each kernel's byte count; tools/fetch_calib.py joins the two).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

// bijection of [0, n) for n a power of two (odd multiplier, xor-shift)
__device__ __forceinline__ unsigned perm(unsigned i, unsigned n) {
    unsigned v = (i * 2654435761u) & (n - 1);   // odd multiply mod n = 2^k
    v ^= v >> 7;                                 // xor-shift within k bits
    return (v * 0x9E3779B1u) & (n - 1);
}

__global__ void c_stream16(const v2d* __restrict__ a, size_t n16, double* __restrict__ out) {
    v2d s = {0.0, 0.0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s.x == 12345.678) out[0] = s.y;
}

__global__ void c_seg64(const v2d* __restrict__ a, unsigned nseg, double* __restrict__ out) {
    v2d s = {0.0, 0.0};
    const unsigned q = threadIdx.x & 3;
    for (unsigned g = (blockIdx.x * blockDim.x + threadIdx.x) >> 2; g < nseg; g += (gridDim.x * blockDim.x) >> 2)
        s += a[(size_t)perm(g, nseg) * 4 + q];
    if (s.x == 12345.678) out[0] = s.y;
}

__global__ void c_gather32(const v2d* __restrict__ a, unsigned nrec, double* __restrict__ out) {
    v2d s = {0.0, 0.0};
    for (unsigned g = blockIdx.x * blockDim.x + threadIdx.x; g < nrec; g += gridDim.x * blockDim.x) {
        const size_t r = perm(g, nrec);
        s += a[2 * r] + a[2 * r + 1];
    }
    if (s.x == 12345.678) out[0] = s.y;
}

__global__ void c_gather8(const double* __restrict__ a, unsigned nw, double* __restrict__ out) {
    double s = 0.0;
    for (unsigned g = blockIdx.x * blockDim.x + threadIdx.x; g < nw; g += gridDim.x * blockDim.x) s += a[perm(g, nw)];
    if (s == 12345.678) out[0] = s;
}

// one 64-B piece per wave iteration, read with a wave-uniform address (scalar loads)
__global__ void c_scalar64(const double* __restrict__ a, unsigned nseg, double* __restrict__ out) {
    double s = 0.0;
    const unsigned wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const unsigned nwave = (gridDim.x * blockDim.x) >> 6;
    for (unsigned g = wave; g < nseg; g += nwave) {
        const double* p = a + (size_t)__builtin_amdgcn_readfirstlane(perm(g, nseg)) * 8;
        double x[8];
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = p[i];
#pragma unroll
        for (int i = 0; i < 8; i++) s = fma(x[i], (double)(threadIdx.x & 63), s);
    }
    if (s == 12345.678) out[0] = s;
}

// 21 lanes per 168-B run; the run starts are a permutation of the region's 168-B slots
__global__ void c_rows168(const double* __restrict__ a, unsigned nrun, double* __restrict__ out) {
    double s = 0.0;
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
    // lanes past the last full run of a wave idle, as in the interpolation's staging (21 * 3 = 63)
    const unsigned lane = threadIdx.x & 63, wave = t >> 6, nwave = nt >> 6;
    if (lane < 63) {
        for (unsigned g = wave * 3 + lane / 21; g < nrun; g += nwave * 3) s += a[(size_t)perm(g, nrun) * 21 + lane % 21];
    }
    if (s == 12345.678) out[0] = s;
}

__global__ void w_stream16(v2d* __restrict__ a, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        a[i] = v2d{(double)i, 1.0};
}

__global__ void w_seg64(v2d* __restrict__ a, unsigned nseg) {
    const unsigned q = threadIdx.x & 3;
    for (unsigned g = (blockIdx.x * blockDim.x + threadIdx.x) >> 2; g < nseg; g += (gridDim.x * blockDim.x) >> 2)
        a[(size_t)perm(g, nseg) * 4 + q] = v2d{(double)g, 2.0};
}

int main() {
    const size_t bytes = (size_t)1 << 30;      // buffer
    const size_t moved = (size_t)1 << 28;      // bytes each kernel moves (256 MiB), every byte once
    void* buf;
    double* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 0, bytes));
    CK(hipDeviceSynchronize());
    const int grid = 256 * 8 * 4, blk = 256;
    // the buffer is four 256-MiB regions; each kernel reads every byte of one region once
    auto run = [&](const char* name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        std::printf("%-12s bytes %zu\n", name, moved);
    };
    // (c_scalar64 re-reads region 0 after 768 MiB of other traffic: nothing of it is left in L2)
    run("c_stream16", [&] { c_stream16<<<grid, blk>>>((const v2d*)buf, moved / 16, out); });
    // the permuted patterns visit every piece of their region once, in the order of perm (a bijection)
    run("c_seg64", [&] { c_seg64<<<grid, blk>>>((const v2d*)buf + moved / 16, (unsigned)(moved / 64), out); });
    run("c_gather32", [&] { c_gather32<<<grid, blk>>>((const v2d*)buf + 2 * (moved / 16), (unsigned)(moved / 32), out); });
    run("c_gather8", [&] { c_gather8<<<grid, blk>>>((const double*)buf + 3 * (moved / 8), (unsigned)(moved / 8), out); });
    run("c_scalar64", [&] { c_scalar64<<<grid, blk>>>((const double*)buf, (unsigned)(moved / 64), out); });
    // 2^21 runs of 168 B (336 MiB) in region 0..1, every run once; bytes = 2^21 * 168
    {
        const unsigned nrun = 1u << 21;
        c_rows168<<<grid, blk>>>((const double*)buf, nrun, out);
        CK(hipDeviceSynchronize());
        std::printf("%-12s bytes %zu\n", "c_rows168", (size_t)nrun * 168);
    }
    run("w_stream16", [&] { w_stream16<<<grid, blk>>>((v2d*)buf + moved / 16, moved / 16); });
    run("w_seg64", [&] { w_seg64<<<grid, blk>>>((v2d*)buf + 2 * (moved / 16), (unsigned)(moved / 64)); });
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
