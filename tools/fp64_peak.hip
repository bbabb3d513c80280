// fp64 throughput microbenchmark for the roofline denominator (MI355X_MICROARCH.md lists
// no FP64 matrix rate): v_mfma_f64_16x16x4_f64 with NACC independent accumulators per
// wave and v_fma_f64 with 16 chains, at 1/2/4 waves per SIMD, on every CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

// NOTE: __launch_bounds__(512) keeps the accumulators in arch VGPRs.  With (256) hipcc
// (ROCm 7.2) placed them in AGPRs and copied them back and forth around every group of
// MFMAs, which halves the measured rate (r01 first measurement: 47 TF/s).
template <int NACC>
__global__ void __launch_bounds__(512) mfma_loop(const double* in, double* out, int iters) {
    double a = in[threadIdx.x], b = in[threadIdx.x + 256];
    d4 acc[NACC];
#pragma unroll
    for (int k = 0; k < NACC; k++) acc[k] = (d4){in[k], in[k + 1], in[k + 2], in[k + 3]};
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < NACC; k++) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < NACC; k++) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) fma_loop(const double* in, double* out, int iters) {
    double x[16];
    double m = in[threadIdx.x], c = in[threadIdx.x + 1];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = in[k + threadIdx.x % 7];
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 16; k++) x[k] = fma(x[k], m, c);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) s += x[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// co-issue probe: waves 0-3 of a 512-thread block run MFMA, waves 4-7 run v_fma_f64
__global__ void __launch_bounds__(512) mixed_loop(const double* in, double* out, int iters_m, int iters_v) {
    if (threadIdx.x < 256) {
        double a = in[threadIdx.x], b = in[threadIdx.x + 256];
        d4 acc[4];
#pragma unroll
        for (int k = 0; k < 4; k++) acc[k] = (d4){in[k], in[k + 1], in[k + 2], in[k + 3]};
        for (int it = 0; it < iters_m; it++) {
#pragma unroll
            for (int k = 0; k < 4; k++) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
        }
        double s = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
        out[blockIdx.x * 512 + threadIdx.x] = s;
    } else {
        double x[16];
        double m = in[threadIdx.x - 256], c = in[threadIdx.x - 255];
#pragma unroll
        for (int k = 0; k < 16; k++) x[k] = in[k + threadIdx.x % 7];
        for (int it = 0; it < iters_v; it++) {
#pragma unroll
            for (int k = 0; k < 16; k++) x[k] = fma(x[k], m, c);
        }
        double s = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) s += x[k];
        out[blockIdx.x * 512 + threadIdx.x] = s;
    }
}

static hipEvent_t ea, eb;

template <int NACC>
void run_mfma(const double* in, double* out, int ncu, int bpc) {
    // bpc = waves per SIMD: 512-thread blocks hold 2 waves per SIMD, so bpc=1 uses 256 threads
    int threads = bpc == 1 ? 256 : 512;
    int blocks = ncu * (bpc == 1 ? 1 : bpc / 2), iters = 160000 / NACC;
    float ms = 0;
    for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(ea);
        hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
        (void)hipEventRecord(eb);
        (void)hipEventSynchronize(eb);
        (void)hipEventElapsedTime(&ms, ea, eb);
    }
    double flops = (double)blocks * (threads / 64) * iters * NACC * 2048.0;
    printf("waves/SIMD=%d mfma_f64_16x16x4 acc=%2d: %6.2f TFLOP/s\n", bpc, NACC, flops / ms / 1e9);
}

int main() {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<double> h(1024);
    for (int i = 0; i < 1024; i++) h[i] = 0.5 + 1e-3 * ((i * 7919) % 1000) / 1000.0;
    double *in, *out;
    (void)hipMalloc(&in, 1024 * 8);
    (void)hipMalloc(&out, (size_t)ncu * 8 * 512 * 8);
    (void)hipMemcpy(in, h.data(), 1024 * 8, hipMemcpyHostToDevice);
    (void)hipEventCreate(&ea); (void)hipEventCreate(&eb);
    for (int bpc = 1; bpc <= 4; bpc *= 2) {
        run_mfma<2>(in, out, ncu, bpc);
        run_mfma<4>(in, out, ncu, bpc);
        run_mfma<8>(in, out, ncu, bpc);
        run_mfma<16>(in, out, ncu, bpc);
        int blocks = ncu * bpc, iters = 20000;
        float ms = 0;
        for (int rep = 0; rep < 2; rep++) {
            (void)hipEventRecord(ea);
            hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(256), 0, 0, in, out, iters);
            (void)hipEventRecord(eb);
            (void)hipEventSynchronize(eb);
            (void)hipEventElapsedTime(&ms, ea, eb);
        }
        double flops = (double)blocks * 256 * iters * 16 * 2.0;
        printf("waves/SIMD=%d v_fma_f64 16 chains:     %6.2f TFLOP/s\n", bpc, flops / ms / 1e9);
    }
    // co-issue: same MFMA work as 'waves/SIMD=1 acc=4' plus VALU work sized to take about as long
    for (int vshare = 0; vshare <= 2; vshare++) {
        int iters_m = 40000, iters_v = vshare == 0 ? 0 : (vshare == 1 ? 15000 : 30000);
        float ms = 0;
        for (int rep = 0; rep < 2; rep++) {
            (void)hipEventRecord(ea);
            hipLaunchKernelGGL(mixed_loop, dim3(ncu), dim3(512), 0, 0, in, out, iters_m, iters_v);
            (void)hipEventRecord(eb);
            (void)hipEventSynchronize(eb);
            (void)hipEventElapsedTime(&ms, ea, eb);
        }
        double fm = (double)ncu * 4 * iters_m * 4 * 2048.0;
        double fv = (double)ncu * 256 * iters_v * 16 * 2.0;
        printf("co-issue: MFMA %.2f TF + VALU %.2f TF = %.2f TF (%.3f ms)\n", fm / ms / 1e9, fv / ms / 1e9,
               (fm + fv) / ms / 1e9, ms);
    }
    return 0;
}
