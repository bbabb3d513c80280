// fp64 throughput microbenchmark for the roofline denominator (MI355X_MICROARCH.md lists
// no FP64 matrix rate): v_mfma_f64_16x16x4_f64 and v_fma_f64 on every CU, random data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) mfma_loop(const double* in, double* out, int iters) {
    double a = in[threadIdx.x], b = in[threadIdx.x + 256];
    d4 acc[8];
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = (d4){in[k], in[k + 1], in[k + 2], in[k + 3]};
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
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

int main() {
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    std::vector<double> h(1024);
    for (int i = 0; i < 1024; i++) h[i] = 0.5 + 1e-3 * ((i * 7919) % 1000) / 1000.0;
    double *in, *out;
    hipMalloc(&in, 1024 * 8);
    hipMalloc(&out, (size_t)ncu * 8 * 256 * 8);
    hipMemcpy(in, h.data(), 1024 * 8, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int bpc = 1; bpc <= 4; bpc *= 2) {  // 4-wave blocks per CU = waves per SIMD
        int blocks = ncu * bpc;
        int iters = 20000;
        float ms;
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a);
            hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, in, out, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        double flops = (double)blocks * 4 /*waves*/ * iters * 8 * 2048.0;
        printf("waves/SIMD=%d mfma_f64_16x16x4 (8 acc): %.2f TFLOP/s\n", bpc, flops / ms / 1e9);
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a);
            hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(256), 0, 0, in, out, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        flops = (double)blocks * 256 * iters * 16 * 2.0;
        printf("waves/SIMD=%d v_fma_f64 (16 chains):     %.2f TFLOP/s\n", bpc, flops / ms / 1e9);
    }
    return 0;
}
