// Issue cost of the fp64 VALU forms the interpolation uses, on one MI355X (gfx950):
//   fma   : v_fma_f64 with VGPR operands
//   dpp   : v_fmac_f64_dpp row_newbcast (the k_g_interp2 contraction)
//   sgpr  : v_fma_f64 with an SGPR operand
// Every CU runs `waves` waves per SIMD of a loop of 8 independent accumulation chains; the
// result is cycles per wave-instruction per SIMD at the measured clock (clock from
// s_memtime / s_memrealtime inside the kernel, 100 MHz real-time counter).
// Build: hipcc -O3 --offload-arch=gfx950 -o f64_issue f64_issue.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kIters = 4096;

template <int MODE>
__global__ void __launch_bounds__(256) k_issue(double* out, double s, long long* clk) {
    double a[8];
    const double x = threadIdx.x * 1e-3, y = 1.0 + threadIdx.x * 1e-6;
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = i;
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if constexpr (MODE == 0) {
                asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(y));
            } else if constexpr (MODE == 1) {
                asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(x), "v"(y));
            } else {
                asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a[i]) : "v"(x), "s"(s));
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int MODE>
static void run(const char* name, int waves_per_simd, int ncu) {
    const int blocks = ncu * waves_per_simd;   // 256 threads = 4 waves = one per SIMD
    double* out;
    long long* clk;
    hipMalloc(&out, sizeof(double) * blocks * 256);
    hipMalloc(&clk, sizeof(long long) * 2 * blocks);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(k_issue<MODE>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, clk);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_issue<MODE>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    long long* h = (long long*)malloc(sizeof(long long) * 2 * blocks);
    hipMemcpy(h, clk, sizeof(long long) * 2 * blocks, hipMemcpyDeviceToHost);
    double cyc = 0, real = 0;
    for (int b = 0; b < blocks; b++) { cyc += h[2 * b]; real += h[2 * b + 1]; }
    cyc /= blocks; real /= blocks;
    const double ghz = cyc / (real / 100e6) / 1e9;
    const double instr_per_simd = (double)waves_per_simd * kIters * 8;
    // cycles per wave-instruction per SIMD over the loop (all waves of a SIMD resident together)
    printf("%-5s waves/SIMD %d: %.2f cyc per instruction per SIMD (loop %.0f cyc, %.2f GHz), kernel %.3f ms\n", name,
           waves_per_simd, cyc / instr_per_simd, cyc, ghz, ms);
    free(h);
    hipFree(out);
    hipFree(clk);
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int w : {1, 2, 4}) {
        run<0>("fma", w, ncu);
        run<1>("dpp", w, ncu);
        run<2>("sgpr", w, ncu);
    }
    return 0;
}
