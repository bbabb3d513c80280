// Accuracy of v_rsq_f64 and of one / two Newton steps on it, over r^2 in [1e-3, 4]
// (the pair kernel's range), against 1/sqrt in long double on the host.
// hipcc --offload-arch=gfx950 -O3 -o tools/rsq_probe tools/rsq_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const double* x, double* y0, double* y1, double* y2, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double r2 = x[i];
    double y = __builtin_amdgcn_rsq(r2);
    y0[i] = y;
    const double h = 0.5 * r2;
    y = y * fma(-h * y, y, 1.5);
    y1[i] = y;
    y = y * fma(-h * y, y, 1.5);
    y2[i] = y;
}

int main() {
    const int n = 1 << 22;
    std::vector<double> x(n), y0(n), y1(n), y2(n);
    for (int i = 0; i < n; i++) x[i] = 1e-3 * std::pow(4000.0, (i + 0.5) / n);
    double *dx, *d0, *d1, *d2;
    (void)hipMalloc(&dx, n * 8); (void)hipMalloc(&d0, n * 8); (void)hipMalloc(&d1, n * 8); (void)hipMalloc(&d2, n * 8);
    (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, dx, d0, d1, d2, n);
    (void)hipMemcpy(y0.data(), d0, n * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(y1.data(), d1, n * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(y2.data(), d2, n * 8, hipMemcpyDeviceToHost);
    double e0 = 0, e1 = 0, e2 = 0;
    for (int i = 0; i < n; i++) {
        long double ex = 1.0L / sqrtl((long double)x[i]);
        e0 = std::fmax(e0, (double)fabsl((y0[i] - ex) / ex));
        e1 = std::fmax(e1, (double)fabsl((y1[i] - ex) / ex));
        e2 = std::fmax(e2, (double)fabsl((y2[i] - ex) / ex));
    }
    std::printf("max rel error: v_rsq_f64 %.3e  one Newton %.3e  two Newton %.3e  (ulp %.3e)\n", e0, e1, e2,
                std::ldexp(1.0, -52));
    return 0;
}
