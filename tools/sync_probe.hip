// Cross-stream synchronization latency on one device (tools/sync_probe.hip).
// Two streams A and B; each iteration runs a tiny kernel on A, hands over to B (which runs a
// tiny kernel), and hands back to A.  Per iteration time for each hand-over mechanism:
//   none      both kernels on A (no cross-stream dependency: the floor)
//   event     hipEventRecord + hipStreamWaitEvent (default flags, DisableTiming)
//   evdev     the same with hipEventDisableSystemFence
//   value     hipStreamWriteValue32 on the producer, hipStreamWaitValue32 on the consumer
// build: hipcc -O2 --offload-arch=gfx950 tools/sync_probe.hip -o tools/sync_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

__global__ void tiny(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

int main() {
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    int* buf;
    CK(hipMalloc(&buf, 64 * sizeof(int)));
    CK(hipMemset(buf, 0, 64 * sizeof(int)));
    unsigned* flag;
    CK(hipMalloc(&flag, 2 * sizeof(unsigned)));
    CK(hipMemset(flag, 0, 2 * sizeof(unsigned)));
    hipEvent_t e1, e2, d1, d2;
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&d1, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&d2, hipEventDisableTiming | hipEventDisableSystemFence));
    const int iters = 400;
    for (int mode = 0; mode < 4; mode++) {
        for (int rep = 0; rep < 2; rep++) {
            CK(hipDeviceSynchronize());
            unsigned seq = 0;
            CK(hipMemset(flag, 0, 2 * sizeof(unsigned)));
            CK(hipDeviceSynchronize());
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < iters; i++) {
                hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, a, buf);
                if (mode == 0) {
                    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, a, buf + 16);
                } else if (mode == 1 || mode == 2) {
                    hipEvent_t x = mode == 1 ? e1 : d1, y = mode == 1 ? e2 : d2;
                    CK(hipEventRecord(x, a));
                    CK(hipStreamWaitEvent(b, x, 0));
                    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, b, buf + 16);
                    CK(hipEventRecord(y, b));
                    CK(hipStreamWaitEvent(a, y, 0));
                } else {
                    seq++;
                    CK(hipStreamWriteValue32(a, flag, seq, 0));
                    CK(hipStreamWaitValue32(b, flag, seq, hipStreamWaitValueGte, 0xffffffffu));
                    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, b, buf + 16);
                    CK(hipStreamWriteValue32(b, flag + 1, seq, 0));
                    CK(hipStreamWaitValue32(a, flag + 1, seq, hipStreamWaitValueGte, 0xffffffffu));
                }
            }
            CK(hipStreamSynchronize(a));
            CK(hipStreamSynchronize(b));
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            const char* names[] = {"none", "event", "evdev", "value"};
            std::printf("%-6s rep %d: %.2f us per iteration (2 kernels, 2 hand-overs)\n", names[mode], rep, us / iters);
        }
    }
    return 0;
}
