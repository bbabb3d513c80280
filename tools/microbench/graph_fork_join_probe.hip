// Does a stream that waits on an event recorded right after a hipGraphLaunch see the graph's work
// done?  The library's graph mode (cf_api.hip launch_full) replays three graphs per evaluation with
// event hand-overs between them:
//   main: PRO graph ; record fork ; [aux: wait fork ; DCH graph (memset node + kernels) ; record join]
//   main: REC graph ; wait join ; eager kernel (k_assemble_energy: clears the rebuild flag)
// This probe replays the same shape with kernels that only count: every kernel spins, then checks
// the counters its predecessors must have advanced, and counts violations (no memory access depends
// on the counters, so a violation cannot fault).  Variants: the DCH graph with / without a memset
// node first, events with the library's flags (DisableTiming | DisableSystemFence) or default, and
// the eager form of the same sequence as the control.
// Build: hipcc -O2 --offload-arch=gfx950 -o graph_fork_join_probe graph_fork_join_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

// counters: [0] PRO done, [1] DCH done, [2] REC done, [3] ASM done, [4] DCH's memset target,
// [8..] violations per check point
__device__ void spin(long cycles) {
    const long t0 = clock64();
    while (clock64() - t0 < cycles) {}
}
__device__ int ld(const int* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM); }
__device__ void st_inc(int* p) { __hip_atomic_fetch_add(p, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM); }

// Every kernel but ASM runs G blocks; each block checks at its start that its predecessors have
// finished (counters of finished blocks), spins, and counts itself finished at its end.
// PRO(n): ASM(n-1) done
__global__ void k_pro(int* c, long cyc, int G) {
    if (threadIdx.x) return;
    if (ld(c + 3) != ld(c + 0) / G) atomicAdd(c + 8, 1);
    spin(cyc);
    st_inc(c + 0);
}
// DCH(n): PRO(n) and DCH(n-1) done, and this graph's memset set c[4] = 1
__global__ void k_dch(int* c, long cyc, int check_memset, int G) {
    if (threadIdx.x) return;
    if (ld(c + 0) != G * (ld(c + 1) / G + 1)) atomicAdd(c + 9, 1);
    if (check_memset && ld(c + 4) != 1) atomicAdd(c + 10, 1);
    spin(cyc);
    st_inc(c + 1);
}
// REC(n): PRO(n) done
__global__ void k_rec(int* c, long cyc, int G) {
    if (threadIdx.x) return;
    if (ld(c + 0) != G * (ld(c + 2) / G + 1)) atomicAdd(c + 11, 1);
    spin(cyc);
    st_inc(c + 2);
}
// ASM(n) (one block): DCH(n) (the join) and REC(n) done; clears c[4] like the rebuild flag
__global__ void k_asm(int* c, int G) {
    if (threadIdx.x) return;
    const int n = ld(c + 3) + 1;
    if (ld(c + 1) != G * n) atomicAdd(c + 12, 1);
    if (ld(c + 2) != G * n) atomicAdd(c + 13, 1);
    __hip_atomic_store(c + 4, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    st_inc(c + 3);
}

static void ck(hipError_t e, const char* w) {
    if (e != hipSuccess) { printf("%s: %s\n", w, hipGetErrorString(e)); exit(1); }
}

template <class F>
static hipGraphExec_t capture(hipStream_t cap, F&& f) {
    hipGraph_t g = nullptr;
    ck(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal), "begin capture");
    f(cap);
    ck(hipStreamEndCapture(cap, &g), "end capture");
    hipGraphExec_t x = nullptr;
    ck(hipGraphInstantiate(&x, g, nullptr, nullptr, 0), "instantiate");
    (void)hipGraphDestroy(g);
    return x;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    const int G = argc > 2 ? atoi(argv[2]) : 1;   // blocks per kernel (the library's kernels: 32-4096)
    int* c;
    ck(hipMalloc(&c, 64 * sizeof(int)), "malloc");
    hipStream_t cap, main_s, aux;
    ck(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking), "stream");
    ck(hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking), "stream");
    // argv[3] == "null": the caller's stream is the null stream (torch's default current stream,
    // which the library's tests and bench hand to cf_options.stream)
    if (argc > 3 && argv[3][0] == 'n') main_s = nullptr;
    ck(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking), "stream");
    const char* names[6] = {"PRO after ASM(n-1)", "DCH after fork", "memset node first", "REC after PRO",
                            "ASM after join", "ASM after REC"};
    struct Case { const char* what; bool graph; bool memset; unsigned evf; long cyc_dch, cyc_rec; bool recapture; };
    const unsigned lib = hipEventDisableTiming | hipEventDisableSystemFence;
    Case cases[] = {
        {"eager, library events", false, true, lib, 40000, 20000, false},
        {"graph, memset node, library events", true, true, lib, 40000, 20000, false},
        {"graph, no memset node, library events", true, false, lib, 40000, 20000, false},
        {"graph, memset node, default events", true, true, 0u, 40000, 20000, false},
        {"graph, memset node, library events, slow REC", true, true, lib, 20000, 60000, false},
        {"graph, recapture 3 in 4, memset node, library events", true, true, lib, 40000, 20000, true},
        {"graph, recapture 3 in 4, no memset node", true, false, lib, 40000, 20000, true},
        {"graph, recapture 3 in 4, slow REC", true, true, lib, 20000, 60000, true},
    };
    for (const Case& cs : cases) {
        hipEvent_t fork, join;
        ck(hipEventCreateWithFlags(&fork, cs.evf), "event");
        ck(hipEventCreateWithFlags(&join, cs.evf), "event");
        ck(hipMemset(c, 0, 64 * sizeof(int)), "memset");
        ck(hipDeviceSynchronize(), "sync");
        auto pro = [&](hipStream_t s) { hipLaunchKernelGGL(k_pro, dim3(G), dim3(64), 0, s, c, 4000L, G); };
        auto dch = [&](hipStream_t s) {
            if (cs.memset) ck(hipMemsetD32Async(c + 4, 1, 1, s), "memsetD32");
            hipLaunchKernelGGL(k_dch, dim3(G), dim3(64), 0, s, c, cs.cyc_dch, cs.memset ? 1 : 0, G);
        };
        auto rec = [&](hipStream_t s) { hipLaunchKernelGGL(k_rec, dim3(G), dim3(64), 0, s, c, cs.cyc_rec, G); };
        hipGraphExec_t gp = nullptr, gd = nullptr, gr = nullptr;
        if (cs.graph) { gp = capture(cap, pro); gd = capture(cap, dch); gr = capture(cap, rec); }
        for (int it = 0; it < iters; it++) {
            // recapture: like cf_api.hip run_segment when the key changes (the flags alternate):
            // three evaluations in four re-capture every segment, draining only the stream the old
            // graph ran on (main for PRO / REC, aux for DCH) before destroying it
            const bool re = cs.recapture && (it % 4 != 3);
            if (re) {
                ck(hipStreamSynchronize(main_s), "drain"); ck(hipStreamSynchronize(aux), "drain");
                (void)hipGraphExecDestroy(gp); gp = capture(cap, pro);
            }
            if (cs.graph) ck(hipGraphLaunch(gp, main_s), "launch"); else pro(main_s);
            ck(hipEventRecord(fork, main_s), "record fork");
            ck(hipStreamWaitEvent(aux, fork, 0), "wait fork");
            if (re) { ck(hipStreamSynchronize(aux), "drain"); (void)hipGraphExecDestroy(gd); gd = capture(cap, dch); }
            if (cs.graph) ck(hipGraphLaunch(gd, aux), "launch"); else dch(aux);
            ck(hipEventRecord(join, aux), "record join");
            if (re) {
                ck(hipStreamSynchronize(main_s), "drain"); ck(hipStreamSynchronize(aux), "drain");
                (void)hipGraphExecDestroy(gr); gr = capture(cap, rec);
            }
            if (cs.graph) ck(hipGraphLaunch(gr, main_s), "launch"); else rec(main_s);
            ck(hipStreamWaitEvent(main_s, join, 0), "wait join");
            hipLaunchKernelGGL(k_asm, dim3(1), dim3(64), 0, main_s, c, G);
        }
        ck(hipDeviceSynchronize(), "sync");
        int h[64];
        ck(hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost), "copy");
        printf("%s %-52s G %d iterations %d (counters %d %d %d %d):", main_s ? "own main stream" : "null stream as main", cs.what, G, iters, h[0], h[1], h[2], h[3]);
        for (int k = 0; k < 6; k++) printf("  %s: %d", names[k], h[8 + k]);
        printf("\n");
        if (cs.graph) { (void)hipGraphExecDestroy(gp); (void)hipGraphExecDestroy(gd); (void)hipGraphExecDestroy(gr); }
        (void)hipEventDestroy(fork);
        (void)hipEventDestroy(join);
    }
    return 0;
}
