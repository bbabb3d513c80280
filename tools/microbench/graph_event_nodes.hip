// Which event-record forms can sit inside a captured hipGraph on this runtime (cf_api.hip graph
// mode): hipEventRecordWithFlags(..., hipEventRecordExternal) during stream capture and
// hipGraphAddEventRecordNode, for events created with the flags the library uses.  Prints the
// return code of every attempt and, for the forms that capture, whether a stream waiting on the
// event after the graph launch sees the graph's kernel done.
// Build: hipcc -O2 --offload-arch=gfx950 -o graph_event_nodes graph_event_nodes.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_spin(int* p, long iters) {
    if (threadIdx.x == 0) {
        long t0 = clock64();
        while (clock64() - t0 < iters) {}
        *p = 1;
    }
}
__global__ void k_read(const int* p, int* out) {
    if (threadIdx.x == 0) *out = *p;
}

static const char* name(hipError_t e) { return hipGetErrorName(e); }

int main() {
    int *flag, *seen;
    (void)hipMalloc(&flag, sizeof(int));
    (void)hipMalloc(&seen, sizeof(int));
    hipStream_t cap, main_s, aux;
    (void)hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&aux, hipStreamNonBlocking);
    const unsigned flag_sets[3] = {0u, hipEventDisableTiming, hipEventDisableTiming | hipEventDisableSystemFence};
    const char* flag_names[3] = {"default", "DisableTiming", "DisableTiming|DisableSystemFence"};
    for (int f = 0; f < 3; f++) {
        hipEvent_t ev;
        (void)hipEventCreateWithFlags(&ev, flag_sets[f]);
        // (a) record with hipEventRecordExternal during capture
        hipGraph_t g = nullptr;
        hipError_t eb = hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, cap, flag, 20000000L);
        hipError_t er = hipEventRecordWithFlags(ev, cap, hipEventRecordExternal);
        hipError_t ee = hipStreamEndCapture(cap, &g);
        printf("[%s] capture: begin %s, record(External) %s, end %s\n", flag_names[f], name(eb), name(er), name(ee));
        if (er == hipSuccess && ee == hipSuccess && g) {
            hipGraphExec_t x = nullptr;
            hipError_t ei = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
            (void)hipMemset(flag, 0, sizeof(int));
            (void)hipMemset(seen, -1, sizeof(int));
            (void)hipDeviceSynchronize();
            hipError_t el = hipGraphLaunch(x, main_s);
            hipError_t ew = hipStreamWaitEvent(aux, ev, 0);
            hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, aux, flag, seen);
            hipError_t es = hipDeviceSynchronize();
            int h = -1;
            (void)hipMemcpy(&h, seen, sizeof(int), hipMemcpyDeviceToHost);
            printf("    instantiate %s, launch %s, wait %s, sync %s: consumer saw flag = %d (1 = ordered)\n", name(ei),
                   name(el), name(ew), name(es), h);
            if (x) (void)hipGraphExecDestroy(x);
        }
        if (g) (void)hipGraphDestroy(g);
        // (b) explicit event-record node after a captured kernel node
        hipGraph_t g2 = nullptr;
        (void)hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, cap, flag, 20000000L);
        (void)hipStreamEndCapture(cap, &g2);
        size_t n = 0;
        (void)hipGraphGetNodes(g2, nullptr, &n);
        hipGraphNode_t nodes[8];
        (void)hipGraphGetNodes(g2, nodes, &n);
        hipGraphNode_t rec = nullptr;
        hipError_t ea = hipGraphAddEventRecordNode(&rec, g2, nodes, n, ev);
        printf("[%s] hipGraphAddEventRecordNode after %zu captured node(s): %s\n", flag_names[f], n, name(ea));
        if (ea == hipSuccess) {
            hipGraphExec_t x = nullptr;
            hipError_t ei = hipGraphInstantiate(&x, g2, nullptr, nullptr, 0);
            (void)hipMemset(flag, 0, sizeof(int));
            (void)hipMemset(seen, -1, sizeof(int));
            (void)hipDeviceSynchronize();
            hipError_t el = hipGraphLaunch(x, main_s);
            hipError_t ew = hipStreamWaitEvent(aux, ev, 0);
            hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, aux, flag, seen);
            hipError_t es = hipDeviceSynchronize();
            int h = -1;
            (void)hipMemcpy(&h, seen, sizeof(int), hipMemcpyDeviceToHost);
            printf("    instantiate %s, launch %s, wait %s, sync %s: consumer saw flag = %d (1 = ordered)\n", name(ei),
                   name(el), name(ew), name(es), h);
            if (x) (void)hipGraphExecDestroy(x);
        }
        if (g2) (void)hipGraphDestroy(g2);
        (void)hipEventDestroy(ev);
    }
    // (c) the library's sequence: capture with the record node, replay several times (a stream
    // waiting on the event each time), then capture again with the same event (a new key), and an
    // eager record of the event on another stream in between
    {
        hipEvent_t ev;
        (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence);
        for (int round = 0; round < 3; round++) {
            hipGraph_t g = nullptr;
            (void)hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, cap, flag, 2000000L);
            hipError_t er = hipEventRecordWithFlags(ev, cap, hipEventRecordExternal);
            hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, cap, flag, seen);
            hipError_t ee = hipStreamEndCapture(cap, &g);
            hipGraphExec_t x = nullptr;
            hipError_t ei = (ee == hipSuccess && g) ? hipGraphInstantiate(&x, g, nullptr, nullptr, 0) : ee;
            int ok = 0;
            for (int rep = 0; rep < 4 && x; rep++) {
                (void)hipGraphLaunch(x, main_s);
                (void)hipStreamWaitEvent(aux, ev, 0);
                hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, aux, flag, seen);
                ok += hipStreamSynchronize(aux) == hipSuccess;
            }
            (void)hipDeviceSynchronize();
            hipError_t eg = hipEventRecord(ev, aux);   // eager record between captures
            hipError_t es = hipDeviceSynchronize();
            printf("[sequence round %d] record(External) %s, end %s, instantiate %s, replays ok %d/4, eager record %s, sync %s\n",
                   round, name(er), name(ee), name(ei), ok, name(eg), name(es));
            if (x) (void)hipGraphExecDestroy(x);
            if (g) (void)hipGraphDestroy(g);
        }
        (void)hipEventDestroy(ev);
    }
    // (d) as (c) with the graphs launched on the legacy null stream (a torch current stream of 0)
    // after eager work on it, and the waits on a second non-blocking stream
    {
        hipEvent_t ev;
        (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence);
        hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, 0, flag, seen);   // eager work on the null stream
        for (int round = 0; round < 2; round++) {
            hipGraph_t g = nullptr;
            hipError_t eb = hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, cap, flag, 2000000L);
            hipError_t er = hipEventRecordWithFlags(ev, cap, hipEventRecordExternal);
            hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, cap, flag, seen);
            hipError_t ee = hipStreamEndCapture(cap, &g);
            hipGraphExec_t x = nullptr;
            hipError_t ei = (ee == hipSuccess && g) ? hipGraphInstantiate(&x, g, nullptr, nullptr, 0) : ee;
            int ok = 0;
            for (int rep = 0; rep < 4 && x; rep++) {
                (void)hipGraphLaunch(x, 0);
                (void)hipStreamWaitEvent(aux, ev, 0);
                hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, aux, flag, seen);
                ok += hipStreamSynchronize(aux) == hipSuccess;
            }
            hipError_t es = hipDeviceSynchronize();
            printf("[null-stream round %d] begin %s, record(External) %s, end %s, instantiate %s, replays ok %d/4, sync %s\n",
                   round, name(eb), name(er), name(ee), name(ei), ok, name(es));
            if (x) (void)hipGraphExecDestroy(x);
            if (g) (void)hipGraphDestroy(g);
        }
        (void)hipEventDestroy(ev);
    }
    // (e) a captured graph as a child node, an event-record node after it, a second captured graph
    // as a child node after the record (the explicit form of (c))
    {
        hipEvent_t ev;
        (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence);
        hipGraph_t ga = nullptr, gb = nullptr, g = nullptr;
        (void)hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, cap, flag, 2000000L);
        (void)hipStreamEndCapture(cap, &ga);
        (void)hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
        hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, cap, flag, seen);
        (void)hipStreamEndCapture(cap, &gb);
        hipError_t ec = hipGraphCreate(&g, 0);
        hipGraphNode_t na = nullptr, nr = nullptr, nb = nullptr;
        hipError_t e1 = hipGraphAddChildGraphNode(&na, g, nullptr, 0, ga);
        hipError_t e2 = hipGraphAddEventRecordNode(&nr, g, &na, 1, ev);
        hipError_t e3 = hipGraphAddChildGraphNode(&nb, g, &nr, 1, gb);
        hipGraphExec_t x = nullptr;
        hipError_t ei = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
        int ok = 0;
        for (int rep = 0; rep < 4 && x; rep++) {
            (void)hipMemset(seen, -1, sizeof(int));
            (void)hipMemset(flag, 0, sizeof(int));
            (void)hipDeviceSynchronize();
            (void)hipGraphLaunch(x, 0);
            (void)hipStreamWaitEvent(aux, ev, 0);
            hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, aux, flag, seen);
            (void)hipDeviceSynchronize();
            int h = -1;
            (void)hipMemcpy(&h, seen, sizeof(int), hipMemcpyDeviceToHost);
            ok += h == 1;
        }
        printf("[child graphs + record node] create %s, child %s, record %s, child %s, instantiate %s, ordered %d/4\n",
               name(ec), name(e1), name(e2), name(e3), name(ei), ok);
        if (x) (void)hipGraphExecDestroy(x);
        (void)hipGraphDestroy(g); (void)hipGraphDestroy(ga); (void)hipGraphDestroy(gb);
        (void)hipEventDestroy(ev);
    }
    return 0;
}
