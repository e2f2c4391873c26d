// What a kernel can learn about its own dispatch: the AQL packet's header (barrier bit), the queue
// it was read from, and its dispatch id, under each way the library gets launched (legacy null
// stream, created streams beyond GPU_MAX_HW_QUEUES, hipStreamPerThread from two threads, a graph
// replayed on two streams). Also times two long kernels on streams that share an HSA queue to see
// whether they overlap. Experiment for the status-histogram tree's per-queue ownership.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <thread>
#include <vector>

struct Info {
    unsigned long long queue, dispatch_id, pkt;
    unsigned header;
    unsigned long long t0, t1;
};

__global__ void probe(Info* out, int slot, unsigned long long spin) {
    if (threadIdx.x || blockIdx.x) return;
    if (slot < 0) slot = 48 + atomicAdd(reinterpret_cast<int*>(out + 63), 1);
    const uint16_t* pkt = (const uint16_t*)(__builtin_amdgcn_dispatch_ptr());
    Info i;
    i.queue = (unsigned long long)(__builtin_amdgcn_queue_ptr());
    i.dispatch_id = 0;
    i.pkt = reinterpret_cast<unsigned long long>(pkt);
    i.header = pkt[0];
    i.t0 = wall_clock64();
    while (wall_clock64() - i.t0 < spin) {
    }
    i.t1 = wall_clock64();
    out[slot] = i;
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            return 1;                                                          \
        }                                                                      \
    } while (0)

static void show(const char* what, const Info& i) {
    printf("%-28s queue=%#llx id=%llu pkt=%#llx header=%#06x barrier=%u t=[%llu,%llu]\n", what, i.queue,
           i.dispatch_id, i.pkt, i.header, (i.header >> 8) & 1u, i.t0, i.t1);
}

int main() {
    Info* d;
    CK(hipMalloc(&d, 64 * sizeof(Info)));
    CK(hipMemset(d, 0, 64 * sizeof(Info)));
    int slot = 0;
    const unsigned long long spin = 100000;  // 1 ms at 100 MHz
    hipLaunchKernelGGL(probe, 1, 64, 0, 0, d, slot++, 0);
    hipLaunchKernelGGL(probe, 1, 64, 0, 0, d, slot++, 0);
    CK(hipDeviceSynchronize());
    std::vector<hipStream_t> ss(10);
    for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int first_stream = slot;
    for (auto& s : ss) hipLaunchKernelGGL(probe, 1, 64, 0, s, d, slot++, spin);
    CK(hipDeviceSynchronize());
    const int first_pt = slot;
    std::thread a([&] { hipLaunchKernelGGL(probe, 1, 64, 0, hipStreamPerThread, d, first_pt, spin);
                        hipStreamSynchronize(hipStreamPerThread); });
    std::thread b([&] { hipLaunchKernelGGL(probe, 1, 64, 0, hipStreamPerThread, d, first_pt + 1, spin);
                        hipStreamSynchronize(hipStreamPerThread); });
    a.join();
    b.join();
    slot += 2;
    // a graph of one node, replayed on two streams at once
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(ss[0], hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(probe, 1, 64, 0, ss[0], d, -1, spin);
    CK(hipStreamEndCapture(ss[0], &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, ss[1]));
    CK(hipDeviceSynchronize());
    Info h1[64];
    CK(hipMemcpy(h1, d, sizeof(h1), hipMemcpyDeviceToHost));
    CK(hipGraphLaunch(ge, ss[1]));
    CK(hipGraphLaunch(ge, ss[2]));
    CK(hipDeviceSynchronize());
    Info h[64];
    CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    show("null stream #0", h[0]);
    show("null stream #1", h[1]);
    for (int k = 0; k < 10; ++k) {
        char buf[64];
        snprintf(buf, sizeof buf, "stream %d", k);
        show(buf, h[first_stream + k]);
    }
    show("per-thread A", h[first_pt]);
    show("per-thread B", h[first_pt + 1]);
    show("graph replay (alone)", h1[48]);
    show("graph replay on ss1", h[49]);
    show("graph replay on ss2", h[50]);
    printf("graph replays overlap=%d\n", !(h[49].t1 <= h[50].t0 || h[50].t1 <= h[49].t0));
    // overlap between streams that share a queue
    for (int x = 0; x < 10; ++x)
        for (int y = x + 1; y < 10; ++y) {
            const Info &p = h[first_stream + x], &q = h[first_stream + y];
            if (p.queue == q.queue)
                printf("streams %d,%d share queue: overlap=%d\n", x, y, !(p.t1 <= q.t0 || q.t1 <= p.t0));
        }
    {
        const Info &p = h[first_pt], &q = h[first_pt + 1];
        printf("per-thread A,B same queue=%d overlap=%d\n", p.queue == q.queue, !(p.t1 <= q.t0 || q.t1 <= p.t0));
    }
    return 0;
}
