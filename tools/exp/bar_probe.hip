// Tools only: can the host write straight into device memory (large BAR), and what does a
// host -> GPU -> host ping-pong cost when the request side lives there instead of in pinned host
// memory? Every spin is bounded (iterations and a real-time deadline) so the kernel always exits.
// build: hipcc --offload-arch=gfx950 -O2 tools/exp/bar_probe.hip -o tools/exp/bar_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                    \
            return 1;                                                              \
        }                                                                          \
    } while (0)

// Serves `rounds` requests: waits for *req == k (request side), then writes *ack = k (response side).
// Gives up after `deadline_ticks` of the 100 MHz real-time counter without a request.
__global__ void pingpong(const uint32_t* req, uint32_t* ack, uint32_t rounds, uint64_t deadline_ticks,
                         uint32_t* status) {
    if (threadIdx.x != 0) return;
    for (uint32_t k = 1; k <= rounds; ++k) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t v = 0;
        for (;;) {
            v = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
            if (v >= k) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > deadline_ticks) {
                status[0] = 0xDEADu;
                status[1] = k;
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(ack, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    status[0] = 1;
}

static double pingpong_us(volatile uint32_t* h_req, uint32_t* d_req, volatile uint32_t* h_ack, uint32_t* d_ack,
                          uint32_t* d_status, uint32_t rounds) {
    *h_req = 0;
    *h_ack = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    hipLaunchKernelGGL(pingpong, dim3(1), dim3(64), 0, nullptr, d_req, d_ack, rounds, 200000000ull /* 2 s */,
                       d_status);
    // let the kernel start
    const auto tw = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - tw < std::chrono::milliseconds(20)) {
    }
    std::vector<double> us;
    for (uint32_t k = 1; k <= rounds; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        *h_req = k;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        bool ok = false;
        for (long spin = 0; spin < 200000000L; ++spin) {
            if (*h_ack >= k) {
                ok = true;
                break;
            }
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (!ok) {
            printf("  host gave up at round %u\n", k);
            break;
        }
        us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    (void)hipDeviceSynchronize();
    if (us.empty()) return -1;
    std::sort(us.begin(), us.end());
    return us[us.size() / 2];
}

int main() {
    int dev = 0, large_bar = -1, host_atomic = -1;
    CK(hipSetDevice(dev));
    CK(hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, dev));
    (void)hipDeviceGetAttribute(&host_atomic, hipDeviceAttributeHostNativeAtomicSupported, dev);
    printf("isLargeBar=%d hostNativeAtomic=%d\n", large_bar, host_atomic);

    uint32_t* d_status = nullptr;
    CK(hipMalloc(&d_status, 64));
    CK(hipMemset(d_status, 0, 64));

    // pinned host request + pinned host ack: the current resident-consumer layout
    uint32_t *h_req = nullptr, *h_ack = nullptr, *d_hreq = nullptr, *d_hack = nullptr;
    CK(hipHostMalloc(&h_req, 4096, hipHostMallocDefault));
    CK(hipHostMalloc(&h_ack, 4096, hipHostMallocDefault));
    CK(hipHostGetDevicePointer((void**)&d_hreq, h_req, 0));
    CK(hipHostGetDevicePointer((void**)&d_hack, h_ack, 0));
    printf("pinned req / pinned ack: median %.2f us per round trip\n",
           pingpong_us(h_req, d_hreq, h_ack, d_hack, d_status, 2000));

    if (large_bar != 1) {
        printf("no large BAR: the host cannot map device memory\n");
        return 0;
    }
    for (unsigned flags : {(unsigned)hipDeviceMallocFinegrained, (unsigned)hipDeviceMallocUncached}) {
        uint32_t* d = nullptr;
        hipError_t e = hipExtMallocWithFlags((void**)&d, 1 << 20, flags);
        if (e != hipSuccess) {
            printf("hipExtMallocWithFlags(%u): %s\n", flags, hipGetErrorString(e));
            continue;
        }
        hipPointerAttribute_t a{};
        e = hipPointerGetAttributes(&a, d);
        printf("flags %u: dev ptr %p attr rc=%d type=%d hostPointer=%p\n", flags, (void*)d, (int)e, (int)a.type,
               a.hostPointer);
        // the host writes through the same address (ROCm maps large-BAR VRAM into the process)
        volatile uint32_t* hv = d;
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < 1000; ++r)
            for (int i = 0; i < 1024; ++i) hv[i] = 0xA5000000u + i + r;
        const auto t1 = std::chrono::steady_clock::now();
        std::vector<uint32_t> back(1024);
        CK(hipMemcpy(back.data(), d, 4096, hipMemcpyDeviceToHost));
        bool ok = true;
        for (int i = 0; i < 1024; ++i) ok = ok && back[i] == 0xA5000000u + i + 999;
        printf("  host wrote 1000 x 4 KB in %.1f us (%.2f us per 4 KB), readback %s\n",
               std::chrono::duration<double, std::micro>(t1 - t0).count(),
               std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000, ok ? "ok" : "MISMATCH");
        printf("  device req / pinned ack: median %.2f us per round trip\n",
               pingpong_us(hv, d, h_ack, d_hack, d_status, 2000));
        uint32_t st[2] = {0, 0};
        CK(hipMemcpy(st, d_status, 8, hipMemcpyDeviceToHost));
        printf("  kernel status %x round %u\n", st[0], st[1]);
        CK(hipFree(d));
    }
    return 0;
}
