// resident.hip — the host side of the resident consumer (rx_parse.hip ring_service_kernel): one
// control block in pinned coherent memory, one kernel that stays on kSvcGroups CUs while requests
// keep coming, and the registry that lets a device drain stop every consumer first.
//
// Two users: rings attached with HALO_RING_PERSISTENT (ring_rx.hip, BASELINE config 1) and host
// contexts with halo_rx_host_ctx_set_resident (host_path.hip: PacketHandle-sized batches of a cgo
// caller, and the single-frame Parse* wrappers). Both replace a launch + stream synchronisation
// per call (~17-20 us on these boxes, profiles/r03/r3c/ringprof) with a request line the consumer
// polls and per-group completion slots the host polls.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <new>
#include <vector>

#include "halo_common.h"

namespace halo {

struct Resident {
    int device = 0;
    RingServiceCtl* ctl = nullptr;    // pinned, coherent
    RingServiceCtl* d_ctl = nullptr;  // its device address
    uint32_t* d_quit = nullptr;       // device word: a group that idled out tells the others
    hipStream_t stream = nullptr;
    const uint8_t* d_data = nullptr;
    const uint32_t* d_off = nullptr;
    const uint16_t* d_len = nullptr;
    std::mutex mu;                    // one request at a time; a drain parks under it
    uint32_t seq = 0;                 // the last request made
    bool launched = false;
    std::chrono::steady_clock::time_point last_done{};
    uint64_t timeout_us = 2000000;
    ResidentStats st{};
};

namespace {
using clk = std::chrono::steady_clock;

std::mutex g_live_mu;            // guards g_live; taken before any Resident::mu
std::vector<Resident*> g_live;
std::atomic<int> g_parked[64];   // per device: drains in progress

bool parked(int device) { return device >= 0 && device < 64 && g_parked[device].load(std::memory_order_acquire) > 0; }

// The consumer is stopped and its kernel has ended (s->mu held). The stop flag is cleared again
// once the grid is gone, so the next launch starts clean.
void stop_locked(Resident* s) {
    if (!s->launched) return;
    __atomic_store_n(&s->ctl->stop, 1u, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(s->stream);
    __atomic_store_n(&s->ctl->stop, 0u, __ATOMIC_RELEASE);
    s->launched = false;
}

bool launch_locked(Resident* s, uint32_t last) {
    s->launched = launch_ring_service(s->d_ctl, s->d_data, s->d_off, s->d_len, s->d_quit, last, kSvcIdleUs,
                                      s->stream) == HALO_OK;
    s->st.launches += s->launched;
    return s->launched;
}

// True when some group has left without publishing `seq` and the whole grid is gone (the stream is
// idle): the request can only be served by a new launch.
bool needs_relaunch(const Resident* s, uint32_t seq) {
    bool gone = false;
    for (uint32_t g = 0; g < kSvcGroups; ++g)
        gone |= __atomic_load_n(&s->ctl->alive[g], __ATOMIC_ACQUIRE) == 0 &&
                __atomic_load_n(&s->ctl->done_seq[g], __ATOMIC_ACQUIRE) != seq;
    return gone && hipStreamQuery(s->stream) == hipSuccess;
}
}  // namespace

int resident_create(int device, const uint8_t* d_data, const uint32_t* d_off, const uint16_t* d_len, Resident** out) {
    *out = nullptr;
    if (device < 0 || device >= 64) return HALO_E_NODEV;
    auto* s = new (std::nothrow) Resident;
    if (!s) return HALO_E_NOMEM;
    s->device = device;
    s->d_data = d_data;
    s->d_off = d_off;
    s->d_len = d_len;
    void* cp = nullptr;
    bool ok = hipHostMalloc(&cp, sizeof(RingServiceCtl), hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess;
    s->ctl = static_cast<RingServiceCtl*>(cp);
    if (ok) {
        memset(cp, 0, sizeof(RingServiceCtl));
        void* dv = nullptr;
        ok = hipHostGetDevicePointer(&dv, cp, 0) == hipSuccess && dv;
        s->d_ctl = static_cast<RingServiceCtl*>(dv);
    }
    ok = ok && hipMalloc((void**)&s->d_quit, sizeof(uint32_t)) == hipSuccess;
    ok = ok && hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        resident_destroy(s);
        return HALO_E_NOMEM;
    }
    std::lock_guard<std::mutex> g(g_live_mu);
    g_live.push_back(s);
    *out = s;
    return HALO_OK;
}

void resident_destroy(Resident* s) {
    if (!s) return;
    ParkUsed park(s->device);  // hipFree / hipHostFree below wait for kernels on every device
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        g_live.erase(std::remove(g_live.begin(), g_live.end(), s), g_live.end());
    }
    {
        std::lock_guard<std::mutex> lk(s->mu);
        if (s->ctl) stop_locked(s);
    }
    if (s->stream) (void)hipStreamDestroy(s->stream);
    if (s->d_quit) (void)hipFree(s->d_quit);
    if (s->ctl) (void)hipHostFree(s->ctl);
    delete s;
}

void resident_set_timeout(Resident* s, uint64_t us) {
    std::lock_guard<std::mutex> lk(s->mu);
    s->timeout_us = us ? us : 2000000;
}

void resident_set_arrays(Resident* s, const uint8_t* d_data, const uint32_t* d_off, const uint16_t* d_len) {
    std::lock_guard<std::mutex> lk(s->mu);
    stop_locked(s);  // already parked by the caller: a no-op unless it was relaunched since
    s->d_data = d_data;
    s->d_off = d_off;
    s->d_len = d_len;
}

ResidentStats resident_stats(const Resident* s) {
    std::lock_guard<std::mutex> lk(const_cast<Resident*>(s)->mu);
    return s->st;
}

// The request fields and their check first, then req_seq with release; spin until every group's
// done_seq slot holds it. A consumer that went idle (or exited between its last check and the
// request) is relaunched: its alive slots and the stream say whether the grid is gone. Every wait
// is bounded, and a request that times out is retired before the error is returned.
int resident_request(Resident* s, uint32_t n, uint32_t flags, const halo_rx_netif_t* netif, halo_rx_result_t* dout,
                     uint32_t uni_off, uint32_t uni_stride, uint32_t uni_len) {
    std::lock_guard<std::mutex> lk(s->mu);
    if (parked(s->device)) {
        ++s->st.parked;
        return kResidentParked;
    }
    RingServiceCtl* c = s->ctl;
    const uint32_t seq = s->seq + 1;
    const uint64_t out = reinterpret_cast<uint64_t>(dout);
    c->n = n;
    c->flags = flags;
    c->mac_lo = (uint32_t)netif->mac[0] | ((uint32_t)netif->mac[1] << 8) | ((uint32_t)netif->mac[2] << 16) |
                ((uint32_t)netif->mac[3] << 24);
    c->mac_hi = (uint32_t)netif->mac[4] | ((uint32_t)netif->mac[5] << 8);
    c->own_ip = netif->ip;
    c->out_lo = (uint32_t)out;
    c->out_hi = (uint32_t)(out >> 32);
    c->uni_off = uni_off;
    c->uni_stride = uni_stride;
    c->uni_len = uni_len;
    __atomic_store_n(&c->check, svc_check(seq, n, flags, c->mac_lo, c->mac_hi, c->own_ip, c->out_lo, c->out_hi,
                                          uni_off, uni_stride, uni_len),
                     __ATOMIC_RELEASE);
    // idle past half the timeout: the kernel may have exited; ask the stream (cheap, rare)
    if (!s->launched ||
        (clk::now() - s->last_done > std::chrono::microseconds(kSvcIdleUs / 2) && hipStreamQuery(s->stream) == hipSuccess)) {
        if (!launch_locked(s, s->seq)) return HALO_E_HIP;
    }
    s->seq = seq;
    __atomic_store_n(&c->req_seq, seq, __ATOMIC_RELEASE);
    const auto t0 = clk::now();
    auto t_check = t0;
    for (uint32_t k = 1;; ++k) {
        uint32_t done = 0;
        for (uint32_t g = 0; g < kSvcGroups; ++g) done += __atomic_load_n(&c->done_seq[g], __ATOMIC_ACQUIRE) == seq;
        if (done == kSvcGroups) break;
        __builtin_ia32_pause();
        if ((k & 63u) == 0) {
            const auto now = clk::now();
            if (now - t_check > std::chrono::microseconds(20)) {
                t_check = now;
                // the grid ended before it saw this request (an idle exit racing it): start another
                if (needs_relaunch(s, seq) && !launch_locked(s, seq - 1)) return HALO_E_HIP;
            }
            if (now - t0 > std::chrono::microseconds(s->timeout_us)) {
                // retire the request: once the kernel has ended nothing more is written to dout
                stop_locked(s);
                return HALO_E_HIP;
            }
        }
    }
    s->last_done = clk::now();
    ++s->st.requests;
    uint64_t seen = c->t_seen[0], fin = c->t_done[0];
    for (uint32_t g = 1; g < kSvcGroups; ++g) {
        seen = std::min(seen, c->t_seen[g]);
        fin = std::max(fin, c->t_done[g]);
    }
    s->st.gpu_ns += (fin - seen) * 10u;  // 100 MHz ticks: first group in to last group out
    return HALO_OK;
}

ParkResidents::ParkResidents(int device) : device_(device) {
    if (device < 0 || device >= 64) return;
    g_parked[device].fetch_add(1, std::memory_order_acq_rel);  // before any consumer is stopped
    std::lock_guard<std::mutex> g(g_live_mu);
    for (Resident* s : g_live) {
        if (s->device != device) continue;
        std::lock_guard<std::mutex> lk(s->mu);  // waits for a request in flight to finish
        stop_locked(s);
    }
}

ParkResidents::~ParkResidents() {
    if (device_ >= 0 && device_ < 64) g_parked[device_].fetch_sub(1, std::memory_order_acq_rel);
}

int current_device() {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return cur;
}

int drain_device(int device) {
    if (device < 0 || device >= 64) return HALO_E_NODEV;
    ParkResidents park(device);
    const int cur = current_device();
    int rc = HALO_OK;
    if (hipSetDevice(device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = HALO_E_HIP;
    if (cur != device) (void)hipSetDevice(cur);
    return rc;
}

}  // namespace halo
