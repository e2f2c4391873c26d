// host_path.hip — device selection, the host-memory batch path (SURVEY.md §8f row f1:
// drain host frames into pinned chunks, double-buffered H2D -> kernel -> D2H) and the
// reference engine's per-frame decision over the kernel's records.
#include <hip/hip_runtime.h>
#include <string.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <new>
#include <utility>
#include <vector>

#include "halo_common.h"

namespace halo {

namespace {
std::atomic<uint64_t> g_devices_used{0};  // bit d: this library has launched work on device d
}

int check_device() {
    static std::atomic<int> verdict[64];  // 0 = unknown, 1 = gfx950, <0 = HALO_E_*
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return HALO_E_NODEV;
    if (dev < 64) {
        const int v = verdict[dev].load(std::memory_order_relaxed);
        if (v == 1) {
            g_devices_used.fetch_or(1ull << dev, std::memory_order_relaxed);
            return HALO_OK;
        }
        if (v < 0) return v;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return HALO_E_NODEV;
    const int v = strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : HALO_E_ARCH;
    if (dev < 64) verdict[dev].store(v, std::memory_order_relaxed);
    if (v == 1 && dev < 64) g_devices_used.fetch_or(1ull << dev, std::memory_order_relaxed);
    return v == 1 ? HALO_OK : v;
}

// ---- host registrations (the interval bookkeeping is RegMap, host_logic.cc) ------------------
namespace {
// Waits for all work this library queued on any device: a DMA or kernel still reading or
// writing the range must finish before its pages are unpinned.
// Resident consumers are stopped first (ParkResidents, held by the caller): their kernels would
// otherwise keep the device busy until they idle out, or forever while another thread keeps polling
// (ADVICE r3).
int sync_used_devices() {
    const uint64_t used = g_devices_used.load(std::memory_order_relaxed);
    int rc = HALO_OK;
    for (int d = 0; d < 64; ++d)
        if ((used >> d) & 1)
            if (drain_device(d) != HALO_OK) rc = HALO_E_HIP;
    return rc;
}


}  // namespace

ParkUsed::ParkUsed(int also) {
    uint64_t used = g_devices_used.load(std::memory_order_relaxed);
    if (also >= 0 && also < 64) used |= 1ull << also;
    for (int d = 0; d < 64; ++d)
        if ((used >> d) & 1) parks.emplace_back(new ParkResidents(d));
}

namespace {
// True while the runtime still maps host address p for the device.
bool runtime_maps(void* p) {
    void* d = nullptr;
    const bool mapped = hipHostGetDevicePointer(&d, p, 0) == hipSuccess && d;
    (void)hipGetLastError();  // a failed query must not surface at a later launch check
    return mapped;
}
}  // namespace

uint64_t host_page_size() {
    static const uint64_t page = [] {
        const long p = sysconf(_SC_PAGESIZE);
        return p > 0 ? (uint64_t)p : 4096ull;
    }();
    return page;
}

// The range is reserved first (refused if it shares a page with any registration), registered
// with the runtime with no lock held, then published.
int host_reg_add(void* base, uint64_t bytes, HostRegKind kind) {
    const uintptr_t b = reinterpret_cast<uintptr_t>(base);
    int rc = registry().reserve(b, bytes, host_page_size(), kind);
    if (rc) return rc;
    ParkUsed park;  // hipHostRegister may wait for the device
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        registry().cancel(b);
        return HALO_E_NODEV;
    }
    if (hipHostRegister(base, bytes, hipHostRegisterDefault) != hipSuccess) {
        (void)hipGetLastError();
        registry().cancel(b);
        return HALO_E_HIP;
    }
    void* dev = nullptr;
    if (hipHostGetDevicePointer(&dev, base, 0) != hipSuccess) {
        (void)hipGetLastError();
        dev = nullptr;  // no device view: the range is still usable as a DMA source
    }
    registry().commit(b, static_cast<uint8_t*>(dev));
    return HALO_OK;
}

bool host_reg_find(const void* p, uintptr_t* base, uint64_t* bytes, uint8_t** dev) {
    return registry().find(reinterpret_cast<uintptr_t>(p), base, bytes, dev);
}

void* host_reg_device_view(const void* p, uint64_t bytes) {
    return registry().view(reinterpret_cast<uintptr_t>(p), bytes);
}

// The entry is marked as being removed (lookups stop seeing it) and the device synchronisation and
// hipHostUnregister run with no lock held, so other threads' lookups do not wait on device work.
int host_reg_remove(void* base, HostRegKind kind) {
    const uintptr_t b = reinterpret_cast<uintptr_t>(base);
    if (!registry().begin_remove(b, kind)) return HALO_E_INVAL;  // not a live base of this kind
    ParkUsed park;                                                // through the unregistration
    int rc = sync_used_devices();                                 // the pages stay pinned on failure
    if (rc == HALO_OK && hipHostUnregister(base) != hipSuccess) {
        (void)hipGetLastError();
        rc = HALO_E_HIP;
    }
    if (rc == HALO_OK && runtime_maps(base)) rc = HALO_E_HIP;  // still mapped: the caller keeps the memory
    registry().end_remove(b, rc == HALO_OK);
    return rc;
}

}  // namespace halo

extern "C" HALO_API int halo_rx_init(int device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return HALO_E_NODEV;
    if (device < 0 || device >= count) return HALO_E_NODEV;
    if (hipSetDevice(device) != hipSuccess) return HALO_E_NODEV;
    const int rc = halo::check_device();
    if (rc) return rc;
    // the trees are only needed by histogram-on calls: a failure here (e.g. a global-mode capture on
    // another stream refusing the allocation) is left for such a call to report
    (void)halo::hist_trees(device, nullptr);
    (void)hipGetLastError();
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_device_synchronize(int device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return HALO_E_NODEV;
    return halo::drain_device(device);
}

extern "C" HALO_API int halo_rx_release(int device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return HALO_E_NODEV;
    halo::ParkResidents park(device);
    const int rc = halo::drain_device(device);
    if (rc) return rc;
    // the tree set itself stays (a captured graph holds its address); its keys are handed back, so
    // the queues of streams destroyed since can no longer exhaust them
    return halo::hist_trees_reset_keys(device);
}

extern "C" HALO_API int halo_rx_debug_hist_keys(int device, int op, uint32_t arg) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return HALO_E_NODEV;
    if (op < 0 || op > 3) return HALO_E_INVAL;
    if (op != 0) {  // writes: nothing of this library's may be running on the device
        halo::ParkResidents park(device);
        const int rc = halo::drain_device(device);
        if (rc) return rc;
        return halo::hist_keys_debug(device, op, arg);
    }
    return halo::hist_keys_debug(device, op, arg);
}

// ---- host-memory batch path ---------------------------------------------------------------
struct halo_rx_host_ctx {
    // halo_rx_host_ctx_set_resident: batches of up to max_frames frames / max_bytes bytes are packed
    // into pinned staging and served by a resident consumer (no launch, no stream synchronisation)
    struct Resident {
        halo::Resident* svc = nullptr;
        uint32_t max_frames = 0;
        uint64_t max_bytes = 0;
        uint8_t* h_bytes = nullptr;  // pinned; d_* are the device's addresses of the same memory
        uint8_t* d_bytes = nullptr;
        uint32_t* h_off = nullptr;
        uint32_t* d_off = nullptr;
        uint16_t* h_len = nullptr;
        uint16_t* d_len = nullptr;
        halo_rx_result_t* h_res = nullptr;
        halo_rx_result_t* d_res = nullptr;
    } res;
    halo_rx_host_stats_t stats{};
    int device;
    uint32_t chunk_frames;
    uint32_t zc_frames;  // chunk of the zero-copy path with GPU-converted metadata (no host staging)
    uint64_t chunk_bytes;
    bool zero_copy = true;  // registered frames are parsed where they lie (no H2D of frame bytes)
    struct Slot {
        hipStream_t stream = nullptr;
        uint8_t* h_bytes = nullptr;   // pinned staging
        uint32_t* h_off = nullptr;
        uint16_t* h_len = nullptr;
        uint8_t* d_bytes = nullptr;
        uint32_t* d_off = nullptr;
        uint16_t* d_len = nullptr;
        halo_rx_result_t* d_res = nullptr;
        uint32_t* d_hist = nullptr;
        uint32_t* d_hist_try = nullptr;  // zero-copy chunks with GPU-converted metadata count here first
        uint32_t* d_flag = nullptr;      // set by zc_meta_kernel when a frame lies outside the registration
        uint32_t* h_flag = nullptr;      // pinned copy of d_flag
        bool zc_meta = false;            // the chunk in flight converted its metadata on the GPU
        // chunk currently in flight in this slot
        bool busy = false;
        uint64_t first = 0;
        uint32_t count = 0;
    } slot[2];
};

namespace {
void free_resident(halo_rx_host_ctx::Resident& r) {
    halo::resident_destroy(r.svc);  // stops the consumer and waits for its kernel to end
    if (r.h_bytes) (void)hipHostFree(r.h_bytes);
    if (r.h_off) (void)hipHostFree(r.h_off);
    if (r.h_len) (void)hipHostFree(r.h_len);
    if (r.h_res) (void)hipHostFree(r.h_res);
    r = halo_rx_host_ctx::Resident{};
}

template <typename T>
bool pinned_mapped(T** h, T** d, uint64_t bytes) {
    void* p = nullptr;
    void* dv = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocMapped) != hipSuccess) return false;
    *h = static_cast<T*>(p);
    if (hipHostGetDevicePointer(&dv, p, 0) != hipSuccess || !dv) {
        (void)hipGetLastError();
        return false;
    }
    *d = static_cast<T*>(dv);
    return true;
}

void free_ctx(halo_rx_host_ctx* c) {
    free_resident(c->res);
    for (auto& s : c->slot) {
        if (s.stream) (void)hipStreamDestroy(s.stream);
        if (s.h_bytes) (void)hipHostFree(s.h_bytes);
        if (s.h_off) (void)hipHostFree(s.h_off);
        if (s.h_len) (void)hipHostFree(s.h_len);
        if (s.d_bytes) (void)hipFree(s.d_bytes);
        if (s.d_off) (void)hipFree(s.d_off);
        if (s.d_len) (void)hipFree(s.d_len);
        if (s.d_res) (void)hipFree(s.d_res);
        if (s.d_hist) (void)hipFree(s.d_hist);
        if (s.d_hist_try) (void)hipFree(s.d_hist_try);
        if (s.d_flag) (void)hipFree(s.d_flag);
        if (s.h_flag) (void)hipHostFree(s.h_flag);
    }
    delete c;
}

// Zero-copy metadata: the caller's own u64 byte offsets and u16 lengths (registered host memory,
// read over PCIe) become the kernel's u32 dword offsets into the frames' registration. A frame not
// wholly inside that registration, or not 4-byte aligned in it, gets length 0 (never read) and
// raises the flag: the host then re-parses that chunk on the DMA path (and its status counts
// never reach the histogram: zc_hist_commit drops them).
__global__ void __launch_bounds__(256) zc_meta_kernel(const uint64_t* __restrict__ offs,
                                                      const uint16_t* __restrict__ lens, uint32_t n,
                                                      uint64_t delta, uint64_t reg_bytes, uint32_t* d_off,
                                                      uint16_t* d_len, uint32_t* flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t rel = offs[i] + delta;  // byte offset in the registration (mod 2^64)
    const uint32_t L = lens[i];
    const bool ok = rel < reg_bytes && L <= reg_bytes - rel && (rel & 3u) == 0;
    d_off[i] = ok ? (uint32_t)(rel >> 2) : 0u;
    d_len[i] = ok ? (uint16_t)L : (uint16_t)0;
    if (!ok) atomicOr(flag, 1u);
}

// Adds the chunk's status counts to the slot's histogram unless the chunk is to be re-parsed.
__global__ void zc_hist_commit(const uint32_t* flag, uint32_t* try_hist, uint32_t* hist) {
    const uint32_t t = threadIdx.x;
    if (t >= HALO_RX_STATUS_COUNT) return;
    if (*flag == 0) hist[t] += try_hist[t];
    try_hist[t] = 0;
}
}  // namespace

extern "C" HALO_API int halo_rx_host_ctx_create(int device, uint32_t chunk_frames, uint64_t chunk_bytes,
                                                halo_rx_host_ctx_t** out) {
    if (!out) return HALO_E_INVAL;
    *out = nullptr;
    int rc = halo_rx_init(device);
    if (rc) return rc;
    if (chunk_frames == 0) chunk_frames = 1u << 18;
    if (chunk_bytes == 0) chunk_bytes = 64ull << 20;
    if (chunk_bytes < 65536) return HALO_E_INVAL;
    auto* c = new (std::nothrow) halo_rx_host_ctx;
    if (!c) return HALO_E_NOMEM;
    halo::ParkUsed park(device);  // pinned allocations (and a failed create's frees: hipHostFree waits on every device)
    c->device = device;
    c->chunk_frames = chunk_frames;
    // zero-copy chunks with GPU-converted metadata stage nothing on the host, so they can be
    // larger: fewer chunk boundaries (1M x 64 B: 1.87 ms in 256k-frame chunks, 1.60 ms in one;
    // profiles/r02/r2o/host_zc_sweep.log); the device metadata and record buffers are sized for them
    c->zc_frames = (uint32_t)std::min<uint64_t>(4ull * chunk_frames, 0xFFFFFFFFull);
    c->chunk_bytes = chunk_bytes;
    bool ok = true;
    for (auto& s : c->slot) {
        ok = ok && hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) == hipSuccess;
        ok = ok && hipHostMalloc((void**)&s.h_bytes, chunk_bytes, hipHostMallocDefault) == hipSuccess;
        ok = ok && hipHostMalloc((void**)&s.h_off, 4ull * chunk_frames, hipHostMallocDefault) == hipSuccess;
        ok = ok && hipHostMalloc((void**)&s.h_len, 2ull * chunk_frames, hipHostMallocDefault) == hipSuccess;
        ok = ok && hipMalloc((void**)&s.d_bytes, chunk_bytes) == hipSuccess;
        ok = ok && hipMalloc((void**)&s.d_off, 4ull * c->zc_frames) == hipSuccess;
        ok = ok && hipMalloc((void**)&s.d_len, 2ull * c->zc_frames) == hipSuccess;
        ok = ok && hipMalloc((void**)&s.d_res, sizeof(halo_rx_result_t) * c->zc_frames) == hipSuccess;
        ok = ok && hipMalloc((void**)&s.d_hist, 4 * HALO_RX_STATUS_COUNT) == hipSuccess;
        ok = ok && hipMemsetAsync(s.d_hist, 0, 4 * HALO_RX_STATUS_COUNT, s.stream) == hipSuccess;  // before its parses
        ok = ok && hipMalloc((void**)&s.d_hist_try, 4 * HALO_RX_STATUS_COUNT) == hipSuccess;
        ok = ok && hipMemsetAsync(s.d_hist_try, 0, 4 * HALO_RX_STATUS_COUNT, s.stream) == hipSuccess;
        ok = ok && hipMalloc((void**)&s.d_flag, 4) == hipSuccess;
        ok = ok && hipMemsetAsync(s.d_flag, 0, 4, s.stream) == hipSuccess;
        ok = ok && hipHostMalloc((void**)&s.h_flag, 4, hipHostMallocDefault) == hipSuccess;
        if (ok) *s.h_flag = 0;
    }
    if (!ok) {
        free_ctx(c);
        return HALO_E_NOMEM;
    }
    *out = c;
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_host_ctx_destroy(halo_rx_host_ctx_t* ctx) {
    if (!ctx) return HALO_E_INVAL;
    (void)hipSetDevice(ctx->device);
    halo::ParkUsed park(ctx->device);  // hipFree waits for the device's kernels, hipHostFree for every device's
    for (auto& s : ctx->slot)
        if (s.stream) (void)hipStreamSynchronize(s.stream);
    free_ctx(ctx);
    return HALO_OK;
}

namespace {
using clk = std::chrono::steady_clock;
uint64_t ns_between(clk::time_point a, clk::time_point b) {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
}

// The resident path of halo_rx_parse_batch_host: the frames are packed into the context's pinned
// staging (4-byte aligned starts; frames over the length cap are not copied, their verdict needs no
// byte), and one request to the resident consumer parses them there over PCIe and writes the records
// into `out` directly when it is registered, else into pinned staging that is copied out. A batch
// whose frames all have one length travels as the uniform layout (frame i at i * stride: the consumer
// reads no offset / length arrays). Returns 1 when the frames do not fit the staging area (the caller
// takes the chunked path). With the consumer parked by a device drain, the same staging is parsed by
// one launch instead.
int resident_batch(halo_rx_host_ctx* c, const uint8_t* bytes, const uint64_t* offsets, const uint16_t* lens,
                   uint32_t n, uint32_t flags, uint32_t cap, const halo_rx_netif_t* netif, halo_rx_result_t* out,
                   uint32_t* status_hist) {
    auto& R = c->res;
    const auto t0 = clk::now();
    uint64_t used = 0;
    // checked before any byte is copied: a batch that does not fit is staged once, by the chunked path
    if (halo::pack_need(lens, n, cap) > R.max_bytes) return 1;
    if (halo::pack_chunk(bytes, offsets, lens, n, 0, n, R.max_bytes, cap, R.h_bytes, R.h_off, R.h_len, &used) != n)
        return 1;
    uint32_t ulen = lens[0], ustride = 0;
    for (uint32_t i = 1; i < n && ulen; ++i) ulen = lens[i] == ulen ? ulen : 0u;
    if (ulen > cap || (flags & HALO_RX_L3_START)) ulen = 0;  // the strided layout has no L3 form
    if (ulen) ustride = (ulen + 3u) >> 2;                      // pack_chunk laid them i * stride apart
    const uint64_t rb = sizeof(halo_rx_result_t) * (uint64_t)n;
    auto* dout = static_cast<halo_rx_result_t*>(halo::host_reg_device_view(out, rb));
    if (reinterpret_cast<uintptr_t>(dout) & 15u) dout = nullptr;
    halo_rx_result_t* dst = dout ? dout : R.d_res;
    const auto t1 = clk::now();
    int rc = halo::resident_request(R.svc, n, flags & ~HALO_RX_VARIANT_MASK, netif, dst, 0u, ustride, ulen);
    if (rc == halo::kResidentParked) {
        hipStream_t st = c->slot[0].stream;  // idle between calls: the API is synchronous
        rc = ulen ? halo_rx_parse_strided_device(R.d_bytes, 4ull * ustride, nullptr, ulen, n, flags, netif, dst,
                                                 nullptr, st)
                  : halo_rx_parse_batch_device(R.d_bytes, R.d_off, R.d_len, n, flags, netif, 0, dst, nullptr, st);
        if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = HALO_E_HIP;
        ++c->stats.resident_parked;
    }
    const auto t2 = clk::now();
    c->stats.pack_ns += ns_between(t0, t1);
    c->stats.wait_ns += ns_between(t1, t2);
    if (rc) return rc;
    ++c->stats.resident_calls;
    if (!dout) memcpy(out, R.h_res, rb);
    if (status_hist)
        for (uint32_t i = 0; i < n; ++i) ++status_hist[out[i].status];  // the statuses the kernel wrote
    return HALO_OK;
}
}  // namespace

extern "C" HALO_API int halo_rx_parse_batch_host(halo_rx_host_ctx_t* ctx, const uint8_t* bytes,
                                                 const uint64_t* offsets, const uint16_t* lens, uint32_t n,
                                                 uint32_t flags, const halo_rx_netif_t* netif,
                                                 halo_rx_result_t* out, uint32_t* status_hist) {
    if (!ctx || !netif) return HALO_E_INVAL;
    if (n == 0) return HALO_OK;
    if (!bytes || !offsets || !lens || !out) return HALO_E_INVAL;
    if (flags & HALO_RX_RECORD_COMPACT) return HALO_E_INVAL;  // host path returns full records
    if (flags & ~(HALO_RX_CSUM_ENABLE | HALO_RX_JUMBO_EXT | HALO_RX_UNIFORM_LEN | HALO_RX_L3_START |
                  HALO_RX_VARIANT_MASK))
        return HALO_E_INVAL;
    if (hipSetDevice(ctx->device) != hipSuccess) return HALO_E_NODEV;
    const uint32_t cap = (flags & HALO_RX_L3_START) ? ((flags & HALO_RX_JUMBO_EXT) ? halo::kIpMaxJumbo : halo::kIpMax)
                                                    : ((flags & HALO_RX_JUMBO_EXT) ? halo::kEthMaxJumbo : halo::kEthMax);
    ++ctx->stats.calls;
    ctx->stats.frames += n;
    if (ctx->res.svc && n <= ctx->res.max_frames) {
        const int r = resident_batch(ctx, bytes, offsets, lens, n, flags, cap, netif, out, status_hist);
        if (r <= 0) return r;  // 1: larger than the staging area -> the chunked path below
    }
    int rc = HALO_OK;
    std::vector<std::pair<uint64_t, uint32_t>> redo;  // zero-copy chunks to re-parse on the DMA path
    auto drain = [&](halo_rx_host_ctx::Slot& s) -> int {
        if (!s.busy) return HALO_OK;
        s.busy = false;
        if (hipStreamSynchronize(s.stream) != hipSuccess) return HALO_E_HIP;
        if (s.zc_meta && *s.h_flag) redo.emplace_back(s.first, s.count);
        s.zc_meta = false;
        *s.h_flag = 0;
        return HALO_OK;
    };
    uint64_t next = 0;
    uint32_t k = 0;
    while (next < n && rc == HALO_OK) {
        auto& s = ctx->slot[k & 1];
        if ((rc = drain(s))) break;
        // Zero-copy mode: frames 4-byte aligned relative to each other inside one live
        // registration (a registered ring segment or packed batch) are read by the kernel in
        // place over PCIe, and the records are written straight into `out` when it is registered
        // too: no staging, no DMA of frame bytes (tools/exp/zc_probe.py: the kernel reads host
        // memory at the link rate, where the DMA-then-parse pipeline lost a third of it).
        if (ctx->zero_copy) {
            uint32_t cnt = (uint32_t)((n - next) < ctx->zc_frames ? (n - next) : ctx->zc_frames);
            const uint64_t* o = offsets + next;
            const uint16_t* l = lens + next;
            // (a) offsets and lengths registered too: the GPU converts them (no host pass over the
            // metadata, which cost ~1.4 ms per 1M frames on the host: profiles/r02/host_zc_sweep.log)
            const auto* d_o = static_cast<const uint64_t*>(halo::host_reg_device_view(o, 8ull * cnt));
            const auto* d_l = d_o ? static_cast<const uint16_t*>(halo::host_reg_device_view(l, 2ull * cnt)) : nullptr;
            uintptr_t rb = 0;
            uint64_t rbytes = 0;
            uint8_t* rdev = nullptr;
            if (d_l && !(reinterpret_cast<uintptr_t>(d_o) & 7u) && !(reinterpret_cast<uintptr_t>(d_l) & 1u) &&
                halo::host_reg_find(bytes + o[0], &rb, &rbytes, &rdev) && rdev && rbytes <= (16ull << 30) &&
                !(reinterpret_cast<uintptr_t>(rdev) & 3u)) {
                const uint64_t delta = reinterpret_cast<uintptr_t>(bytes) - rb;  // frame at rdev + o + delta
                auto* out_view = static_cast<halo_rx_result_t*>(
                    halo::host_reg_device_view(out + next, sizeof(halo_rx_result_t) * cnt));
                if (reinterpret_cast<uintptr_t>(out_view) & 15u) out_view = nullptr;
                hipLaunchKernelGGL(zc_meta_kernel, dim3((cnt + 255) / 256), dim3(256), 0, s.stream, d_o, d_l, cnt,
                                   delta, rbytes, s.d_off, s.d_len, s.d_flag);
                if (hipGetLastError() != hipSuccess) { rc = HALO_E_HIP; break; }
                rc = halo_rx_parse_batch_device(rdev, s.d_off, s.d_len, cnt, flags, netif, 0,
                                                out_view ? out_view : s.d_res,
                                                status_hist ? s.d_hist_try : nullptr, s.stream);
                if (rc) break;
                if (status_hist) {
                    hipLaunchKernelGGL(zc_hist_commit, dim3(1), dim3(64), 0, s.stream, s.d_flag, s.d_hist_try, s.d_hist);
                    if (hipGetLastError() != hipSuccess) { rc = HALO_E_HIP; break; }
                }
                hipError_t e = hipSuccess;
                if (!out_view)
                    e = hipMemcpyAsync(out + next, s.d_res, sizeof(halo_rx_result_t) * cnt, hipMemcpyDeviceToHost,
                                       s.stream);
                if (e == hipSuccess) e = hipMemcpyAsync(s.h_flag, s.d_flag, 4, hipMemcpyDeviceToHost, s.stream);
                if (e == hipSuccess) e = hipMemsetAsync(s.d_flag, 0, 4, s.stream);
                if (e != hipSuccess) { rc = HALO_E_HIP; break; }
                s.zc_meta = true;
                s.busy = true;
                s.first = next;
                s.count = cnt;
                next += cnt;
                ++k;
                continue;
            }
            // (b) metadata converted by the host, into the slot's pinned staging
            if (cnt > ctx->chunk_frames) cnt = ctx->chunk_frames;
            uint64_t lo = 0, hi = 0;
            const bool rel_aligned = halo::span_aligned(o, l, cnt, &lo, &hi);
            const uint64_t span = hi > lo ? hi - lo : 1;
            const uint8_t* view = !rel_aligned || span > (16ull << 30)
                                      ? nullptr
                                      : static_cast<const uint8_t*>(halo::host_reg_device_view(bytes + lo, span));
            if (view && !(reinterpret_cast<uintptr_t>(view) & 3u)) {
                for (uint32_t j = 0; j < cnt; ++j) {
                    s.h_off[j] = (uint32_t)((o[j] - lo) >> 2);
                    s.h_len[j] = l[j];
                }
                auto* out_view = static_cast<halo_rx_result_t*>(
                    halo::host_reg_device_view(out + next, sizeof(halo_rx_result_t) * cnt));
                if (reinterpret_cast<uintptr_t>(out_view) & 15u) out_view = nullptr;
                hipError_t e = hipMemcpyAsync(s.d_off, s.h_off, 4ull * cnt, hipMemcpyHostToDevice, s.stream);
                if (e == hipSuccess) e = hipMemcpyAsync(s.d_len, s.h_len, 2ull * cnt, hipMemcpyHostToDevice, s.stream);
                if (e != hipSuccess) { rc = HALO_E_HIP; break; }
                rc = halo_rx_parse_batch_device(view, s.d_off, s.d_len, cnt, flags, netif, 0,
                                                out_view ? out_view : s.d_res, status_hist ? s.d_hist : nullptr,
                                                s.stream);
                if (rc) break;
                if (!out_view && hipMemcpyAsync(out + next, s.d_res, sizeof(halo_rx_result_t) * cnt,
                                                hipMemcpyDeviceToHost, s.stream) != hipSuccess) {
                    rc = HALO_E_HIP;
                    break;
                }
                s.busy = true;
                s.first = next;
                s.count = cnt;
                next += cnt;
                ++k;
                continue;
            }
        }
        // Direct mode: frames in order, 4-byte aligned relative to the first, spanning at most
        // chunk_bytes (a drained ring segment, or a packed batch): one DMA of the caller's span
        // (pinned if registered with halo_rx_host_register), no CPU copy of frame bytes.
        uint64_t used = 0, lo = 0, hi = 0;
        const uint8_t* src = s.h_bytes;
        uint32_t cnt = halo::plan_direct(offsets, lens, n, next, ctx->chunk_frames, ctx->chunk_bytes, s.h_off, s.h_len,
                                         &lo, &hi);
        if (cnt) {
            used = hi - lo;
            src = bytes + lo;
        } else {
            // Pack mode: copy frames [next, ...) into the pinned slot, 4-byte aligned (ring-record style)
            cnt = halo::pack_chunk(bytes, offsets, lens, n, next, ctx->chunk_frames, ctx->chunk_bytes, cap, s.h_bytes,
                                   s.h_off, s.h_len, &used);
        }
        hipError_t e = hipSuccess;
        if (used) e = hipMemcpyAsync(s.d_bytes, src, used, hipMemcpyHostToDevice, s.stream);
        if (e == hipSuccess) e = hipMemcpyAsync(s.d_off, s.h_off, 4ull * cnt, hipMemcpyHostToDevice, s.stream);
        if (e == hipSuccess) e = hipMemcpyAsync(s.d_len, s.h_len, 2ull * cnt, hipMemcpyHostToDevice, s.stream);
        if (e != hipSuccess) { rc = HALO_E_HIP; break; }
        rc = halo_rx_parse_batch_device(s.d_bytes, s.d_off, s.d_len, cnt, flags, netif, 0, s.d_res,
                                        status_hist ? s.d_hist : nullptr, s.stream);
        if (rc) break;
        // records go straight to the caller's array (full rate when it is pinned/registered)
        if (hipMemcpyAsync(out + next, s.d_res, sizeof(halo_rx_result_t) * cnt, hipMemcpyDeviceToHost, s.stream) !=
            hipSuccess) { rc = HALO_E_HIP; break; }
        s.busy = true;
        s.first = next;
        s.count = cnt;
        next += cnt;
        ++k;
    }
    for (auto& s : ctx->slot) {
        int r2 = drain(s);
        if (!rc) rc = r2;
    }
    if (rc == HALO_OK && status_hist) {
        for (auto& s : ctx->slot) {
            uint32_t h[HALO_RX_STATUS_COUNT];
            // on the slot's own (non-blocking) stream: a null-stream hipMemset is not ordered
            // before the next call's launches there, and could zero counts they already added
            if (hipMemcpyAsync(h, s.d_hist, sizeof h, hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
                hipMemsetAsync(s.d_hist, 0, sizeof h, s.stream) != hipSuccess ||
                hipStreamSynchronize(s.stream) != hipSuccess)
                return HALO_E_HIP;
            for (int j = 0; j < HALO_RX_STATUS_COUNT; ++j) status_hist[j] += h[j];
        }
    }
    if (rc == HALO_OK && !redo.empty()) {  // frames outside the registration: those chunks again, by DMA
        ctx->zero_copy = false;
        for (const auto& r : redo) {
            rc = halo_rx_parse_batch_host(ctx, bytes, offsets + r.first, lens + r.first, r.second, flags, netif,
                                          out + r.first, status_hist);
            if (rc) break;
        }
        ctx->zero_copy = true;
    }
    return rc;
}

extern "C" HALO_API int halo_rx_host_ctx_set_resident(halo_rx_host_ctx_t* ctx, uint32_t max_frames,
                                                      uint64_t max_bytes) {
    if (!ctx) return HALO_E_INVAL;
    if (max_frames > halo::kSvcMaxFrames || max_bytes > (64ull << 20)) return HALO_E_INVAL;
    if (hipSetDevice(ctx->device) != hipSuccess) return HALO_E_NODEV;
    halo::ParkUsed park(ctx->device);  // frees and pinned allocations below (hipHostFree: every device)
    free_resident(ctx->res);
    if (max_frames == 0) return HALO_OK;
    // default: room for max_frames full-MTU frames, so a PacketHandle batch of 1514 B frames is served
    if (max_bytes == 0) max_bytes = std::min<uint64_t>(1516ull * max_frames, 64ull << 20);
    max_bytes = (max_bytes + 3) & ~3ull;
    auto& R = ctx->res;
    bool ok = pinned_mapped(&R.h_bytes, &R.d_bytes, max_bytes + 64) &&  // + a dword tail any load may cover
              pinned_mapped(&R.h_off, &R.d_off, 4ull * max_frames) && pinned_mapped(&R.h_len, &R.d_len, 2ull * max_frames) &&
              pinned_mapped(&R.h_res, &R.d_res, sizeof(halo_rx_result_t) * (uint64_t)max_frames);
    ok = ok && halo::resident_create(ctx->device, R.d_bytes, R.d_off, R.d_len, &R.svc) == HALO_OK;
    if (!ok) {
        free_resident(R);
        return HALO_E_NOMEM;
    }
    memset(R.h_bytes, 0, max_bytes + 64);
    R.max_frames = max_frames;
    R.max_bytes = max_bytes;
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_host_ctx_set_service_timeout(halo_rx_host_ctx_t* ctx, uint64_t us) {
    if (!ctx || !ctx->res.svc) return HALO_E_INVAL;
    halo::resident_set_timeout(ctx->res.svc, us);
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_host_ctx_get_stats(const halo_rx_host_ctx_t* ctx, halo_rx_host_stats_t* out) {
    if (!ctx || !out) return HALO_E_INVAL;
    *out = ctx->stats;
    if (ctx->res.svc) {
        const halo::ResidentStats s = halo::resident_stats(ctx->res.svc);
        out->service_launches = s.launches;
        out->service_gpu_ns = s.gpu_ns;
    }
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_host_ctx_set_zero_copy(halo_rx_host_ctx_t* ctx, int enable) {
    if (!ctx) return HALO_E_INVAL;
    ctx->zero_copy = enable != 0;
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_host_register(const void* ptr, uint64_t bytes) {
    return halo::host_reg_add(const_cast<void*>(ptr), bytes, halo::kRegUser);
}

extern "C" HALO_API int halo_rx_host_unregister(const void* ptr) {
    return halo::host_reg_remove(const_cast<void*>(ptr), halo::kRegUser);
}

extern "C" HALO_API uint32_t halo_rx_host_registered_count(void) {
    return halo::registry().list(nullptr, nullptr, 0);
}

extern "C" HALO_API uint32_t halo_rx_host_registrations(void** bases, uint64_t* bytes, uint32_t cap) {
    return halo::registry().list(bases, bytes, cap);
}
