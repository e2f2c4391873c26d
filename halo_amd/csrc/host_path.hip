// host_path.hip — device selection, the host-memory batch path (SURVEY.md §8f row f1:
// drain host frames into pinned chunks, double-buffered H2D -> kernel -> D2H) and the
// reference engine's per-frame decision over the kernel's records.
#include <hip/hip_runtime.h>
#include <string.h>

#include <unistd.h>

#include <atomic>
#include <algorithm>
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
int sync_used_devices() {
    const uint64_t used = g_devices_used.load(std::memory_order_relaxed);
    if (!used) return HALO_OK;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return HALO_E_HIP;
    int rc = HALO_OK;
    for (int d = 0; d < 64; ++d)
        if ((used >> d) & 1)
            if (hipSetDevice(d) != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = HALO_E_HIP;
    (void)hipSetDevice(cur);
    return rc;
}

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
    return halo::check_device();
}

// ---- host-memory batch path ---------------------------------------------------------------
struct halo_rx_host_ctx {
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
void free_ctx(halo_rx_host_ctx* c) {
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
    for (auto& s : ctx->slot)
        if (s.stream) (void)hipStreamSynchronize(s.stream);
    free_ctx(ctx);
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_parse_batch_host(halo_rx_host_ctx_t* ctx, const uint8_t* bytes,
                                                 const uint64_t* offsets, const uint16_t* lens, uint32_t n,
                                                 uint32_t flags, const halo_rx_netif_t* netif,
                                                 halo_rx_result_t* out, uint32_t* status_hist) {
    if (!ctx || !netif) return HALO_E_INVAL;
    if (n == 0) return HALO_OK;
    if (!bytes || !offsets || !lens || !out) return HALO_E_INVAL;
    if (flags & HALO_RX_RECORD_COMPACT) return HALO_E_INVAL;  // host path returns full records
    if (hipSetDevice(ctx->device) != hipSuccess) return HALO_E_NODEV;
    const uint32_t cap = (flags & HALO_RX_L3_START) ? ((flags & HALO_RX_JUMBO_EXT) ? halo::kIpMaxJumbo : halo::kIpMax)
                                                    : ((flags & HALO_RX_JUMBO_EXT) ? halo::kEthMaxJumbo : halo::kEthMax);
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
