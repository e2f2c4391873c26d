// bench_loop.hip — native timed step loop for bench.py (measurement tooling, not the product).
//
// bench.py's Python loop cost several microseconds of host time per launch, comparable to a
// 25 us kernel. This loop issues the same C-ABI calls a compiled host (the Go reference's
// PacketHandle replacement) would: one halo_rx_parse_*_device call per step, back to back on
// one stream. One HIP event pair brackets the whole timed region on that stream: the average
// launch duration is its elapsed time / steps. (An event pair around every launch would add
// about 2.5 us to each launch on the GPU timeline: measured in tools/gap_probe.py.)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>

#include "halo_rx.h"

extern "C" __attribute__((visibility("default"))) int halo_bench_steps(
    int nbatch, const uint8_t* const* bytes, const uint32_t* const* offsets_dw, const uint16_t* const* lens,
    uint32_t n, uint64_t stride, uint32_t len, uint32_t flags, const halo_rx_netif_t* netif, uint32_t hint,
    halo_rx_result_t* out, int warmup, int steps, void* stream, float* region_ms, double* wall_s) {
    if (nbatch <= 0 || steps <= 0 || !region_ms || !wall_s) return HALO_E_INVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto launch = [&](int k) -> int {
        const int b = k % nbatch;
        if (offsets_dw)
            return halo_rx_parse_batch_device(bytes[b], offsets_dw[b], lens[b], n, flags, netif, hint, out, nullptr,
                                              stream);
        return halo_rx_parse_strided_device(bytes[b], stride, lens ? lens[b] : nullptr, len, n, flags, netif, out,
                                            nullptr, stream);
    };
    int rc = HALO_OK;
    for (int k = 0; k < warmup && rc == HALO_OK; ++k) rc = launch(k);
    if (rc) return rc;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return HALO_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return HALO_E_HIP;
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipEventRecord(e0, s);
    for (int k = 0; k < steps && rc == HALO_OK; ++k) rc = launch(k);
    (void)hipEventRecord(e1, s);
    if (hipStreamSynchronize(s) != hipSuccess && rc == HALO_OK) rc = HALO_E_HIP;
    const auto t1 = std::chrono::steady_clock::now();
    *wall_s = std::chrono::duration<double>(t1 - t0).count();
    *region_ms = -1.0f;
    (void)hipEventElapsedTime(region_ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

// The same loop for the forward / transmit rewrite (halo_tx_fixup_batch_device, §8f row f2).
extern "C" __attribute__((visibility("default"))) int halo_bench_tx_steps(
    int nbatch, uint8_t* const* bytes, const uint32_t* const* offsets_dw, const uint16_t* const* lens, uint32_t n,
    const halo_tx_op_t* ops, uint32_t flags, uint32_t hint, uint8_t* result, int warmup, int steps, void* stream,
    float* region_ms, double* wall_s) {
    if (nbatch <= 0 || steps <= 0 || !region_ms || !wall_s) return HALO_E_INVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto launch = [&](int k) -> int {
        const int b = k % nbatch;
        return halo_tx_fixup_batch_device(bytes[b], offsets_dw[b], lens[b], n, ops, flags, hint, result, stream);
    };
    int rc = HALO_OK;
    for (int k = 0; k < warmup && rc == HALO_OK; ++k) rc = launch(k);
    if (rc) return rc;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return HALO_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return HALO_E_HIP;
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipEventRecord(e0, s);
    for (int k = 0; k < steps && rc == HALO_OK; ++k) rc = launch(k);
    (void)hipEventRecord(e1, s);
    if (hipStreamSynchronize(s) != hipSuccess && rc == HALO_OK) rc = HALO_E_HIP;
    const auto t1 = std::chrono::steady_clock::now();
    *wall_s = std::chrono::duration<double>(t1 - t0).count();
    *region_ms = -1.0f;
    (void)hipEventElapsedTime(region_ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

// Generic timed loop over a launch callback (row f3 kernels: flow-key hashing, XXH3 batches).
template <typename F>
static int timed_loop(F launch, int warmup, int steps, hipStream_t s, float* region_ms, double* wall_s) {
    if (steps <= 0 || !region_ms || !wall_s) return HALO_E_INVAL;
    int rc = HALO_OK;
    for (int k = 0; k < warmup && rc == HALO_OK; ++k) rc = launch(k);
    if (rc) return rc;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return HALO_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return HALO_E_HIP;
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipEventRecord(e0, s);
    for (int k = 0; k < steps && rc == HALO_OK; ++k) rc = launch(k);
    (void)hipEventRecord(e1, s);
    if (hipStreamSynchronize(s) != hipSuccess && rc == HALO_OK) rc = HALO_E_HIP;
    const auto t1 = std::chrono::steady_clock::now();
    *wall_s = std::chrono::duration<double>(t1 - t0).count();
    *region_ms = -1.0f;
    (void)hipEventElapsedTime(region_ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

extern "C" __attribute__((visibility("default"))) int halo_bench_flow_steps(
    int nbatch, const halo_rx_result_t* const* recs, uint32_t n, uint32_t kind, uint32_t nat_type, uint64_t* hash,
    uint32_t buckets, uint32_t* bucket, int warmup, int steps, void* stream, float* region_ms, double* wall_s) {
    if (nbatch <= 0) return HALO_E_INVAL;
    auto launch = [&](int k) {
        return halo_flow_hash_device(recs[k % nbatch], n, kind, nat_type, hash, buckets, bucket, stream);
    };
    return timed_loop(launch, warmup, steps, static_cast<hipStream_t>(stream), region_ms, wall_s);
}

extern "C" __attribute__((visibility("default"))) int halo_bench_xxh3_steps(
    int nbatch, const uint8_t* const* bytes, const uint64_t* const* offsets, const uint32_t* const* lens, uint32_t n,
    uint64_t* hash, int warmup, int steps, void* stream, float* region_ms, double* wall_s) {
    if (nbatch <= 0) return HALO_E_INVAL;
    auto launch = [&](int k) {
        const int b = k % nbatch;
        return halo_xxh3_64_batch_device(bytes[b], offsets[b], lens[b], n, hash, stream);
    };
    return timed_loop(launch, warmup, steps, static_cast<hipStream_t>(stream), region_ms, wall_s);
}

extern "C" __attribute__((visibility("default"))) int halo_bench_route_steps(
    int nbatch, const halo_route_table_t* t, const uint32_t* const* ips, uint32_t n, uint32_t* out, int warmup,
    int steps, void* stream, float* region_ms, double* wall_s) {
    if (nbatch <= 0) return HALO_E_INVAL;
    auto launch = [&](int k) { return halo_route_lookup_device(t, ips[k % nbatch], n, out, stream); };
    return timed_loop(launch, warmup, steps, static_cast<hipStream_t>(stream), region_ms, wall_s);
}

// Row f1: the device-resident record walk of halo's packet ring (halo_rx_ring_scan_device).
extern "C" __attribute__((visibility("default"))) int halo_bench_ring_scan_steps(
    int nbatch, const uint8_t* const* spans, uint64_t used, uint64_t ring_size, uint32_t capacity, uint32_t* off,
    uint16_t* lens, halo_rx_ring_scan_t* info, void* ws, uint64_t ws_bytes, int warmup, int steps, void* stream,
    float* region_ms, double* wall_s) {
    if (nbatch <= 0) return HALO_E_INVAL;
    auto launch = [&](int k) {
        return halo_rx_ring_scan_device(spans[k % nbatch], used, ring_size, capacity, 0, off, lens, info, ws, ws_bytes,
                                        stream);
    };
    return timed_loop(launch, warmup, steps, static_cast<hipStream_t>(stream), region_ms, wall_s);
}

// Measured streaming-read ceiling (the roofline is reported against the HBM3E spec
// peak AND a read-only streaming kernel on the same box): every 16-byte chunk of `bytes` read once
// with fully coalesced loads, 8 in flight per lane, folded into one word per block so nothing is
// optimised away. Not part of the product library.
namespace {
// Each block streams whole 64 KB tiles (tile = blockIdx.x + k * gridDim.x): 16 loads of 16 bytes per
// thread per tile, issued 8 at a time, consecutive threads on consecutive chunks — DRAM pages are
// swept in order, as a group of lanes sweeps a long frame.
__global__ void __launch_bounds__(256) read_peak_kernel(const uint4* __restrict__ src, uint64_t n16,
                                                        uint32_t* __restrict__ sink) {
    constexpr uint32_t kTile16 = 4096;  // 64 KB
    uint32_t acc = 0;
    const uint64_t tiles = n16 / kTile16;
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const uint4* p = src + t * kTile16 + threadIdx.x;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = p[(h * 8 + u) * 256];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;  // practically never: keeps the loads live
}

// Size-matched speed-of-light probe: block t reads 16 KB tile t of `src` (four 16-byte loads per
// thread in flight) and writes its share of `dst` with coalesced 16-byte stores — the rx kernel's
// bytes (frames + metadata in, records out) with perfect access patterns and no work.
__global__ void __launch_bounds__(256) stream_rw_kernel(const uint4* __restrict__ src, uint64_t r16,
                                                        uint4* __restrict__ dst, uint64_t w16, uint64_t wt16,
                                                        uint32_t* __restrict__ sink) {
    constexpr uint32_t kTile16 = 1024;  // 16 KB
    const uint64_t t = blockIdx.x;
    uint32_t acc = 0;
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t k = t * kTile16 + u * 256 + threadIdx.x;
        v[u] = k < r16 ? src[k] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    const uint64_t w0 = t * wt16, w1 = w0 + wt16 < w16 ? w0 + wt16 : w16;
    for (uint64_t k = w0 + threadIdx.x; k < w1; k += 256) dst[k] = make_uint4((uint32_t)k, (uint32_t)t, 0, 0);
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;  // practically never: keeps the loads live
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int halo_bench_read_peak(const void* buf, uint64_t bytes,
                                                                            uint32_t* sink, int warmup, int steps,
                                                                            void* stream, float* region_ms,
                                                                            double* wall_s) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const char* gb = getenv("HALO_READ_PEAK_BLOCKS");  // measurement tooling knob
    const uint32_t grid_blocks = gb ? (uint32_t)atoi(gb) : 256u * 32u;  // best of 1k..8k blocks (tools/exp/read_peak_sweep.sh)
    auto launch = [&](int) {
        hipLaunchKernelGGL(read_peak_kernel, dim3(grid_blocks), dim3(256), 0, s, static_cast<const uint4*>(buf),
                           bytes / 16, sink);
        return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
    };
    return timed_loop(launch, warmup, steps, s, region_ms, wall_s);
}

// The size-matched probe over `nbuf` rotating (src, dst) pairs, like the rx steps rotate batches.
extern "C" __attribute__((visibility("default"))) int halo_bench_stream_rw(const void* const* srcs,
                                                                            void* const* dsts, int nbuf,
                                                                            uint64_t read_bytes, uint64_t write_bytes,
                                                                            uint32_t* sink, int warmup, int steps,
                                                                            void* stream, float* region_ms,
                                                                            double* wall_s) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t r16 = read_bytes / 16, w16 = write_bytes / 16;
    const uint64_t tiles = (r16 + 1023) / 1024;
    if (!tiles || nbuf <= 0) return HALO_E_INVAL;
    const uint64_t wt16 = (w16 + tiles - 1) / tiles;
    auto launch = [&](int step) {
        const int b = step % nbuf;
        hipLaunchKernelGGL(stream_rw_kernel, dim3((uint32_t)tiles), dim3(256), 0, s, static_cast<const uint4*>(srcs[b]),
                           r16, static_cast<uint4*>(dsts[b]), w16, wt16, sink);
        return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
    };
    return timed_loop(launch, warmup, steps, s, region_ms, wall_s);
}

// Which physical device a rank ran on (bench.py's per-rank identity in the N-GPU line).
extern "C" __attribute__((visibility("default"))) int halo_bench_pci_bus_id(int device, char* buf, int len) {
    if (!buf || len < 13) return HALO_E_INVAL;
    return hipDeviceGetPCIBusId(buf, len, device) == hipSuccess ? HALO_OK : HALO_E_HIP;
}

// The fused receive + NAT flow-key pass (halo_rx_parse_flow_batch_device), rotating batches.
extern "C" __attribute__((visibility("default"))) int halo_bench_rx_flow_steps(
    int nbatch, const uint8_t* const* bytes, const uint32_t* const* offsets_dw, const uint16_t* const* lens,
    uint32_t n, uint32_t flags, const halo_rx_netif_t* netif, uint32_t hint, halo_rx_result_t* out, uint32_t kind,
    uint32_t nat_type, uint64_t* hash, uint32_t buckets, uint32_t* bucket, int warmup, int steps, void* stream,
    float* region_ms, double* wall_s) {
    if (nbatch <= 0) return HALO_E_INVAL;
    auto launch = [&](int k) {
        const int b = k % nbatch;
        return halo_rx_parse_flow_batch_device(bytes[b], offsets_dw[b], lens[b], n, flags, netif, hint, out, nullptr,
                                               kind, nat_type, hash, buckets, bucket, stream);
    };
    return timed_loop(launch, warmup, steps, static_cast<hipStream_t>(stream), region_ms, wall_s);
}

// BASELINE config 1 as a compiled caller runs it (the cgo PacketHandle of go/gpurx/ring.go): per
// batch the producer writes m frames into the ring (WritePacket per frame, untimed: the NIC side
// of engine.Wire / the DPDK lcore), then one halo_rx_ring_poll + halo_rx_ring_commit is timed —
// no Python between batches. us[k] = batch k's poll + commit time; *bad counts batches that did
// not return exactly m frames, all OK.
extern "C" __attribute__((visibility("default"))) int halo_bench_ring_polls(
    void* ring_mem, halo_rx_ring_t* ring, const uint8_t* bytes, const uint64_t* offs, const uint16_t* lens, uint32_t m,
    uint32_t flags, const halo_rx_netif_t* netif, halo_rx_result_t* out, int warmup, int iters, double* us,
    uint32_t* bad) {
    if (!ring_mem || !ring || !netif || !out || !us || !bad || iters <= 0) return HALO_E_INVAL;
    *bad = 0;
    for (int k = 0; k < warmup + iters; ++k) {
        uint32_t w = 0;
        int rc = halo_ring_write_batch(ring_mem, bytes, offs, lens, m, nullptr, &w);
        if (rc) return rc;
        if (w != m) return HALO_E_RANGE;  // the ring is full: the caller sized it wrong
        halo_rx_ring_scan_t info;
        const auto t0 = std::chrono::steady_clock::now();
        rc = halo_rx_ring_poll(ring, flags, netif, out, nullptr, nullptr, &info);
        if (!rc) rc = halo_rx_ring_commit(ring);
        const auto t1 = std::chrono::steady_clock::now();
        if (rc) return rc;
        bool ok = info.n_frames == m;
        for (uint32_t i = 0; ok && i < m; ++i) ok = out[i].status == HALO_RX_OK;
        if (!ok) ++*bad;
        if (k >= warmup) us[k - warmup] = std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    return HALO_OK;
}
