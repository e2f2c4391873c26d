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

// The end of a timed region: wait for the stream's last event, then synchronise the stream. With
// HALO_BENCH_SPIN=1 the host polls the event first (hipEventQuery) instead of letting
// hipStreamSynchronize fall back to a blocking, interrupt-woken wait once its short active-wait
// window has passed; either way the region ends only when every launch of it has completed.
// Off by default: polling was slower at 20 steps, 22.99 against 22.03 us per step.
static hipError_t finish_region(hipStream_t s, hipEvent_t last) {
    const char* v = getenv("HALO_BENCH_SPIN");
    if (v && v[0] == '1')
        while (hipEventQuery(last) == hipErrorNotReady) {
        }
    return hipStreamSynchronize(s);
}

// `hist` (optional, device): the status histogram every launch counts into (the §5 metrics output).
extern "C" __attribute__((visibility("default"))) int halo_bench_steps(
    int nbatch, const uint8_t* const* bytes, const uint32_t* const* offsets_dw, const uint16_t* const* lens,
    uint32_t n, uint64_t stride, uint32_t len, uint32_t flags, const halo_rx_netif_t* netif, uint32_t hint,
    halo_rx_result_t* out, uint32_t* hist, int warmup, int steps, void* stream, float* region_ms, double* wall_s) {
    if (nbatch <= 0 || steps <= 0 || !region_ms || !wall_s) return HALO_E_INVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto launch = [&](int k) -> int {
        const int b = k % nbatch;
        if (offsets_dw)
            return halo_rx_parse_batch_device(bytes[b], offsets_dw[b], lens[b], n, flags, netif, hint, out, hist,
                                              stream);
        return halo_rx_parse_strided_device(bytes[b], stride, lens ? lens[b] : nullptr, len, n, flags, netif, out,
                                            hist, stream);
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
    if (finish_region(s, e1) != hipSuccess && rc == HALO_OK) rc = HALO_E_HIP;
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
    if (finish_region(s, e1) != hipSuccess && rc == HALO_OK) rc = HALO_E_HIP;
    const auto t1 = std::chrono::steady_clock::now();
    *wall_s = std::chrono::duration<double>(t1 - t0).count();
    *region_ms = -1.0f;
    (void)hipEventElapsedTime(region_ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

// Generic timed loop over a launch callback (row f3 kernels: flow-key hashing, XXH3 batches).
// The headline step on `nq` streams at once (step k on stream k % nq, writing outs[k % nq]): a
// caller that keeps several batches in flight, as one NIC queue per stream would. The first stream is
// the caller's; the others are created here, start after an event on it and are joined back into it
// before the closing event, so one event pair on the caller's stream brackets every launch.
extern "C" __attribute__((visibility("default"))) int halo_bench_steps_queues(
    int nbatch, const uint8_t* const* bytes, const uint32_t* const* offsets_dw, const uint16_t* const* lens,
    uint32_t n, uint32_t flags, const halo_rx_netif_t* netif, uint32_t hint, halo_rx_result_t* const* outs, int nq,
    int warmup, int steps, void* stream, float* region_ms, double* wall_s) {
    if (nbatch <= 0 || nq <= 0 || nq > 8 || steps <= 0 || !region_ms || !wall_s) return HALO_E_INVAL;
    hipStream_t s0 = static_cast<hipStream_t>(stream);
    hipStream_t q[8] = {s0};
    hipEvent_t join[8] = {};
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = HALO_OK;
    for (int k = 1; k < nq && rc == HALO_OK; ++k)
        if (hipStreamCreateWithFlags(&q[k], hipStreamNonBlocking) != hipSuccess) rc = HALO_E_HIP;
    for (int k = 0; k < nq && rc == HALO_OK; ++k)
        if (hipEventCreateWithFlags(&join[k], hipEventDisableTiming) != hipSuccess) rc = HALO_E_HIP;
    if (rc == HALO_OK && (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) rc = HALO_E_HIP;
    auto launch = [&](int k) -> int {
        const int b = k % nbatch, j = k % nq;
        return halo_rx_parse_batch_device(bytes[b], offsets_dw[b], lens[b], n, flags, netif, hint, outs[j], nullptr,
                                          q[j]);
    };
    for (int k = 0; k < warmup && rc == HALO_OK; ++k) rc = launch(k);
    if (rc == HALO_OK && hipDeviceSynchronize() != hipSuccess) rc = HALO_E_HIP;
    if (rc == HALO_OK) {
        const auto t0 = std::chrono::steady_clock::now();
        (void)hipEventRecord(e0, s0);
        for (int k = 1; k < nq; ++k) (void)hipStreamWaitEvent(q[k], e0, 0);
        for (int k = 0; k < steps && rc == HALO_OK; ++k) rc = launch(k);
        for (int k = 1; k < nq; ++k) {
            (void)hipEventRecord(join[k], q[k]);
            (void)hipStreamWaitEvent(s0, join[k], 0);
        }
        (void)hipEventRecord(e1, s0);
        if (hipStreamSynchronize(s0) != hipSuccess && rc == HALO_OK) rc = HALO_E_HIP;
        const auto t1 = std::chrono::steady_clock::now();
        *wall_s = std::chrono::duration<double>(t1 - t0).count();
        *region_ms = -1.0f;
        (void)hipEventElapsedTime(region_ms, e0, e1);
    }
    (void)hipDeviceSynchronize();
    for (int k = 1; k < nq; ++k)
        if (q[k]) (void)hipStreamDestroy(q[k]);
    for (int k = 0; k < nq; ++k)
        if (join[k]) (void)hipEventDestroy(join[k]);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return rc;
}

// Tools only (tools/exp/split_steps.py): each step's batch split into `parts` index ranges launched
// on as many streams at once (fork from the caller's stream by an event, join back by events), so a
// single batch is fed by several HSA queues. Records are the same as one launch's.
extern "C" __attribute__((visibility("default"))) int halo_bench_split_steps(
    int nbatch, const uint8_t* const* bytes, const uint32_t* const* offsets_dw, const uint16_t* const* lens,
    uint32_t n, uint32_t flags, const halo_rx_netif_t* netif, uint32_t hint, halo_rx_result_t* out, int parts,
    int warmup, int steps, void* stream, float* region_ms, double* wall_s) {
    if (nbatch <= 0 || parts <= 0 || parts > 8 || steps <= 0 || !region_ms || !wall_s) return HALO_E_INVAL;
    hipStream_t s0 = static_cast<hipStream_t>(stream);
    hipStream_t q[8] = {s0};
    hipEvent_t fork = nullptr, join[8] = {}, e0 = nullptr, e1 = nullptr;
    int rc = HALO_OK;
    for (int k = 1; k < parts && rc == HALO_OK; ++k)
        if (hipStreamCreateWithFlags(&q[k], hipStreamNonBlocking) != hipSuccess) rc = HALO_E_HIP;
    if (rc == HALO_OK && hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess) rc = HALO_E_HIP;
    for (int k = 1; k < parts && rc == HALO_OK; ++k)
        if (hipEventCreateWithFlags(&join[k], hipEventDisableTiming) != hipSuccess) rc = HALO_E_HIP;
    if (rc == HALO_OK && (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) rc = HALO_E_HIP;
    const uint32_t per = ((n + parts - 1) / parts + 63u) & ~63u;  // whole 64-frame windows per part
    auto launch = [&](int k) -> int {
        const int b = k % nbatch;
        int r = HALO_OK;
        if (parts > 1) {
            (void)hipEventRecord(fork, s0);
            for (int j = 1; j < parts; ++j) (void)hipStreamWaitEvent(q[j], fork, 0);
        }
        for (int j = 0; j < parts && r == HALO_OK; ++j) {
            const uint32_t lo = j * per, cnt = lo >= n ? 0u : (n - lo < per ? n - lo : per);
            if (cnt)
                r = halo_rx_parse_batch_device(bytes[b], offsets_dw[b] + lo, lens[b] + lo, cnt, flags, netif, hint,
                                               out + lo, nullptr, q[j]);
        }
        for (int j = 1; j < parts; ++j) {
            (void)hipEventRecord(join[j], q[j]);
            (void)hipStreamWaitEvent(s0, join[j], 0);
        }
        return r;
    };
    for (int k = 0; k < warmup && rc == HALO_OK; ++k) rc = launch(k);
    if (rc == HALO_OK && hipDeviceSynchronize() != hipSuccess) rc = HALO_E_HIP;
    if (rc == HALO_OK) {
        const auto t0 = std::chrono::steady_clock::now();
        (void)hipEventRecord(e0, s0);
        for (int k = 0; k < steps && rc == HALO_OK; ++k) rc = launch(k);
        (void)hipEventRecord(e1, s0);
        if (hipStreamSynchronize(s0) != hipSuccess && rc == HALO_OK) rc = HALO_E_HIP;
        const auto t1 = std::chrono::steady_clock::now();
        *wall_s = std::chrono::duration<double>(t1 - t0).count();
        *region_ms = -1.0f;
        (void)hipEventElapsedTime(region_ms, e0, e1);
    }
    (void)hipDeviceSynchronize();
    for (int k = 1; k < parts; ++k) {
        if (q[k]) (void)hipStreamDestroy(q[k]);
        if (join[k]) (void)hipEventDestroy(join[k]);
    }
    if (fork) (void)hipEventDestroy(fork);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return rc;
}

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
    if (finish_region(s, e1) != hipSuccess && rc == HALO_OK) rc = HALO_E_HIP;
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

extern "C" __attribute__((visibility("default"))) int halo_bench_flow_compact_steps(
    int nbatch, const halo_rx_record16_t* const* recs, uint32_t n, uint32_t kind, uint32_t nat_type, uint64_t* hash,
    uint32_t buckets, uint32_t* bucket, int warmup, int steps, void* stream, float* region_ms, double* wall_s) {
    if (nbatch <= 0) return HALO_E_INVAL;
    auto launch = [&](int k) {
        return halo_flow_hash_compact_device(recs[k % nbatch], n, kind, nat_type, hash, buckets, bucket, stream);
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

// flow_hash.hip built again as the XXH3 load-pattern probe (halo_amd/build.py build_bench)
extern "C" int halo_bench_xxh3_probe_launch(const uint8_t* d_bytes, const uint64_t* d_offsets, const uint32_t* d_lens,
                                            uint32_t n, uint64_t* d_hash, void* stream);
extern "C" __attribute__((visibility("default"))) int halo_bench_xxh3_probe_steps(
    int nbatch, const uint8_t* const* bytes, const uint64_t* const* offsets, const uint32_t* const* lens, uint32_t n,
    uint64_t* hash, int warmup, int steps, void* stream, float* region_ms, double* wall_s) {
    if (nbatch <= 0) return HALO_E_INVAL;
    auto launch = [&](int k) {
        const int b = k % nbatch;
        return halo_bench_xxh3_probe_launch(bytes[b], offsets[b], lens[b], n, hash, stream);
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

// The read probe family (halo_bench_read_probe): block b reads tile b once — BLOCK threads x U
// chunks of 16 B, all U loads in flight per lane, consecutive lanes on consecutive chunks — with
// plain or non-temporal loads. No grid-stride loop: like the rx kernels, one wave never loops, the
// dispatcher refills CUs. bench.py takes the fastest of the family and of read_peak_kernel as the
// box's measured read peak (a single probe shape was beaten by the jumbo kernel).
template <int BLOCK, int U, bool NT>
__global__ void __launch_bounds__(BLOCK) read_tile_kernel(const uint4* __restrict__ src, uint64_t n16,
                                                          uint32_t* __restrict__ sink) {
    const uint64_t base = (uint64_t)blockIdx.x * U * BLOCK + threadIdx.x;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t k = base + (uint64_t)u * BLOCK;
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        if (k < n16 && NT) {
            const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + k);
            v[u] = make_uint4(t.x, t.y, t.z, t.w);
        } else {
            v[u] = k < n16 ? src[k] : make_uint4(0, 0, 0, 0);
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    if (acc == 0x9E3779B9u) sink[blockIdx.x & 4095u] = acc;  // practically never: keeps the loads live
}

// Size-matched speed-of-light probe: block t reads tile t of `src` (U 16-byte loads per thread in
// flight: a 4U KB tile) and writes its share of `dst` with coalesced 16-byte stores — the rx kernel's
// bytes (frames + metadata in, records out) with perfect access patterns and no work. A family of
// shapes (tile size, non-temporal loads and stores) of which bench.py takes the fastest, so that the
// probe is a ceiling at every size (the 16 KB plain shape alone ran slower than the
// rx kernel at 16M frames).
template <int U, bool NT, bool NT_ST = NT>
__global__ void __launch_bounds__(256) stream_rw_kernel(const uint4* __restrict__ src, uint64_t r16,
                                                        uint4* __restrict__ dst, uint64_t w16, uint64_t wt16,
                                                        uint32_t* __restrict__ sink) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    constexpr uint32_t kTile16 = 256 * U;
    const uint64_t t = blockIdx.x;
    uint32_t acc = 0;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t k = t * kTile16 + u * 256 + threadIdx.x;
        if (NT && k < r16) {
            const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + k);
            v[u] = make_uint4(x.x, x.y, x.z, x.w);
        } else {
            v[u] = k < r16 ? src[k] : make_uint4(0, 0, 0, 0);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    const uint64_t w0 = t * wt16, w1 = w0 + wt16 < w16 ? w0 + wt16 : w16;
    for (uint64_t k = w0 + threadIdx.x; k < w1; k += 256) {
        if (NT_ST) {
            const u32x4 x = {(uint32_t)k, (uint32_t)t, 0u, 0u};
            __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(dst) + k);
        } else {
            dst[k] = make_uint4((uint32_t)k, (uint32_t)t, 0, 0);
        }
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x & 0xFFFFFu] = acc;  // practically never: keeps the loads live
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

// Read probe `variant` over `bytes` (a multiple of 64 KiB): 0 = read_peak_kernel (8192 blocks of
// 256 threads streaming 64 KB tiles), 1.. = read_tile_kernel shapes (see kReadProbes). Returns
// HALO_E_RANGE past the last variant.
namespace {
struct ReadProbe {
    const char* name;
    void (*launch)(const uint4*, uint64_t, uint32_t*, hipStream_t);
};
template <int BLOCK, int U, bool NT>
void launch_tile(const uint4* src, uint64_t n16, uint32_t* sink, hipStream_t s) {
    const uint64_t blocks = (n16 + (uint64_t)U * BLOCK - 1) / ((uint64_t)U * BLOCK);
    hipLaunchKernelGGL((read_tile_kernel<BLOCK, U, NT>), dim3((uint32_t)blocks), dim3(BLOCK), 0, s, src, n16, sink);
}
const ReadProbe kReadProbes[] = {
    {"tile256_u4", launch_tile<256, 4, false>},   {"tile256_u8", launch_tile<256, 8, false>},
    {"tile256_u16", launch_tile<256, 16, false>}, {"tile256_u8_nt", launch_tile<256, 8, true>},
    {"tile256_u16_nt", launch_tile<256, 16, true>}, {"tile64_u8", launch_tile<64, 8, false>},
    {"tile64_u16", launch_tile<64, 16, false>},   {"tile1024_u4", launch_tile<1024, 4, false>},
};
}  // namespace

extern "C" __attribute__((visibility("default"))) const char* halo_bench_read_probe_name(int variant) {
    if (variant == 0) return "persistent256_64KB";
    if (variant < 1 || variant > (int)(sizeof kReadProbes / sizeof kReadProbes[0])) return nullptr;
    return kReadProbes[variant - 1].name;
}

extern "C" __attribute__((visibility("default"))) int halo_bench_read_probe(const void* buf, uint64_t bytes,
                                                                             uint32_t* sink, int variant,
                                                                             int warmup, int steps, void* stream,
                                                                             float* region_ms, double* wall_s) {
    if (variant == 0) return halo_bench_read_peak(buf, bytes, sink, warmup, steps, stream, region_ms, wall_s);
    if (variant < 1 || variant > (int)(sizeof kReadProbes / sizeof kReadProbes[0])) return HALO_E_RANGE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const ReadProbe& p = kReadProbes[variant - 1];
    auto launch = [&](int) {
        p.launch(static_cast<const uint4*>(buf), bytes / 16, sink, s);
        return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
    };
    return timed_loop(launch, warmup, steps, s, region_ms, wall_s);
}

// The size-matched probe over `nbuf` rotating (src, dst) pairs, like the rx steps rotate batches.
// `variant` picks the shape (halo_bench_stream_rw_name): HALO_E_RANGE past the last one.
namespace {
struct RwProbe {
    const char* name;
    uint32_t u;  // 16-byte loads per thread: the tile is 4u KB
    void (*kernel)(const uint4*, uint64_t, uint4*, uint64_t, uint64_t, uint32_t*);
};
const RwProbe kRwProbes[] = {
    {"tile16k", 4, stream_rw_kernel<4, false>},     {"tile16k_nt", 4, stream_rw_kernel<4, true>},
    {"tile32k_nt", 8, stream_rw_kernel<8, true>},   {"tile64k_nt", 16, stream_rw_kernel<16, true>},
    {"tile32k", 8, stream_rw_kernel<8, false>},
    // which half of the non-temporal gain is whose: NT loads with plain stores, and the reverse
    {"tile16k_ntld", 4, stream_rw_kernel<4, true, false>}, {"tile16k_ntst", 4, stream_rw_kernel<4, false, true>},
};
constexpr int kNumRwProbes = sizeof kRwProbes / sizeof kRwProbes[0];
}  // namespace

extern "C" __attribute__((visibility("default"))) const char* halo_bench_stream_rw_name(int variant) {
    return variant >= 0 && variant < kNumRwProbes ? kRwProbes[variant].name : nullptr;
}

extern "C" __attribute__((visibility("default"))) int halo_bench_stream_rw_v(const void* const* srcs,
                                                                              void* const* dsts, int nbuf,
                                                                              uint64_t read_bytes, uint64_t write_bytes,
                                                                              uint32_t* sink, int variant, int warmup,
                                                                              int steps, void* stream, float* region_ms,
                                                                              double* wall_s) {
    if (variant < 0 || variant >= kNumRwProbes) return HALO_E_RANGE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const RwProbe& pr = kRwProbes[variant];
    const uint64_t r16 = read_bytes / 16, w16 = write_bytes / 16;
    const uint64_t tile16 = 256ull * pr.u;
    const uint64_t tiles = (r16 + tile16 - 1) / tile16;
    if (!tiles || nbuf <= 0 || tiles > 0xFFFFFFFFull) return HALO_E_INVAL;
    const uint64_t wt16 = (w16 + tiles - 1) / tiles;
    auto launch = [&](int step) {
        const int b = step % nbuf;
        hipLaunchKernelGGL(pr.kernel, dim3((uint32_t)tiles), dim3(256), 0, s, static_cast<const uint4*>(srcs[b]), r16,
                           static_cast<uint4*>(dsts[b]), w16, wt16, sink);
        return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
    };
    return timed_loop(launch, warmup, steps, s, region_ms, wall_s);
}

// The first shape (16 KB tiles, plain loads and stores): round 5's probe.
extern "C" __attribute__((visibility("default"))) int halo_bench_stream_rw(const void* const* srcs,
                                                                            void* const* dsts, int nbuf,
                                                                            uint64_t read_bytes, uint64_t write_bytes,
                                                                            uint32_t* sink, int warmup, int steps,
                                                                            void* stream, float* region_ms,
                                                                            double* wall_s) {
    return halo_bench_stream_rw_v(srcs, dsts, nbuf, read_bytes, write_bytes, sink, 0, warmup, steps, stream, region_ms,
                                  wall_s);
}

// The transmit build's own layout with no build work (the tx_build line's layout-matched probe):
// waves own 64-frame tiles like tx_build_kernel (lane l loads descriptor l's 40 bytes), then 32
// lanes per frame, two frames per step, three 16-byte chunks per lane: payload bytes [16c - 42,
// +16) of the frame's payload (unaligned 16-byte loads from the same addresses the build reads; payload i at pitch * i),
// the slot's dwords up to the frame's end stored at the same addresses, then length and result.
// What the output format (1514 B frames in 1516 B slots, payloads 1472 B apart) costs before any
// arithmetic; the size-matched probe streams the same byte counts aligned and contiguous.
__global__ void __launch_bounds__(256) tx_layout_probe_kernel(const uint2* desc, const uint8_t* pay, uint32_t plen,
                                                              uint32_t pitch, uint8_t* frames, uint32_t stride, uint32_t flen,
                                                              uint16_t* lens, uint8_t* res, uint32_t n,
                                                              uint32_t* sink, uint32_t interleave) {
    typedef uint32_t u32x4b __attribute__((ext_vector_type(4), aligned(1)));
    const uint32_t lane = threadIdx.x & 63u, j = lane & 31u, g = lane >> 5;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    const uint32_t chunks = (flen + 15u) / 16u, ndw = (flen + 3u) / 4u, tiles = (n + 63u) / 64u;
    for (uint32_t t = wave; t < tiles; t += nw) {
        uint32_t x = 0;
        if (t * 64u + lane < n) {
            const uint2* d = desc + 5ull * (t * 64u + lane);
#pragma unroll
            for (int k = 0; k < 5; ++k) x ^= d[k].x + d[k].y;
        }
#pragma unroll 1
        for (uint32_t step = 0; step < 32; ++step) {
            // interleave (a diagnostic): step s of wave w takes frame pair s * nw + w instead, so the
            // waves in flight at any time cover one contiguous window of frames
            const uint32_t f = interleave ? 2 * ((t - wave) / nw * 32 * nw + step * nw + wave) + g
                                          : t * 64u + 2 * step + g;
            const uint32_t y = (uint32_t)__shfl((int)x, (int)(2 * step + g), 64);
            if (f >= n) continue;
            uint32_t w[3][4];
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const uint32_t c = j + 32u * u;
                w[u][0] = w[u][1] = w[u][2] = w[u][3] = y + c;
                if (16 * c >= 42 && 16 * c + 16 <= 42 + plen) {
                    const u32x4b v = *(const __attribute__((address_space(1))) u32x4b*)(pay + (uint64_t)pitch * f + 16 * c - 42);
                    w[u][0] = v.x; w[u][1] = v.y; w[u][2] = v.z; w[u][3] = v.w;
                }
            }
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const uint32_t c = j + 32u * u;
                if (c >= chunks) continue;
                uint32_t* o = reinterpret_cast<uint32_t*>(frames + (uint64_t)stride * f) + 4 * c;
                if (4 * c + 4 <= ndw) {
                    *reinterpret_cast<uint4*>(o) = make_uint4(w[u][0], w[u][1], w[u][2], w[u][3]);
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (4 * c + i < ndw) o[i] = w[u][i];
                }
            }
            if (j == 0) {
                lens[f] = (uint16_t)flen;
                res[f] = (uint8_t)(y == 0x9E3779B9u);
            }
        }
    }
    if (lane == 64) sink[0] = 0;  // never: keeps the signature uniform with the other probes
}

extern "C" __attribute__((visibility("default"))) int halo_bench_tx_layout_probe(
    const void* desc, const void* pay, uint32_t plen, uint32_t pitch, void* frames, uint32_t stride, uint32_t flen, void* lens,
    void* res, uint32_t n, uint32_t* sink, uint32_t interleave, int warmup, int steps, void* stream, float* region_ms,
    double* wall_s) {
    if (!desc || !pay || !frames || !lens || !res || n == 0 || (stride & 3u) || flen > stride || flen > 1536u ||
        (reinterpret_cast<uintptr_t>(frames) & 3u))
        return HALO_E_INVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint32_t tiles = (n + 63u) / 64u, blocks = (tiles + 3u) / 4u;
    const dim3 grid(blocks < 1024u ? blocks : 1024u);  // tx_build_kernel's grid for this batch
    auto launch = [&](int) {
        hipLaunchKernelGGL(tx_layout_probe_kernel, grid, dim3(256), 0, s, static_cast<const uint2*>(desc),
                           static_cast<const uint8_t*>(pay), plen, pitch, static_cast<uint8_t*>(frames), stride, flen,
                           static_cast<uint16_t*>(lens), static_cast<uint8_t*>(res), n, sink, interleave);
        return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
    };
    return timed_loop(launch, warmup, steps, s, region_ms, wall_s);
}

// The route lookup's access pattern with no lookup logic (the route line's gather probe): one
// table entry per address at a random index (tbl[ip >> 8] over a 2^24-entry, 64 MB table, as
// DIR-24-8's first level), one 4-byte result out, lane per address, rotating address arrays.
__global__ void __launch_bounds__(256) gather_probe_kernel(const uint32_t* __restrict__ tbl,
                                                           const uint32_t* __restrict__ ips, uint32_t n,
                                                           uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) out[i] = tbl[ips[i] >> 8];
}

extern "C" __attribute__((visibility("default"))) int halo_bench_gather_probe(
    const void* tbl, const void* const* ips, int nb, uint32_t n, void* out, int warmup, int steps, void* stream,
    float* region_ms, double* wall_s) {
    if (!tbl || !ips || nb <= 0 || !out || n == 0) return HALO_E_INVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto launch = [&](int step) {
        hipLaunchKernelGGL(gather_probe_kernel, dim3((n + 255u) / 256u), dim3(256), 0, s,
                           static_cast<const uint32_t*>(tbl), static_cast<const uint32_t*>(ips[step % nb]), n,
                           static_cast<uint32_t*>(out));
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

// The drop-in surface as a cgo caller drives it (go/gpurx Ctx.ParseBatch, the batched PacketHandle
// of go/engine at its 99-poll cadence, and — m = 1 — the single-frame Parse* wrappers): per call
// halo_rx_parse_batch_host over m frames in pageable host memory (Go slices) + halo_rx_dispatch over
// the records. us[k] = call k's time; *bad counts calls whose records were not all OK / LOCAL_UDP.
extern "C" __attribute__((visibility("default"))) int halo_bench_host_calls(
    halo_rx_host_ctx_t* ctx, const uint8_t* bytes, const uint64_t* offs, const uint16_t* lens, uint32_t m,
    uint32_t flags, const halo_rx_netif_t* netif, halo_rx_result_t* out, uint8_t* acts, int warmup, int iters,
    double* us, uint32_t* bad) {
    if (!ctx || !netif || !out || !acts || !us || !bad || iters <= 0) return HALO_E_INVAL;
    *bad = 0;
    for (int k = 0; k < warmup + iters; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        int rc = halo_rx_parse_batch_host(ctx, bytes, offs, lens, m, flags, netif, out, nullptr);
        if (!rc) rc = halo_rx_dispatch(out, m, netif, acts, nullptr);
        const auto t1 = std::chrono::steady_clock::now();
        if (rc) return rc;
        bool ok = true;
        for (uint32_t i = 0; ok && i < m; ++i) ok = out[i].status == HALO_RX_OK && acts[i] == HALO_RX_ACT_LOCAL_UDP;
        if (!ok) ++*bad;
        if (k >= warmup) us[k - warmup] = std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    return HALO_OK;
}

// The same per-call loop over the CPU entry point (include/halo_rx_cpu.h), passed as a function
// pointer so that this library does not link libhalo_rx_cpu.so: halo_rx_parse_batch_cpu +
// halo_rx_dispatch per call, on the calling core.
typedef int (*halo_cpu_parse_fn)(const uint8_t*, const uint64_t*, const uint16_t*, uint32_t, uint32_t,
                                 const halo_rx_netif_t*, halo_rx_result_t*, uint32_t*);
extern "C" __attribute__((visibility("default"))) int halo_bench_cpu_calls(
    void* parse_cpu, const uint8_t* bytes, const uint64_t* offs, const uint16_t* lens, uint32_t m, uint32_t flags,
    const halo_rx_netif_t* netif, halo_rx_result_t* out, uint8_t* acts, int warmup, int iters, double* us,
    uint32_t* bad) {
    if (!parse_cpu || !netif || !out || !acts || !us || !bad || iters <= 0) return HALO_E_INVAL;
    const auto fn = reinterpret_cast<halo_cpu_parse_fn>(parse_cpu);
    *bad = 0;
    for (int k = 0; k < warmup + iters; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        int rc = fn(bytes, offs, lens, m, flags, netif, out, nullptr);
        if (!rc) rc = halo_rx_dispatch(out, m, netif, acts, nullptr);
        const auto t1 = std::chrono::steady_clock::now();
        if (rc) return rc;
        bool ok = true;
        for (uint32_t i = 0; ok && i < m; ++i) ok = out[i].status == HALO_RX_OK && acts[i] == HALO_RX_ACT_LOCAL_UDP;
        if (!ok) ++*bad;
        if (k >= warmup) us[k - warmup] = std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    return HALO_OK;
}

// The batch stream handed over k batches per launch (halo_rx_parse_batches_device): step t parses
// batches (t * k + j) % nbatch, j < k, into outs[j].
extern "C" __attribute__((visibility("default"))) int halo_bench_multi_steps(
    int nbatch, const uint8_t* const* bytes, const uint32_t* const* offsets_dw, const uint16_t* const* lens, uint32_t n,
    uint32_t k, uint32_t flags, const halo_rx_netif_t* netif, uint32_t hint, halo_rx_result_t* const* outs,
    uint32_t* hist, int warmup, int steps, void* stream, float* region_ms, double* wall_s) {
    if (nbatch <= 0 || k == 0 || k > 32) return HALO_E_INVAL;
    auto launch = [&](int t) {
        halo_rx_batch_desc_t d[32];
        for (uint32_t j = 0; j < k; ++j) {
            const int b = (int)(((uint64_t)t * k + j) % (uint64_t)nbatch);
            d[j] = halo_rx_batch_desc_t{bytes[b], offsets_dw[b], lens[b], outs[j], n, 0};
        }
        return halo_rx_parse_batches_device(d, k, flags, netif, hint, hist, stream);
    };
    return timed_loop(launch, warmup, steps, static_cast<hipStream_t>(stream), region_ms, wall_s);
}
