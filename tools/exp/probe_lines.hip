// probe_lines.hip — which 128-byte lines get fetched twice when 8-lane groups read packed 1500-byte
// frames (tools only, not shipped). Build: hipcc --offload-arch=gfx950 -O3 -o tools/exp/probe_lines
// tools/exp/probe_lines.hip. Run under rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum ...; each variant is
// its own kernel so the rows attribute by name.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
typedef const __attribute__((address_space(1))) u32x4 gv4;

constexpr uint32_t kLen = 1500, kStride = 1500;  // frames packed back to back (4-byte aligned)

__device__ __forceinline__ u32x4 ld(const uint8_t* base, uint64_t f, uint32_t c) {
    const uint32_t off = 16 * c;
    if (off + 16 > kLen) return (u32x4){0, 0, 0, 0};  // partial tail chunk skipped: lines only
    return *(gv4*)(base + f * kStride + off);
}

// 12 rows of 8 lanes x 16 B per frame, all issued before any is used (one round)
__global__ void __launch_bounds__(256) one_round(const uint8_t* base, uint32_t n, uint32_t* sink) {
    const uint32_t lane = threadIdx.x & 63u, gl = lane & 7u;
    const uint64_t f = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 3;
    if (f >= n) return;
    u32x4 v[12];
#pragma unroll
    for (int u = 0; u < 12; ++u) v[u] = ld(base, f, u * 8 + gl);
    uint32_t a = 0;
#pragma unroll
    for (int u = 0; u < 12; ++u) a ^= v[u].x + v[u].y + v[u].z + v[u].w;
    if (a == 0x9E3779B9u) sink[f] = a;
}

// rows 0..3, then (their values used first) rows 4..11: two dependent rounds, as rx_group_kernel<8>
__global__ void __launch_bounds__(256) two_rounds(const uint8_t* base, uint32_t n, uint32_t* sink) {
    const uint32_t lane = threadIdx.x & 63u, gl = lane & 7u;
    const uint64_t f = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 3;
    if (f >= n) return;
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld(base, f, u * 8 + gl);
    uint32_t a = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) a ^= v[u].x + v[u].y + v[u].z + v[u].w;
    a = __shfl(a, 0, 64) & 1u;  // a dependency: round 1 waits for round 0
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ld(base, f, (4 + u) * 8 + gl + a * 0x100000u * 0);
#pragma unroll
    for (int u = 0; u < 8; ++u) a ^= v[u].x + v[u].y + v[u].z + v[u].w;
    if (a == 0x9E3779B9u) sink[f] = a;
}

// the wave reads its 8 frames' span as one contiguous stream (1 KB per instruction)
__global__ void __launch_bounds__(256) span_stream(const uint8_t* base, uint32_t n, uint32_t* sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t w = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint64_t f0 = w * 8;
    if (f0 >= n) return;
    const uint64_t lo = (f0 * kStride) & ~15ull, hi = ((f0 + 8) * kStride + 15) & ~15ull;
    uint32_t a = 0;
    u32x4 v[12];
#pragma unroll
    for (int u = 0; u < 12; ++u) {
        const uint64_t o = lo + 1024ull * u + 16ull * lane;
        v[u] = o < hi ? *(gv4*)(base + o) : (u32x4){0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 12; ++u) a ^= v[u].x + v[u].y + v[u].z + v[u].w;
    if (a == 0x9E3779B9u) sink[w] = a;
}

int main() {
    const uint32_t n = 1u << 20;
    uint8_t* buf;
    uint32_t* sink;
    if (hipMalloc(&buf, (uint64_t)n * kStride + 4096) != hipSuccess || hipMalloc(&sink, 4ull * n) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, (uint64_t)n * kStride + 4096);
    const dim3 blk(256), grid((n * 8 + 255) / 256);
    for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(one_round, grid, blk, 0, 0, buf, n, sink);
    for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(two_rounds, grid, blk, 0, 0, buf, n, sink);
    for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(span_stream, grid, blk, 0, 0, buf, n, sink);
    (void)hipDeviceSynchronize();
    printf("frames %u x %u B, span %.1f MB (%.2f lines of 128 B per frame if each line is read once)\n", n, kLen,
           (double)n * kStride / 1e6, kStride / 128.0);
    return 0;
}
