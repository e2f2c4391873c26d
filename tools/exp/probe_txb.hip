// probe_txb.hip — memory-pattern probes for the transmit build (tools only, not shipped).
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_txb tools/exp/probe_txb.hip ; run on the GPU box.
// Each probe moves the bytes of one tx_build workload with as little arithmetic as possible, so
// the gap between a probe and the real kernel is the kernel's own cost.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
typedef const __attribute__((address_space(1))) u32x4 gv4;
typedef const __attribute__((address_space(1))) uint32_t gu32;

// lane per 64 B frame: descriptor (40 B) + 22 B payload in, 64 B frame out (4 x 16 B stores)
template <bool DESC, bool LOAD, bool STORE>
__global__ void __launch_bounds__(256) small_frames(const uint2* desc, const uint8_t* pay, uint8_t* frames, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t x = i;
    if (DESC) {
        const uint2* d = desc + 5ull * i;
#pragma unroll
        for (int k = 0; k < 5; ++k) { const uint2 v = d[k]; x ^= v.x + v.y; }
    }
    uint32_t w[8] = {x, x, x, x, x, x, x, x};
    if (LOAD) {
        const uint64_t a = (uint64_t)pay + 22ull * i;
        const u32x4 v = *(gv4*)(a & ~3ull);
        const uint32_t t = *(gu32*)((a & ~3ull) + 16);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w; w[4] = t;
    }
    if (STORE) {
        uint4* o = reinterpret_cast<uint4*>(frames + 64ull * i);
        o[0] = make_uint4(w[0], w[1], x, w[2]);
        o[1] = make_uint4(w[3], x, w[4], w[1]);
        o[2] = make_uint4(w[2], w[0], x, w[3]);
        o[3] = make_uint4(x, w[4], w[1], w[0]);
    } else if ((w[0] ^ w[1] ^ w[2] ^ w[3] ^ w[4]) == 0x9E3779B9u) {
        frames[i] = 1;
    }
}

// G lanes per frame (stride bytes), CH 16-byte chunks per lane, payload at pstride per frame
template <int G, int CH, bool LOAD, bool STORE>
__global__ void __launch_bounds__(256) big_frames(const uint8_t* pay, uint8_t* frames, uint32_t n, uint32_t flen,
                                                  uint32_t stride, uint32_t pstride) {
    const uint32_t lane = threadIdx.x & 63u, j = lane % G;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t base = wave * (64 / G); base < n; base += nw * (64 / G)) {
        const uint32_t f = base + lane / G;
        if (f >= n) continue;
        uint32_t w[CH][4];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const uint32_t c = j + u * G;
            w[u][0] = w[u][1] = w[u][2] = w[u][3] = c;
            if (LOAD && 16 * c + 16 <= flen) {
                const uint64_t a = (uint64_t)pay + (uint64_t)pstride * f + 16 * c + 2;  // 2-byte misaligned source
                const u32x4 v = *(gv4*)(a & ~3ull);
                w[u][0] = v.x; w[u][1] = v.y; w[u][2] = v.z; w[u][3] = v.w;
            }
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const uint32_t c = j + u * G;
            if (16 * c + 16 > flen) continue;
            if (STORE) {
                *reinterpret_cast<uint4*>(frames + (uint64_t)stride * f + 16 * c) =
                    make_uint4(w[u][0], w[u][1], w[u][2], w[u][3]);
            } else if ((w[u][0] ^ w[u][1] ^ w[u][2] ^ w[u][3]) == 0x9E3779B9u) {
                frames[f] = 1;
            }
        }
    }
}


// lane per 64 B frame as the kernel's build_small loads its payload: NLD clamped dword loads
// (sources 7..16 or 10..16 of the frame in payload space) instead of one 16 B + one 4 B load
template <int NLD>
__global__ void __launch_bounds__(256) small_dwords(const uint2* desc, const uint8_t* pay, uint8_t* frames, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t x = i;
    const uint2* d = desc + 5ull * i;
#pragma unroll
    for (int k = 0; k < 5; ++k) { const uint2 v = d[k]; x ^= v.x + v.y; }
    const uint64_t a = (uint64_t)pay + 22ull * i, lo = a & ~3ull;
    const int32_t last = (int32_t)(((a + 22 + 3) & ~3ull) - lo) / 4 - 1;
    const int32_t r0 = -11 + (int32_t)(x & 1u);
    uint32_t w[10];
#pragma unroll
    for (int m = 0; m < NLD; ++m) {
        const int32_t r = r0 + (10 - NLD) + 7 + m;
        w[m] = ((gu32*)lo)[r < 0 ? 0 : r > last ? last : r];
    }
#pragma unroll
    for (int m = NLD; m < 10; ++m) w[m] = x;
    uint4* o = reinterpret_cast<uint4*>(frames + 64ull * i);
    o[0] = make_uint4(w[0], w[1], x, w[2]);
    o[1] = make_uint4(w[3], w[5], w[4], w[1]);
    o[2] = make_uint4(w[2], w[6], w[7], w[3]);
    o[3] = make_uint4(w[8], w[4], w[9], w[0]);
}

// four lanes per 64 B frame: the tile's descriptors read coalesced (16 B per lane), each lane one
// 16 B payload load and one 16 B store of its chunk (a store instruction covers 16 whole frames)
__global__ void __launch_bounds__(256) quad_frames(const uint4* desc, const uint8_t* pay, uint8_t* frames, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t t = wave; t * 64 < n; t += nw) {
        // 64 descriptors = 2560 B = 160 x 16 B
        uint32_t x = 0;
        const uint4* dt = desc + (uint64_t)t * 160;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint32_t q = lane + 64 * k;
            if (q < 160) { const uint4 v = dt[q]; x ^= v.x + v.y + v.z + v.w; }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint32_t f = t * 64 + s * 16 + lane / 4, j = lane & 3u;
            if (f >= n) continue;
            const uint64_t a = ((uint64_t)pay + 22ull * f + 16 * j) & ~3ull;
            uint32_t w0 = x, w1 = x, w2 = x, w3 = x;
            if (j >= 2) { const u32x4 v = *(gv4*)a; w0 = v.x; w1 = v.y; w2 = v.z; w3 = v.w; }
            *reinterpret_cast<uint4*>(frames + 64ull * f + 16 * j) = make_uint4(w0, w1 ^ x, w2, w3);
        }
    }
}

template <typename F>
static float time_it(F launch, int iters) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int k = 0; k < 3; ++k) launch();
    CK(hipEventRecord(a));
    for (int k = 0; k < iters; ++k) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.0f / iters;  // us
}

int main() {
    const uint32_t n = 1u << 20;
    uint2* desc;
    uint8_t *pay, *frames;
    CK(hipMalloc(&desc, 40ull * n));
    CK(hipMalloc(&pay, 1600ull * (n / 4) + 64));
    CK(hipMalloc(&frames, 1600ull * (n / 4) + 64));
    CK(hipMemset(desc, 1, 40ull * n));
    CK(hipMemset(pay, 2, 1600ull * (n / 4) + 64));
    const dim3 blk(256), grid((n + 255) / 256);
#define SMALL(D, L, S, name)                                                                          \
    {                                                                                                 \
        float us = time_it([&] { hipLaunchKernelGGL((small_frames<D, L, S>), grid, blk, 0, 0, desc, pay, frames, n); }, \
                           50);                                                                       \
        double bytes = (D ? 40.0 : 0) * n + (L ? 24.0 : 0) * n + (S ? 64.0 : 0) * n;                 \
        printf("%-34s %8.2f us  %7.1f GB/s\n", name, us, bytes / us / 1e3);                           \
    }
    SMALL(true, true, true, "64B: desc+payload in, frame out");
    SMALL(false, true, true, "64B: payload in, frame out");
    SMALL(false, false, true, "64B: frame out only");
    SMALL(true, false, false, "64B: desc in only");
    SMALL(false, true, false, "64B: payload in only");
    {
        float us = time_it([&] { hipLaunchKernelGGL(small_dwords<10>, grid, blk, 0, 0, desc, pay, frames, n); }, 50);
        printf("%-34s %8.2f us\n", "64B: 10 dword payload loads", us);
        us = time_it([&] { hipLaunchKernelGGL(small_dwords<7>, grid, blk, 0, 0, desc, pay, frames, n); }, 50);
        printf("%-34s %8.2f us\n", "64B: 7 dword payload loads", us);
        for (uint32_t gq : {1024u, 2048u, 4096u}) {
            us = time_it([&] { hipLaunchKernelGGL(quad_frames, dim3(gq), blk, 0, 0, (const uint4*)desc, pay, frames, n); }, 50);
            printf("64B quad lanes/frame, grid %-5u     %8.2f us\n", gq, us);
        }
    }
    const uint32_t nb = n / 4, flen = 1514, stride = 1516, pstride = 1472;
#define BIG(G, CH, L, S, name)                                                                        \
    {                                                                                                 \
        const dim3 g2(2048);                                                                          \
        float us = time_it([&] { hipLaunchKernelGGL((big_frames<G, CH, L, S>), g2, blk, 0, 0, pay, frames, nb, flen, stride, pstride); }, 30); \
        double bytes = (L ? 1472.0 : 0) * nb + (S ? 1514.0 : 0) * nb;                                 \
        printf("%-34s %8.2f us  %7.1f GB/s\n", name, us, bytes / us / 1e3);                           \
    }
    BIG(32, 3, true, true, "1514B G32: payload in, frame out");
    BIG(32, 3, false, true, "1514B G32: frame out only");
    BIG(32, 3, true, false, "1514B G32: payload in only");
    BIG(16, 6, true, true, "1514B G16: payload in, frame out");
    BIG(8, 12, true, true, "1514B G8: payload in, frame out");
    BIG(64, 2, true, true, "1514B G64: payload in, frame out");
    return 0;
}
