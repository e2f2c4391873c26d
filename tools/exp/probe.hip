// probe.hip — memory-pattern probes for the 64 B-frame hot path (tools only, not shipped).
// Build: hipcc --offload-arch=gfx950 -O3 -o probe tools/exp/probe.hip ; run on the GPU box.
// Every probe moves the config-2 byte volume: 1M frames x 64 B read (+ metadata, + 32 B records
// written), over 8 rotating batches so the working set exceeds the Infinity Cache.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

constexpr uint32_t N = 1u << 20, FB = 64;

// coalesced: lane l of a wave reads 16 B at wave_base + 16 l (1 KB per wave-instruction)
__global__ void __launch_bounds__(256) p_coalesced(const uint4* __restrict__ in, uint32_t* __restrict__ out, uint32_t n16) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s = 0;
    for (; i < n16; i += gridDim.x * blockDim.x) {
        uint4 v = in[i];
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x12345678u) out[0] = s;
}

// lane per frame: 4 x 16 B loads of the lane's own 64 B frame, then a 32 B record per lane
template <bool META, bool WRITE>
__global__ void __launch_bounds__(256) p_lane(const uint8_t* __restrict__ bytes, const uint32_t* __restrict__ off,
                                              const uint16_t* __restrict__ lens, uint4* __restrict__ rec, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* f = bytes + (META ? ((uint64_t)off[i] << 2) : (uint64_t)i * FB);
    uint32_t L = META ? lens[i] : FB;
    const uint4* q = reinterpret_cast<const uint4*>(f);
    uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    uint32_t s = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w + c.x + c.y + c.z + c.w + d.x + d.y + d.z + d.w + L;
    if (WRITE) {
        rec[2 * i] = make_uint4(s, a.x, b.y, c.z);
        rec[2 * i + 1] = make_uint4(d.w, s ^ 1, s ^ 2, s ^ 3);
    } else if (s == 0x12345678u) {
        rec[0] = a;
    }
}

// lane per frame, two frames per lane (8 loads in flight per lane)
__global__ void __launch_bounds__(256) p_lane2(const uint8_t* __restrict__ bytes, const uint32_t* __restrict__ off,
                                               uint4* __restrict__ rec, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t j = i + (gridDim.x * blockDim.x);
    if (i >= n) return;
    const uint4* q = reinterpret_cast<const uint4*>(bytes + ((uint64_t)off[i] << 2));
    const uint4* r = reinterpret_cast<const uint4*>(bytes + ((uint64_t)off[j < n ? j : i] << 2));
    uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    uint4 e = r[0], f = r[1], g = r[2], h = r[3];
    uint32_t s = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w + c.x + c.y + c.z + c.w + d.x + d.y + d.z + d.w;
    uint32_t t = e.x + e.y + e.z + e.w + f.x + f.y + f.z + f.w + g.x + g.y + g.z + g.w + h.x + h.y + h.z + h.w;
    rec[2 * i] = make_uint4(s, a.x, b.y, c.z);
    rec[2 * i + 1] = make_uint4(d.w, s ^ 1, s ^ 2, s ^ 3);
    if (j < n) {
        rec[2 * j] = make_uint4(t, e.x, f.y, g.z);
        rec[2 * j + 1] = make_uint4(h.w, t ^ 1, t ^ 2, t ^ 3);
    }
}

// coalesced load + LDS transpose to lane-per-frame: a wave loads 64 frames (4 KB) with 4
// fully coalesced 1 KB instructions, stages them in LDS (80 B padded rows), each lane reads
// its own frame back
__global__ void __launch_bounds__(256) p_lds(const uint8_t* __restrict__ bytes, const uint32_t* __restrict__ off,
                                             uint4* __restrict__ rec, uint32_t n) {
    __shared__ uint4 lds[4][64 * 5];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t base = (blockIdx.x * blockDim.x + threadIdx.x) & ~63u;
    if (base >= n) return;
    // instruction k: lanes 4g..4g+3 load frame (16k + g)'s chunks 0..3
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t fr = base + 16 * k + (lane >> 2);
        const uint4* q = reinterpret_cast<const uint4*>(bytes + ((uint64_t)off[fr] << 2));
        v[k] = q[lane & 3];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) lds[w][(16 * k + (lane >> 2)) * 5 + (lane & 3)] = v[k];
    __builtin_amdgcn_wave_barrier();
    uint4 a = lds[w][lane * 5 + 0], b = lds[w][lane * 5 + 1], c = lds[w][lane * 5 + 2], d = lds[w][lane * 5 + 3];
    uint32_t s = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w + c.x + c.y + c.z + c.w + d.x + d.y + d.z + d.w;
    const uint32_t i = base + lane;
    rec[2 * i] = make_uint4(s, a.x, b.y, c.z);
    rec[2 * i + 1] = make_uint4(d.w, s ^ 1, s ^ 2, s ^ 3);
}

// record-store shapes (no reads): lane-strided 2 x 16 B (the kernel's), LDS-transposed fully
// coalesced 16 B per lane, and non-temporal lane-strided
template <int MODE>
__global__ void __launch_bounds__(256) p_store(uint4* __restrict__ rec, uint32_t n) {
    __shared__ uint4 lds[4][128];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 lo = make_uint4(i, i ^ 1, i ^ 2, i ^ 3), hi = make_uint4(i ^ 4, i ^ 5, i ^ 6, i ^ 7);
    if (MODE == 0) {
        rec[2 * i] = lo;
        rec[2 * i + 1] = hi;
    } else if (MODE == 1) {
        const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, base = i - lane;
        lds[w][2 * lane] = lo;
        lds[w][2 * lane + 1] = hi;
        __builtin_amdgcn_wave_barrier();
        rec[2 * base + lane] = lds[w][lane];
        rec[2 * base + 64 + lane] = lds[w][64 + lane];
    } else {
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        v4* r = reinterpret_cast<v4*>(rec);
        __builtin_nontemporal_store((v4){lo.x, lo.y, lo.z, lo.w}, &r[2 * i]);
        __builtin_nontemporal_store((v4){hi.x, hi.y, hi.z, hi.w}, &r[2 * i + 1]);
    }
}

int main() {
    const int R = 8, K = 40;
    std::vector<uint8_t*> bytes(R);
    std::vector<uint32_t*> offs(R);
    std::vector<uint16_t*> lens(R);
    uint4* rec;
    uint32_t* sink;
    std::vector<uint32_t> h_off(N);
    std::vector<uint16_t> h_len(N, FB);
    for (uint32_t i = 0; i < N; ++i) h_off[i] = i * (FB / 4);
    for (int r = 0; r < R; ++r) {
        CK(hipMalloc(&bytes[r], (size_t)N * FB));
        CK(hipMemset(bytes[r], r + 1, (size_t)N * FB));
        CK(hipMalloc(&offs[r], N * 4));
        CK(hipMalloc(&lens[r], N * 2));
        CK(hipMemcpy(offs[r], h_off.data(), N * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(lens[r], h_len.data(), N * 2, hipMemcpyHostToDevice));
    }
    CK(hipMalloc(&rec, (size_t)N * 32));
    CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, double mb, auto launch) {
        for (int k = 0; k < 5; ++k) launch(k % R);
        CK(hipDeviceSynchronize());
        float tot = 0;
        for (int k = 0; k < K; ++k) {
            CK(hipEventRecord(e0));
            launch(k % R);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        const double us = tot / K * 1e3;
        printf("%-40s %8.2f us  %8.1f GB/s\n", name, us, mb * 1e6 / us / 1e3);
    };
    const double fr_mb = N * (double)FB / 1e6, rec_mb = N * 32.0 / 1e6, meta_mb = N * 6.0 / 1e6;
    for (int rep = 0; rep < 2; ++rep) {
        run("store 32 MB records, lane-strided 2x16B", rec_mb, [&](int r) {
            (void)r;
            hipLaunchKernelGGL((p_store<0>), dim3(N / 256), dim3(256), 0, 0, rec, N);
        });
        run("store 32 MB records, LDS-transposed", rec_mb, [&](int r) {
            (void)r;
            hipLaunchKernelGGL((p_store<1>), dim3(N / 256), dim3(256), 0, 0, rec, N);
        });
        run("store 32 MB records, nontemporal", rec_mb, [&](int r) {
            (void)r;
            hipLaunchKernelGGL((p_store<2>), dim3(N / 256), dim3(256), 0, 0, rec, N);
        });
        run("coalesced read 64 MB", fr_mb, [&](int r) {
            hipLaunchKernelGGL(p_coalesced, dim3(N * FB / 16 / 256), dim3(256), 0, 0, (const uint4*)bytes[r], sink,
                               N * FB / 16);
        });
        run("coalesced read, grid 4096", fr_mb, [&](int r) {
            hipLaunchKernelGGL(p_coalesced, dim3(4096), dim3(256), 0, 0, (const uint4*)bytes[r], sink, N * FB / 16);
        });
        run("lane/frame read only (no meta)", fr_mb, [&](int r) {
            hipLaunchKernelGGL((p_lane<false, false>), dim3(N / 256), dim3(256), 0, 0, bytes[r], offs[r], lens[r], rec, N);
        });
        run("lane/frame read + 32B rec (no meta)", fr_mb + rec_mb, [&](int r) {
            hipLaunchKernelGGL((p_lane<false, true>), dim3(N / 256), dim3(256), 0, 0, bytes[r], offs[r], lens[r], rec, N);
        });
        run("lane/frame meta + read + rec", fr_mb + rec_mb + meta_mb, [&](int r) {
            hipLaunchKernelGGL((p_lane<true, true>), dim3(N / 256), dim3(256), 0, 0, bytes[r], offs[r], lens[r], rec, N);
        });
        run("lane/frame x2 per lane, meta + rec", fr_mb + rec_mb + 4e-6 * N, [&](int r) {
            hipLaunchKernelGGL(p_lane2, dim3(N / 512), dim3(256), 0, 0, bytes[r], offs[r], rec, N);
        });
        run("coalesced + LDS transpose + rec", fr_mb + rec_mb + 4e-6 * N, [&](int r) {
            hipLaunchKernelGGL(p_lds, dim3(N / 256), dim3(256), 0, 0, bytes[r], offs[r], rec, N);
        });
    }
    return 0;
}
