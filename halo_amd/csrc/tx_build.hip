// tx_build.hip — the transmit-construction half of SURVEY.md §8f row f2 on gfx950: one frame per
// descriptor, built exactly as the reference's locally originated send chain builds it:
//   NetIf.TxUdp / TxTcp / TxIcmp        engine/{udp,tcp,icmp}_engine.go
//    -> protocol.BuildUdpPkt            protocol/udp.go:52-91
//       protocol.BuildTcpPkt            protocol/tcp.go:73-123
//       protocol.BuildIcmpPkt           protocol/icmp.go:66-89
//    -> NetIf.TxIpv4                    engine/ipv4_engine.go:50-99 (LoChan copy :72-79)
//       protocol.BuildIpv4Pkt           protocol/ipv4.go:89-131 (iphId++ per packet, :33)
//    -> NetIf.TxEthernet                engine/ethernet_engine.go:34-50
//       protocol.BuildEthFrm            protocol/ethernet.go:58-82 (zero pad to 60 B)
//
// Shape. Blocks take 256-descriptor tiles in order from a ticket counter. Per tile: the
// descriptors are staged in LDS with coalesced 8-byte loads; each thread decides its frame
// (Build* length limits, slot size) and a block scan plus a decoupled look-back over the tiles
// before it gives every built frame its place in the iphId sequence (BuildIpv4Pkt increments the
// process-global counter once per packet that reaches it, so frame k of the batch carries
// base + k). Then G lanes per frame write it: lane j of the group produces 16-byte output chunks
// j, j+G, ..., each dword = header bytes (kept in registers, from the descriptor) | payload bytes
// (two aligned source loads merged with v_alignbyte: the payload may start at any byte) |
// zero padding. The L4 checksum is summed over the output dwords as they are produced (little-
// endian domain, as rx_parse.hip: the L4 segment starts at an even frame offset), reduced over
// the group with DPP, and patched into the header chunks, which are stored last. HBM-bound: each
// payload byte is read once and each frame byte written once.
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "halo_common.h"

namespace halo {
namespace {

constexpr uint32_t kTile = 256;
constexpr uint64_t kFlagAgg = 1ull << 32, kFlagPrefix = 2ull << 32;

struct BuildParams {
    const halo_tx_build_desc_t* desc;
    const uint8_t* payload;
    uint8_t* frames;
    uint16_t* lens;
    uint8_t* result;
    uint16_t* ip_id;
    uint32_t* ws;                 // [0] tile ticket, [1] blocks done; u64 tile status from byte 8
    uint32_t n, n_tiles, flags, stride;
    uint32_t mac_lo, mac_hi;      // the NetIf's MAC (BuildEthFrm srcMac), little-endian packed
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Mask of the bytes of frame dword k that lie in [lo, hi).
__device__ __forceinline__ uint32_t byte_mask(uint32_t k, uint32_t lo, uint32_t hi) {
    const int32_t l = (int32_t)lo - (int32_t)(4 * k), h = (int32_t)hi - (int32_t)(4 * k);
    const uint32_t mh = h >= 4 ? 0xFFFFFFFFu : (h <= 0 ? 0u : (1u << (8 * h)) - 1u);
    const uint32_t ml = l >= 4 ? 0xFFFFFFFFu : (l <= 0 ? 0u : (1u << (8 * l)) - 1u);
    return mh & ~ml;
}

// One descriptor, decoded. Lengths follow the Build* arithmetic.
struct Frame {
    uint64_t pay;          // payload byte address
    uint32_t plen, proto, aux, sport, dport, src, dst, seq, ack, dmac_lo, dmac_hi, mode;
    uint32_t l4hdr, iplen, base, hdr_end, flen;
};

__device__ __forceinline__ Frame decode(const uint32_t* d, const uint8_t* payload) {
    Frame f;
    f.pay = reinterpret_cast<uint64_t>(payload) + ((uint64_t)d[0] | ((uint64_t)d[1] << 32));
    f.plen = d[2] & 0xFFFFu;
    f.proto = (d[2] >> 16) & 0xFFu;
    f.aux = d[2] >> 24;
    f.sport = d[3] & 0xFFFFu;
    f.dport = d[3] >> 16;
    f.src = d[4]; f.dst = d[5]; f.seq = d[6]; f.ack = d[7];
    f.dmac_lo = d[8];
    f.dmac_hi = d[9] & 0xFFFFu;
    f.mode = (d[9] >> 16) & 0xFFu;
    f.l4hdr = f.proto == kIpTcp ? 20u : 8u;
    f.iplen = 20u + f.l4hdr + f.plen;
    f.base = f.mode == HALO_TX_BUILD_LOOPBACK ? 0u : 14u;
    f.hdr_end = f.base + 20u + f.l4hdr;
    f.flen = f.mode == HALO_TX_BUILD_LOOPBACK ? f.iplen : (f.iplen + 14u < 60u ? 60u : f.iplen + 14u);
    return f;
}

// HALO_TX_B_* of a descriptor, decided before Build* runs (the slot check is build-defined).
__device__ __forceinline__ uint32_t verdict(const Frame& f, uint32_t stride) {
    if (f.proto != kIpUdp && f.proto != kIpTcp && f.proto != kIpIcmp) return HALO_TX_B_PROTO;
    if (f.plen > (f.proto == kIpTcp ? 1460u : 1472u)) return HALO_TX_B_PAYLOAD_LEN;  // udp.go:55 tcp.go:78 icmp.go:71
    if (f.flen > stride) return HALO_TX_B_SLOT;
    return HALO_TX_B_OK;
}

// Header dword k (0..13) of the Ethernet layout, payload bytes zero, L4 checksum field zero.
// e[] is filled once per frame; the loopback layout is the same bytes shifted by 14.
__device__ __forceinline__ void eth_header(const Frame& f, uint32_t id, uint32_t ipck, const BuildParams& p,
                                           uint32_t (&e)[18]) {
    const uint32_t s = bswap32(f.src), t = bswap32(f.dst);
    e[0] = f.dmac_lo;
    e[1] = f.dmac_hi | ((p.mac_lo & 0xFFFFu) << 16);
    e[2] = (p.mac_lo >> 16) | (p.mac_hi << 16);
    e[3] = 0x00450008u;                                       // EtherType 0x0800, 0x45, TOS 0
    e[4] = bswap16(f.iplen) | (bswap16(id) << 16);            // totalLen, identification
    e[5] = (0x80u << 16) | (f.proto << 24);                   // flags/offset 0, TTL 0x80, proto
    e[6] = bswap16(ipck) | ((s & 0xFFFFu) << 16);
    e[7] = (s >> 16) | ((t & 0xFFFFu) << 16);
    e[8] = t >> 16;
    e[9] = e[10] = e[11] = e[12] = e[13] = e[14] = e[15] = e[16] = e[17] = 0u;
    if (f.proto == kIpUdp) {                                   // udp.go:60-67
        e[8] |= bswap16(f.sport) << 16;
        e[9] = bswap16(f.dport) | (bswap16(f.l4hdr + f.plen) << 16);
    } else if (f.proto == kIpTcp) {                            // tcp.go:88-104
        const uint32_t q = bswap32(f.seq), a = bswap32(f.ack);
        e[8] |= bswap16(f.sport) << 16;
        e[9] = bswap16(f.dport) | ((q & 0xFFFFu) << 16);
        e[10] = (q >> 16) | ((a & 0xFFFFu) << 16);
        e[11] = (a >> 16) | (0x50u << 16) | (f.aux << 24);
        e[12] = 0x0001u;                                       // window 256
    } else {                                                   // icmp.go:75-82
        e[8] |= f.aux << 16;
        e[9] = bswap16(f.sport) << 16;                         // icmpId bytes
        e[10] = bswap16(f.dport);                              // icmpSeq
    }
}

// BuildIpv4Pkt's header checksum (ipv4.go:121-128), big-endian value; 0 when disabled.
__device__ __forceinline__ uint32_t ipv4_cksum(const Frame& f, uint32_t id, bool csum) {
    if (!csum) return 0u;
    uint32_t s = 0x4500u + f.iplen + id + ((0x80u << 8) | f.proto);
    s += (f.src >> 16) + (f.src & 0xFFFFu) + (f.dst >> 16) + (f.dst & 0xFFFFu);
    return (~fold16(s)) & 0xFFFFu;
}

// Payload bytes of output dwords [4c, 4c+4): source bytes [16c - hdr_end, +16) of the payload,
// never reading a dword that holds no payload byte (the caller masks what is not payload).
__device__ __forceinline__ void payload_chunk(const Frame& f, uint32_t c, uint32_t (&w)[4]) {
    const int64_t rel = (int64_t)(16 * c) - (int64_t)f.hdr_end;  // payload offset of the chunk's first byte
    const uint64_t a0 = f.pay + rel;                                // may lie before the payload
    const uint64_t A = a0 & ~3ull;
    const uint32_t sh = (uint32_t)(a0 & 3u);
    const uint64_t lo = f.pay & ~3ull, hi = (f.pay + f.plen + 3) & ~3ull;  // readable dwords [lo, hi)
    uint32_t s[5];
    typedef const __attribute__((address_space(1))) uint32_t gu32_t;
    gu32_t* q = (gu32_t*)A;
    if (A >= lo && A + 20 <= hi) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
        const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)q;
        s[0] = v.x; s[1] = v.y; s[2] = v.z; s[3] = v.w;
        s[4] = q[4];
    } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const uint64_t x = A + 4u * i;
            s[i] = (x >= lo && x < hi) ? q[i] : 0u;
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = __builtin_amdgcn_alignbyte(s[i + 1], s[i], sh);
}

// The frame of descriptor f, lane j of its G-lane group. Chunks 0..3 (bytes 0..63, which hold
// every header byte and both checksum fields) are stored after the group's L4 sum is known.
template <int G>
__device__ __forceinline__ void build_frame(const BuildParams& p, const Frame& f, uint32_t id, uint32_t j,
                                            uint8_t* out) {
    const bool csum = (p.flags & HALO_RX_CSUM_ENABLE) != 0;
    const bool l3 = f.mode == HALO_TX_BUILD_LOOPBACK;
    uint32_t e[18];
    eth_header(f, id, ipv4_cksum(f, id, csum), p, e);
    const uint32_t l4s = f.base + 20u, l4e = f.base + f.iplen, pay_end = f.hdr_end + f.plen;
    const uint32_t ndw = (f.flen + 3u) >> 2;  // output dwords (the last one zero-filled past the frame)
    // frame-layout header dword k (0..15): Ethernet as built, loopback = the same bytes from 14 on
    auto hdr = [&](uint32_t k) -> uint32_t {
        uint32_t v = 0;
#pragma unroll
        for (uint32_t m = 0; m < 14; ++m) {
            const uint32_t ev = l3 ? ((e[m + 3] >> 16) | (e[m + 4] << 16)) : e[m];
            v = (k == m) ? ev : v;
        }
        return v;
    };
    constexpr int kDefer = G >= 4 ? 1 : 4;  // header chunks this lane keeps until the sum is known
    uint32_t keep[kDefer][4];
    uint64_t sum = 0;
    for (uint32_t c = j, r = 0; 4 * c < ndw; c += G, ++r) {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        if (16 * c + 16 > f.hdr_end && 16 * c < pay_end && f.plen) payload_chunk(f, c, w);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t k = 4 * c + i;
            w[i] &= byte_mask(k, f.hdr_end, pay_end);
            if (k < 16) w[i] |= hdr(k) & byte_mask(k, 0, f.hdr_end);
            sum += w[i] & byte_mask(k, l4s, l4e);
        }
        if (c < 4) {
            if constexpr (kDefer == 4) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (q == (int)c)
#pragma unroll
                        for (int i = 0; i < 4; ++i) keep[q][i] = w[i];
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) keep[0][i] = w[i];
            }
            continue;
        }
        uint32_t* o = reinterpret_cast<uint32_t*>(out) + 4 * c;
        if (4 * c + 4 <= ndw) {
            *reinterpret_cast<uint4*>(o) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (4 * c + i < ndw) o[i] = w[i];
        }
    }
    // L4 checksum: pseudo header (UDP / TCP) + the segment, one's-complement, LE domain
    uint32_t part = fold64(sum);
    part = group_sum<G>(part);
    uint32_t ck_le = 0;  // the field's two bytes as a little-endian half-word
    uint32_t ck_at;      // frame byte offset of the L4 checksum field
    const bool fill = csum || f.proto == kIpIcmp;
    if (f.proto == kIpUdp || f.proto == kIpTcp) {
        const uint32_t s = bswap32(f.src), t = bswap32(f.dst);
        part += hsum(s) + hsum(t) + (f.proto << 8) + bswap16(f.l4hdr + f.plen);
        ck_at = f.base + 20u + (f.proto == kIpUdp ? 6u : 16u);
    } else {
        ck_at = f.base + 22u;
    }
    if (fill) ck_le = (~fold16(part)) & 0xFFFFu;
    const uint32_t ck_dw = ck_at >> 2, ck_sh = (ck_at & 2u) * 8u;
#pragma unroll
    for (int q = 0; q < kDefer; ++q) {
        const uint32_t c = kDefer == 4 ? (uint32_t)q : j;
        if (c >= 4 || 4 * c >= ndw) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (4 * c + i == ck_dw) keep[q][i] |= ck_le << ck_sh;
        uint32_t* o = reinterpret_cast<uint32_t*>(out) + 4 * c;
        if (4 * c + 4 <= ndw) {
            *reinterpret_cast<uint4*>(o) = make_uint4(keep[q][0], keep[q][1], keep[q][2], keep[q][3]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (4 * c + i < ndw) o[i] = keep[q][i];
        }
    }
}

__device__ __forceinline__ uint64_t status_load(const uint64_t* s) {
    return __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void status_store(uint64_t* s, uint64_t v) {
    __hip_atomic_store(s, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int G>
__global__ void __launch_bounds__(256) tx_build_kernel(const BuildParams p) {
    __shared__ uint32_t s_desc[kTile * 10];
    __shared__ uint32_t s_meta[kTile];     // bit 31 built, bits 0..15 iphId
    __shared__ uint32_t s_wave[4];
    __shared__ uint32_t s_tile, s_excl, s_base, s_last;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint64_t* status = reinterpret_cast<uint64_t*>(p.ws + 2);
    if (tid == 0) s_base = *p.ip_id;  // read before any ticket: the last block rewrites it at the end
    for (;;) {
        if (tid == 0) s_tile = atomicAdd(&p.ws[0], 1u);
        __syncthreads();
        const uint32_t tile = s_tile;
        if (tile >= p.n_tiles) break;
        const uint32_t first = tile * kTile;
        const uint32_t cnt = min(kTile, p.n - first);
        // stage the tile's descriptors (40 B each) with coalesced 8-byte loads
        const uint2* src = reinterpret_cast<const uint2*>(p.desc + first);
        for (uint32_t q = tid; q < 5 * cnt; q += kTile) {
            const uint2 v = src[q];
            s_desc[2 * q] = v.x;
            s_desc[2 * q + 1] = v.y;
        }
        __syncthreads();
        // each thread's descriptor: build or not, and its rank among the tile's built frames
        uint32_t code = HALO_TX_B_PROTO, flen = 0;
        if (tid < cnt) {
            const Frame f = decode(&s_desc[10 * tid], p.payload);
            code = verdict(f, p.stride);
            flen = f.flen;
        }
        const bool ok = tid < cnt && code == HALO_TX_B_OK;
        const uint64_t bal = __ballot(ok);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (lane == 0) s_wave[wave] = __popcll(bal);
        __syncthreads();
        uint32_t before = 0, total = 0;
#pragma unroll
        for (uint32_t w = 0; w < 4; ++w) {
            before += w < wave ? s_wave[w] : 0u;
            total += s_wave[w];
        }
        // decoupled look-back: the number of frames built in all tiles before this one
        if (wave == 0) {
            if (lane == 0) status_store(&status[tile], (tile == 0 ? kFlagPrefix : kFlagAgg) | total);
            uint32_t excl = 0;
            if (tile > 0) {
                int64_t j = (int64_t)tile - 1;
                for (;;) {
                    const int64_t idx = j - (int64_t)lane;
                    uint64_t v = idx >= 0 ? status_load(&status[idx]) : kFlagPrefix;
                    const uint64_t pre = __ballot((v >> 32) == 2u);
                    const uint32_t lim = pre ? (uint32_t)__builtin_ctzll(pre) : 63u;  // lanes 0..lim count
                    const uint64_t zero = __ballot((v >> 32) == 0u);
                    if (zero & ((lim == 63u) ? ~0ull : ((2ull << lim) - 1ull))) continue;  // not published yet
                    uint32_t x = lane <= lim ? (uint32_t)v : 0u;
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o, 64);
                    excl += x;
                    if (pre) break;
                    j -= 64;
                }
                if (lane == 0) status_store(&status[tile], kFlagPrefix | (excl + total));
            }
            if (lane == 0) s_excl = excl;
        }
        __syncthreads();
        const uint32_t id = (s_base + s_excl + before + rank + 1u) & 0xFFFFu;  // iphId++ then use
        if (tid < cnt) {
            s_meta[tid] = (ok ? 0x80000000u : 0u) | id;
            p.lens[first + tid] = ok ? (uint16_t)flen : (uint16_t)0;
            if (p.result) p.result[first + tid] = (uint8_t)code;
        }
        __syncthreads();
        // build: G lanes per frame, 256 / G frames per round
        constexpr uint32_t kPer = kTile / G;
        const uint32_t g = tid / G, jl = tid % G;
#pragma unroll 1
        for (uint32_t r = 0; r < (uint32_t)G; ++r) {
            const uint32_t fi = r * kPer + g;
            if (fi < cnt && (s_meta[fi] >> 31)) {  // uniform over the group
                const Frame f = decode(&s_desc[10 * fi], p.payload);
                build_frame<G>(p, f, s_meta[fi] & 0xFFFFu, jl, p.frames + (uint64_t)(first + fi) * p.stride);
            }
        }
        __syncthreads();  // LDS is reused by the next tile
    }
    // the last block out publishes the new iphId and leaves the workspace zeroed for the next launch
    if (tid == 0) {
        __threadfence();
        s_last = atomicAdd(&p.ws[1], 1u) == gridDim.x - 1u;
    }
    __syncthreads();
    if (s_last) {
        __threadfence();
        if (tid == 0) *p.ip_id = (uint16_t)(s_base + (uint32_t)status_load(&status[p.n_tiles - 1]));
        __syncthreads();
        for (uint32_t t = tid; t < p.n_tiles; t += kTile) status_store(&status[t], 0ull);
        __syncthreads();
        if (tid == 0) {
            p.ws[0] = 0u;
            p.ws[1] = 0u;
            __threadfence();
        }
    }
}

}  // namespace
}  // namespace halo

extern "C" HALO_API uint64_t halo_tx_build_workspace(uint32_t n) {
    return 8ull + 8ull * (((uint64_t)n + halo::kTile - 1) / halo::kTile);
}

extern "C" HALO_API int halo_tx_build_batch_device(const halo_tx_build_desc_t* d_desc, uint32_t n,
                                                   const uint8_t* d_payload, uint32_t flags,
                                                   const halo_rx_netif_t* netif, uint32_t max_payload_hint,
                                                   uint8_t* d_frames, uint32_t out_stride, uint16_t* d_out_lens,
                                                   uint8_t* d_result, uint16_t* d_ip_id, void* d_workspace,
                                                   uint64_t workspace_bytes, halo_stream_t stream) {
    if (!netif || (flags & ~HALO_RX_CSUM_ENABLE)) return HALO_E_INVAL;
    if (n == 0) return HALO_OK;
    if (!d_desc || !d_payload || !d_frames || !d_out_lens || !d_ip_id || !d_workspace) return HALO_E_INVAL;
    if ((out_stride & 3u) || out_stride < 60u) return HALO_E_INVAL;
    if ((reinterpret_cast<uintptr_t>(d_desc) & 7u) || (reinterpret_cast<uintptr_t>(d_frames) & 3u) ||
        (reinterpret_cast<uintptr_t>(d_workspace) & 7u) || (reinterpret_cast<uintptr_t>(d_ip_id) & 1u))
        return HALO_E_INVAL;
    if (workspace_bytes < halo_tx_build_workspace(n)) return HALO_E_INVAL;
    int rc = halo::check_device();
    if (rc) return rc;
    halo::BuildParams p{};
    p.desc = d_desc;
    p.payload = d_payload;
    p.frames = d_frames;
    p.lens = d_out_lens;
    p.result = d_result;
    p.ip_id = d_ip_id;
    p.ws = static_cast<uint32_t*>(d_workspace);
    p.n = n;
    p.n_tiles = (n + halo::kTile - 1) / halo::kTile;
    p.flags = flags;
    p.stride = out_stride;
    p.mac_lo = (uint32_t)netif->mac[0] | ((uint32_t)netif->mac[1] << 8) | ((uint32_t)netif->mac[2] << 16) |
               ((uint32_t)netif->mac[3] << 24);
    p.mac_hi = (uint32_t)netif->mac[4] | ((uint32_t)netif->mac[5] << 8);
    // blocks loop over tiles; 8 resident 256-thread blocks per CU on 256 CUs
    const uint32_t grid = p.n_tiles < 2048u ? p.n_tiles : 2048u;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint32_t h = max_payload_hint ? max_payload_hint : 1472u;
    if (h + 54u <= 128u) hipLaunchKernelGGL(halo::tx_build_kernel<1>, dim3(grid), dim3(256), 0, s, p);
    else if (h + 54u <= 1024u) hipLaunchKernelGGL(halo::tx_build_kernel<4>, dim3(grid), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(halo::tx_build_kernel<8>, dim3(grid), dim3(256), 0, s, p);
    return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
}
