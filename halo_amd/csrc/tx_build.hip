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
// iphId. BuildIpv4Pkt increments the process-global counter once per packet that reaches it, so
// the k-th built frame of the batch carries base + k. A descriptor that Build* rejects is rare
// (a caller error), so frame i is built with base + 1 + i - (rejected descriptors before it in
// its own 64-descriptor tile) — everything its wave knows — and the rejections in earlier tiles
// are settled afterwards by one more launch: it writes the new iphId and, only when a tile marked
// a rejection, patches the identification and header checksum of the frames behind it (RFC 1624).
// No atomics and no inter-block waiting anywhere: a ticketed single pass with a decoupled
// look-back measured 175 us for 1M 64 B frames (its ticket atomics serialise at ~25 ns each: 4096
// tickets alone cost 100 us).
//
// Build. Each wave owns 64-descriptor tiles (grid-stride): lane i loads descriptor i, decides it
// (Build* length limits, slot size), ranks the rejections with a ballot and writes its frame's
// header dwords 0..15 (Ethernet layout, or the loopback packet's) to the wave's LDS region. Then
// G lanes per frame (64 / G frames at a time) produce 16-byte output chunks j, j+G, ..., U per
// memory round trip, each dword = header bytes | payload bytes (two aligned source loads merged
// with v_alignbyte: the payload may start at any byte) | zero padding. The L4 checksum is summed
// over the output dwords as they are produced (v_dot2_u32_u16 of each dword's halves: the
// one's-complement sum in the little-endian domain, as rx_parse.hip; the L4 segment starts at an
// even frame offset), reduced over the group with DPP, and patched into the header chunks, which
// are stored last. Chunks wholly inside the payload skip every mask; a lane-per-frame frame of
// <= 64 B is built whole in registers with no per-dword branch (build_small), staged in LDS and
// stored by the wave four lanes per frame: lane-per-frame stores (one instruction touching 64
// separate slots) cost more than all the rest of the 64 B build (tools/exp/probe_txb.hip,
// DESIGN.md §10.5).
#include <hip/hip_runtime.h>

#include <atomic>
#include <type_traits>

#include "device_util.h"
#include "halo_common.h"

namespace halo {
namespace {

constexpr uint32_t kTile = 64;    // descriptors per tile = one wave's
constexpr uint32_t kBlock = 256;  // threads per block of the build launch

struct BuildParams {
    const halo_tx_build_desc_t* desc;
    const uint8_t* payload;
    uint8_t* frames;
    uint16_t* lens;
    uint8_t* result;
    uint16_t* ip_id;
    uint32_t* ws;                 // [0] the seq of the last launch that saw a rejection, [1 + t] tile t's rejections
    uint32_t n, n_tiles, flags, stride;
    uint32_t mac_lo, mac_hi;      // the NetIf's MAC (BuildEthFrm srcMac), little-endian packed
    uint32_t seq;                 // this launch's sequence number (ws[0] = seq: a tile saw a rejection)
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

// Source dwords for output chunk c (payload bytes [16c - hdr_end, +16) of the frame): five
// aligned dwords, never reading one that holds no payload byte (zeros instead). Issued early;
// merge_chunk turns them into the chunk once they arrive.
__device__ __forceinline__ void payload_raw(const Frame& f, uint32_t c, uint32_t (&s)[5]) {
    const int64_t rel = (int64_t)(16 * c) - (int64_t)f.hdr_end;  // payload offset of the chunk's first byte
    const uint64_t A = (f.pay + rel) & ~3ull;                       // may lie before the payload
    const uint64_t lo = f.pay & ~3ull, hi = (f.pay + f.plen + 3) & ~3ull;  // readable dwords [lo, hi)
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
}

__device__ __forceinline__ bool chunk_has_payload(const Frame& f, uint32_t c, uint32_t ndw) {
    return 4 * c < ndw && 16 * c + 16 > f.hdr_end && 16 * c < f.hdr_end + f.plen && f.plen;
}

// Sum of the four bytes pairs of a dword as 16-bit halves (one v_dot2_u32_u16): the one's-
// complement sum in the little-endian domain accumulates per dword in u32 without overflow for
// any frame here (<= 2 * 65535 per dword).
__device__ __forceinline__ uint32_t hsum_acc(uint32_t w, uint32_t acc) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 one = {1, 1};
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w), one, acc, false);
}

// The frame of descriptor f on lane j of its G-lane group: chunks j, j+G, ... (U per memory
// round trip, all loads of a round issued before any is used) merged, masked, summed and stored;
// then the L4 checksum over the group and the header chunks 0..3 (which hold both checksum
// fields), stored last.
template <int G, int U>
__device__ __forceinline__ void build_frame(const BuildParams& p, const Frame& f, const uint32_t* hdr, uint32_t j,
                                            uint8_t* out) {
    const bool csum = (p.flags & HALO_RX_CSUM_ENABLE) != 0;
    const uint32_t l4s = f.base + 20u, pay_end = f.hdr_end + f.plen;  // the packet ends at pay_end
    const uint32_t ndw = (f.flen + 3u) >> 2;  // output dwords (the last one zero-filled past the frame)
    const uint32_t sh = (uint32_t)((f.pay - f.hdr_end) & 3u);  // source misalignment, every chunk
    constexpr int kDefer = G >= 4 ? 1 : 4;  // header chunks this lane keeps until the sum is known
    uint32_t keep[kDefer][4];
    uint32_t sum = 0;
    // a chunk of frame bytes [16c, 16c+16): header bytes, payload, zero padding; its L4-segment
    // bytes summed
    auto edge = [&](uint32_t c, uint32_t (&w)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t k = 4 * c + i;
            w[i] &= byte_mask(k, f.hdr_end, pay_end);
            if (k < 16) w[i] |= hdr[k] & byte_mask(k, 0, f.hdr_end);
            sum = hsum_acc(w[i] & byte_mask(k, l4s, pay_end), sum);
        }
    };
    auto store = [&](uint32_t c, const uint32_t (&w)[4]) {
        uint32_t* o = reinterpret_cast<uint32_t*>(out) + 4 * c;
        if (4 * c + 4 <= ndw) {
            *reinterpret_cast<uint4*>(o) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (4 * c + i < ndw) o[i] = w[i];
        }
    };
    // Groups (G >= 4) visit the chunks in the order 4, 5, ..., C-1, 0, 1, 2, 3 (C = the frame's
    // chunks): the header chunks and the frame's last, partial chunk — the only ones taking the
    // masked path — then sit next to each other in one row of U * G, so the other rows of the round
    // run the unmasked path on every lane (a row with one masked lane runs both paths). 1514 B
    // frames: one masked row per frame instead of two.
    const uint32_t nch = (ndw + 3u) >> 2;
    auto chunk_of = [&](uint32_t v) -> uint32_t {
        if constexpr (G >= 4) return nch <= 4u ? v : v + 4u < nch ? v + 4u : v + 4u - nch;  // (a LoChan packet can be < 64 B)
        return v;
    };
    uint32_t kc = 4;  // the header chunk this lane keeps (G >= 4: at most one), 4 = none
    for (uint32_t c0 = j; 4 * c0 < ndw; c0 += U * G) {
        uint32_t raw[U][5];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = chunk_of(c0 + u * G);
            if (c0 + u * G < nch && chunk_has_payload(f, c, ndw)) payload_raw(f, c, raw[u]);
            else raw[u][0] = raw[u][1] = raw[u][2] = raw[u][3] = raw[u][4] = 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (c0 + u * G >= nch) break;
            const uint32_t c = chunk_of(c0 + u * G);
            uint32_t w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) w[i] = __builtin_amdgcn_alignbyte(raw[u][i + 1], raw[u][i], sh);
            if (c >= 4 && 16 * c >= f.hdr_end && 16 * c + 16 <= pay_end) {  // payload throughout
#pragma unroll
                for (int i = 0; i < 4; ++i) sum = hsum_acc(w[i], sum);
                store(c, w);
                continue;
            }
            edge(c, w);
            if (c < 4) {  // a header chunk: stored once the checksum is in
                if constexpr (kDefer == 4) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (q == (int)c)
#pragma unroll
                            for (int i = 0; i < 4; ++i) keep[q][i] = w[i];
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i) keep[0][i] = w[i];
                    kc = c;
                }
            } else {
                store(c, w);
            }
        }
    }
    // L4 checksum: pseudo header (UDP / TCP) + the segment, one's-complement, LE domain
    uint32_t part = group_sum<G>(fold16(sum));
    uint32_t ck_le = 0;  // the field's two bytes as a little-endian half-word
    uint32_t ck_at;      // frame byte offset of the L4 checksum field
    if (f.proto == kIpUdp || f.proto == kIpTcp) {
        const uint32_t s = bswap32(f.src), t = bswap32(f.dst);
        part += hsum(s) + hsum(t) + (f.proto << 8) + bswap16(f.l4hdr + f.plen);
        ck_at = f.base + 20u + (f.proto == kIpUdp ? 6u : 16u);
    } else {
        ck_at = f.base + 22u;
    }
    if (csum || f.proto == kIpIcmp) ck_le = (~fold16(part)) & 0xFFFFu;  // ICMP always (icmp.go:84-87)
    const uint32_t ck_dw = ck_at >> 2, ck_sh = (ck_at & 2u) * 8u;
#pragma unroll
    for (int q = 0; q < kDefer; ++q) {
        const uint32_t c = kDefer == 4 ? (uint32_t)q : kc;
        if (c >= 4 || 4 * c >= ndw) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (4 * c + i == ck_dw) keep[q][i] |= ck_le << ck_sh;
        store(c, keep[q]);
    }
}

// Frames built by 16 or more lanes (the 1514 B build; VERDICT r3: 0.46 of 8 TB/s at 15k VALU per
// wave). build_frame runs every chunk through the general path — chunk remapping, payload and frame
// bounds, byte masks — which the compiler turns into ~170 branchy blocks. Here the frame is three
// zones. Body: chunks 4 .. pay_end/16 - 1 are payload bytes only (the header ends by byte 54), so a
// lane loads each as one 16-byte load plus, when the payload is not 4-byte aligned relative to the
// frame, the next dword (every byte of both is a payload byte the chunk needs), merges it with four
// v_alignbyte, sums it with four v_dot2 and stores it: no masks, no bounds, 32-bit chunk indices.
// Head: chunks 0..3 (header | payload, both checksum fields) on lanes 0..3, and the last, partial
// chunk on lane 4, through the masked path; the head chunks are stored once the L4 sum is known.
#ifndef HALO_TXB_BIG_PATH
#define HALO_TXB_BIG_PATH 1
#endif
#ifndef HALO_TXB_HEAD_EARLY  // build_big: the head / tail chunk loads issued with the body's
#define HALO_TXB_HEAD_EARLY 0  // neutral: 0.194 / 0.195 against 0.190 / 0.195 ms (profiles/r04/r4z)
#endif
#ifndef HALO_TXB_BIG_NB  // a chunk's fifth source dword from the neighbour lane (ds_bpermute)
#define HALO_TXB_BIG_NB 1
#endif
#ifndef HALO_TXB_BIG_UNALIGNED  // body chunks as byte-unaligned 16-byte loads instead of aligned + v_alignbyte
#define HALO_TXB_BIG_UNALIGNED 0
#endif
#ifndef HALO_TXB_NT_LD  // body payload loads non-temporal (read once)
#define HALO_TXB_NT_LD 0
#endif
#ifndef HALO_TXB_NT_ST  // body frame stores non-temporal (written once)
#define HALO_TXB_NT_ST 0
#endif
template <int G, int U>
__device__ __forceinline__ void build_big(const BuildParams& p, const Frame& f, const uint32_t* hdr, uint32_t j,
                                          uint8_t* out) {
    static_assert(G >= 8, "lanes 0..4 take the head and tail chunks");
    const bool csum = (p.flags & HALO_RX_CSUM_ENABLE) != 0;
    const uint32_t l4s = f.base + 20u, pay_end = f.hdr_end + f.plen;
    const uint32_t ndw = (f.flen + 3u) >> 2;
    const uint64_t P = f.pay - f.hdr_end;  // the source address of frame byte 0's position
    const uint32_t sh = (uint32_t)(P & 3u);
    const uint32_t cb_end = pay_end >> 4;  // chunks [4, cb_end): payload bytes only
    typedef const __attribute__((address_space(1), unused)) uint32_t gu32_t;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4), unused));
    uint32_t sum = 0;
    // the head / tail chunk of lanes 0..4 (masked path below): its loads go out with the body's,
    // one memory round trip per frame instead of two (HALO_TXB_HEAD_EARLY)
    const uint32_t c = j < 4 ? j : cb_end;
    const bool mine = j < 4 ? 4 * j < ndw : (j == 4 && cb_end >= 4 && 4 * cb_end < ndw);
    uint32_t hraw[5] = {0u, 0u, 0u, 0u, 0u};
    if (HALO_TXB_HEAD_EARLY && mine && chunk_has_payload(f, c, ndw)) payload_raw(f, c, hraw);
    for (uint32_t c0 = 4 + j; c0 < cb_end; c0 += U * G) {
        uint32_t raw[U][5] = {};  // (a row past cb_end is offered to the neighbour lane, never used)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * G;
            if (c < cb_end) {
#if HALO_TXB_BIG_UNALIGNED
                // the chunk's 16 source bytes in one byte-unaligned load: no fifth dword, no merge
                typedef uint32_t u32x4b __attribute__((ext_vector_type(4), aligned(1)));
                const u32x4b v = *(const __attribute__((address_space(1))) u32x4b*)(P + 16ull * c);
                raw[u][0] = v.x; raw[u][1] = v.y; raw[u][2] = v.z; raw[u][3] = v.w;
                raw[u][4] = 0u;
#else
                gu32_t* q = (gu32_t*)((P + 16ull * c) & ~3ull);
#if HALO_TXB_NT_LD
                const u32x4 v = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4*)q);
#else
                const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)q;
#endif
                raw[u][0] = v.x; raw[u][1] = v.y; raw[u][2] = v.z; raw[u][3] = v.w;
#if HALO_TXB_BIG_NB
                // only a chunk whose successor no lane of this round loaded fetches its fifth dword
                raw[u][4] = (sh && (c + 1 == cb_end || (j == G - 1 && u == U - 1))) ? q[4] : 0u;
#else
                raw[u][4] = sh ? q[4] : 0u;
#endif
#endif
            }
        }
#if HALO_TXB_BIG_NB && !HALO_TXB_BIG_UNALIGNED
        // The fifth dword of chunk c is the first dword of chunk c + 1, which lane j + 1 loaded in
        // the same row (lane G - 1: lane 0's next row): one ds_bpermute per row instead of a
        // second global load per chunk. Lane 0 offers its next row's first dword (only lane G - 1
        // asks lane 0), every other lane its own row's.
        {
            const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
            const int src = 4 * (int)(j < G - 1 ? lane + 1 : lane & ~(uint32_t)(G - 1));
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t offer = (j == 0 && u + 1 < U) ? raw[u + 1 < U ? u + 1 : u][0] : raw[u][0];
                const uint32_t nb = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)offer);
                const uint32_t c = c0 + u * G;
                if (!(c + 1 == cb_end || (j == G - 1 && u == U - 1))) raw[u][4] = nb;
            }
        }
#endif
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * G;
            if (c >= cb_end) break;
            uint32_t w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w[i] = HALO_TXB_BIG_UNALIGNED ? raw[u][i] : __builtin_amdgcn_alignbyte(raw[u][i + 1], raw[u][i], sh);
                sum = hsum_acc(w[i], sum);
            }
#if HALO_TXB_NT_ST
            typedef uint32_t u32x4s __attribute__((ext_vector_type(4), aligned(4)));
            __builtin_nontemporal_store(u32x4s{w[0], w[1], w[2], w[3]}, reinterpret_cast<u32x4s*>(out + 16ull * c));
#else
            *reinterpret_cast<uint4*>(out + 16ull * c) = make_uint4(w[0], w[1], w[2], w[3]);
#endif
        }
    }
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (mine) {
        uint32_t* raw = hraw;
        if (!HALO_TXB_HEAD_EARLY && chunk_has_payload(f, c, ndw)) payload_raw(f, c, hraw);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t k = 4 * c + i;
            w[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh) & byte_mask(k, f.hdr_end, pay_end);
            if (k < 16) w[i] |= hdr[k] & byte_mask(k, 0, f.hdr_end);
            sum = hsum_acc(w[i] & byte_mask(k, l4s, pay_end), sum);
        }
        if (j == 4) {  // the frame's last chunk: only its dwords inside the frame
            uint32_t* o = reinterpret_cast<uint32_t*>(out) + 4 * c;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (4 * c + i < ndw) o[i] = w[i];
        }
    }
    // L4 checksum: pseudo header (UDP / TCP) + the segment, one's-complement, LE domain
    uint32_t part = group_sum<G>(fold16(sum));
    uint32_t ck_le = 0;
    uint32_t ck_at;
    if (f.proto == kIpUdp || f.proto == kIpTcp) {
        const uint32_t s = bswap32(f.src), t = bswap32(f.dst);
        part += hsum(s) + hsum(t) + (f.proto << 8) + bswap16(f.l4hdr + f.plen);
        ck_at = f.base + 20u + (f.proto == kIpUdp ? 6u : 16u);
    } else {
        ck_at = f.base + 22u;
    }
    if (csum || f.proto == kIpIcmp) ck_le = (~fold16(part)) & 0xFFFFu;  // ICMP always (icmp.go:84-87)
    if (mine && j < 4) {
        const uint32_t ck_dw = ck_at >> 2, ck_sh = (ck_at & 2u) * 8u;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (4 * c + i == ck_dw) w[i] |= ck_le << ck_sh;
        uint32_t* o = reinterpret_cast<uint32_t*>(out) + 4 * c;
        if (4 * c + 4 <= ndw) {
            *reinterpret_cast<uint4*>(o) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (4 * c + i < ndw) o[i] = w[i];
        }
    }
}

// Tried and removed (round 4; in git history up to commit 68eed30): software pipelining of build_big across the steps of a tile (big_load /
// big_finish, two load buffers), and a tile-flat build with every per-frame step done once by the
// lane owning the frame (flat_tile). Both bit-exact, both slower.

// Bytes [0, n) of a dword as a mask, n clamped to 0..4.
__device__ __forceinline__ uint32_t prefix_mask(int32_t n) {
    const uint32_t c = (uint32_t)(n < 0 ? 0 : n > 4 ? 4 : n);
    return (uint32_t)((1ull << (8 * c)) - 1ull);
}

// A lane's whole frame when it fits in 64 bytes (G = 1): the sixteen output dwords built in
// registers with no per-dword branch. Payload dwords come from ten aligned source loads (output
// dword k takes bytes from sources k and k + 1: the payload lies at frame bytes >= 28 in every
// layout, so sources 7..16 cover it), each address clamped into the payload's readable dwords —
// a clamped value lands only in bytes the masks drop. Header bytes [0, hdr_end) from the lane's
// header dwords, payload [hdr_end, pay_end), zero padding after; the L4 segment summed with one
// v_dot2 per dword. The caller stages o[] in LDS and the wave stores its frames cooperatively.
// UNI: every active lane of the wave has the same header end, payload end and layout (one protocol,
// one payload length: the common batch), so the byte masks and the checksum field's position are
// computed once, in scalar registers (HALO_TXB_SMALL_UNIFORM).
template <bool UNI>
__device__ __forceinline__ void build_small(const BuildParams& p, const Frame& f, const uint32_t* hdr,
                                            const void* safe, uint32_t (&o)[16]) {
    const bool csum = (p.flags & HALO_RX_CSUM_ENABLE) != 0;
    const uint32_t H = UNI ? (uint32_t)__builtin_amdgcn_readfirstlane((int)f.hdr_end) : f.hdr_end;
    const uint32_t PE = UNI ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(f.hdr_end + f.plen)) : f.hdr_end + f.plen;
    const uint64_t sv = f.pay - H;  // virtual address of frame byte 0 in payload space
    const uint32_t sh = (uint32_t)(sv & 3u);
    typedef const __attribute__((address_space(1))) uint32_t gu32_t;
    // source dword 7 + m (frame bytes 4(7+m).. in payload space) as a signed dword index r relative
    // to the payload's first readable dword, clamped into the readable dwords [0, last] in 32 bits
    // (v_med3_i32) on one 64-bit base, instead of two 64-bit clamps per load
    const uint64_t lo = f.pay & ~3ull;
    const int32_t last = (int32_t)(((f.pay + f.plen + 3u) & ~3ull) - lo) / 4 - 1;
    const int32_t r0 = (int32_t)((int64_t)(sv - sh) - (int64_t)lo) / 4;  // exact: both are dword aligned
    gu32_t* base = (gu32_t*)(f.plen ? lo : reinterpret_cast<uint64_t>(safe));
    uint32_t src[10];  // source dwords 7..16
#pragma unroll
    for (int m = 0; m < 10; ++m) {
        const int32_t r = r0 + 7 + m;
        src[m] = base[f.plen ? (r < 0 ? 0 : r > last ? last : r) : 0];
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) o[k] = hdr[k];  // bytes < 28 <= hdr_end: header only
#pragma unroll
    for (int k = 7; k < 16; ++k) {
        const uint32_t pay = __builtin_amdgcn_alignbyte(src[k - 6 < 10 ? k - 6 : 9], src[k - 7], sh);
        const uint32_t hm = prefix_mask((int32_t)H - 4 * k), pm = prefix_mask((int32_t)PE - 4 * k);
        o[k] = (k < 14 ? hdr[k] & hm : 0u) | (pay & pm & ~hm);
    }
    // L4 segment [base + 20, pay_end): everything past it is already zero
    const bool l3 = (UNI ? (uint32_t)__builtin_amdgcn_readfirstlane((int)f.base) : f.base) == 0;
    uint32_t sum = 0;
#pragma unroll
    for (int k = 5; k < 16; ++k) {
        const uint32_t seg = k >= 9 ? 0xFFFFFFFFu : k == 8 ? (l3 ? 0xFFFFFFFFu : 0xFFFF0000u) : (l3 ? 0xFFFFFFFFu : 0u);
        sum = hsum_acc(o[k] & seg, sum);
    }
    uint32_t part = fold16(sum), ck_at;
    if (f.proto == kIpUdp || f.proto == kIpTcp) {
        const uint32_t s = bswap32(f.src), t = bswap32(f.dst);
        part += hsum(s) + hsum(t) + (f.proto << 8) + bswap16(f.l4hdr + f.plen);
        ck_at = f.base + 20u + (f.proto == kIpUdp ? 6u : 16u);
    } else {
        ck_at = f.base + 22u;
    }
    const uint32_t ck_le = (csum || f.proto == kIpIcmp) ? (~fold16(part)) & 0xFFFFu : 0u;
    if constexpr (UNI) {  // the field's dword is the wave's: one OR into it
        const uint32_t at = (uint32_t)__builtin_amdgcn_readfirstlane((int)ck_at);
        const uint32_t ck_v = ck_le << ((at & 2u) * 8u);
        switch (at >> 2) {
            case 5: o[5] |= ck_v; break;
            case 6: o[6] |= ck_v; break;
            case 7: o[7] |= ck_v; break;
            case 8: o[8] |= ck_v; break;
            case 9: o[9] |= ck_v; break;
            case 10: o[10] |= ck_v; break;
            case 11: o[11] |= ck_v; break;
            default: o[12] |= ck_v; break;
        }
    } else {
        const uint32_t ck_dw = ck_at >> 2, ck_v = ck_le << ((ck_at & 2u) * 8u);
#pragma unroll
        for (int k = 5; k < 13; ++k) o[k] |= (uint32_t)k == ck_dw ? ck_v : 0u;
    }
}

// BuildUdpPkt / BuildTcpPkt / BuildIcmpPkt's length limits and the slot check (build-defined):
// HALO_TX_B_* of a descriptor (its dwords 2 and 9) and its frame length.
__device__ __forceinline__ uint32_t verdict(uint32_t d2, uint32_t d9, uint32_t stride, uint32_t& flen) {
    const uint32_t mode = (d9 >> 16) & 0xFFu;
    const uint32_t plen = d2 & 0xFFFFu, proto = (d2 >> 16) & 0xFFu;
    const uint32_t iplen = 20u + (proto == kIpTcp ? 20u : 8u) + plen;
    flen = mode == HALO_TX_BUILD_LOOPBACK ? iplen : (iplen + 14u < 60u ? 60u : iplen + 14u);
    if (proto != kIpUdp && proto != kIpTcp && proto != kIpIcmp) return HALO_TX_B_PROTO;
    if (plen > (proto == kIpTcp ? 1460u : 1472u)) return HALO_TX_B_PAYLOAD_LEN;  // udp.go:55 tcp.go:78 icmp.go:71
    if (flen > stride) return HALO_TX_B_SLOT;
    return HALO_TX_B_OK;
}

// Launch 1: each wave owns tiles of 64 consecutive descriptors (grid-stride). Lane i loads
// descriptor i of the tile and decides it; the wave's ballot ranks the rejections; then the
// wave builds the tile's frames 64 / G at a time, G lanes per frame, each group taking its
// descriptor's dwords from the lane that holds them (ds_bpermute). No LDS, no barrier.
#ifndef HALO_TXB_SMALL  // 1: frames <= 64 B on the branch-free lane path (build_small)
#define HALO_TXB_SMALL 1
#endif
#ifndef HALO_TXB_SMALL_UNIFORM  // 1: build_small's masks in scalar registers when the wave agrees
#define HALO_TXB_SMALL_UNIFORM 1
#endif
#ifndef HALO_TXB_DESC_PREFETCH
#define HALO_TXB_DESC_PREFETCH 1  // 64 B: 24.9 / 24.7 us against 25.5 / 25.0 without (profiles/r05/r5zx)
#endif
#ifndef HALO_TXB_DESC_LDS  // G = 1: the tile's descriptors read coalesced, through LDS
#define HALO_TXB_DESC_LDS 0  // measured slower: 64 B 30.2 / 30.5 us against 29.1 / 29.3 (profiles/r04/r4p)
#endif
#ifndef HALO_TXB_G1_WAVES
#define HALO_TXB_G1_WAVES 4
#endif
// Waves per tile of the 16- and 32-lane builds (HALO_TXB_SPLIT): a 1514 B tile is 97 KB of
// payload that one wave builds in G dependent steps, and 256k frames make only 4096 tiles — four
// waves per SIMD. With S waves per tile, wave `part` of tile t builds the steps congruent to part
// mod S (every wave still decides all 64 descriptors: the ranks need the whole tile's ballot), so
// the grid has S x as many waves, each with 1 / S of the LDS staging.
#ifndef HALO_TXB_SPLIT
#define HALO_TXB_SPLIT 1  // 2 measured neutral: 0.2032 / 0.2021 ms against 0.2021 / 0.2044 (profiles/r04/r4h)
#endif
template <int G>
constexpr uint32_t kSplit = G >= 16 ? HALO_TXB_SPLIT : 1;

template <int G, int U>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(G == 1 ? HALO_TXB_G1_WAVES : 4 * kSplit<G>)))
tx_build_kernel(const BuildParams p) {
#ifndef HALO_TXB_G1_LDS_TRIM
#define HALO_TXB_G1_LDS_TRIM 1
#endif
    // the descriptor staging is only for G > 1 (a lane per frame keeps its own): 11 KB less LDS
    // per block, so the lane-per-frame build fits eight blocks per CU
    constexpr uint32_t S = kSplit<G>, kOwn = kTile / S;  // waves per tile; frames each stages
    constexpr uint32_t kDescDw = (G > 1 || !HALO_TXB_G1_LDS_TRIM) ? kOwn * 10 + 1 : 1;
    constexpr uint32_t kMetaDw = (G > 1 || !HALO_TXB_G1_LDS_TRIM) ? kOwn : 1;
    __shared__ uint32_t s_desc[kBlock / 64][kDescDw];  // per wave: its tile's descriptors
    __shared__ uint32_t s_meta[kBlock / 64][kMetaDw];
    // per wave: frame-layout header dwords 0..15 (G > 1); G = 1: a lane's header for a long frame,
    // or its whole <= 64-byte frame staged for the wave's cooperative store (17-dword rows: the
    // row-wise writes and the chunk-wise reads both spread over the banks)
    constexpr uint32_t kRow = G == 1 ? 17 : 16;
    __shared__ uint32_t s_hdr[kBlock / 64][kOwn * kRow + 1];
    __shared__ uint32_t s_ndw[kBlock / 64][G == 1 ? kTile : 1];  // G = 1: staged frame's dwords (0: none)
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t nw = (gridDim.x * kBlock) >> 6;
    const uint32_t base = *p.ip_id;
    const uint32_t g = lane / G, j = lane % G;
    // descriptor i's ten dwords (zeros past the batch)
    auto load_desc = [&](uint32_t i, uint32_t (&d)[10]) {
        if (i < p.n) {
            const uint2* src = reinterpret_cast<const uint2*>(p.desc + i);
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const uint2 v = src[k];
                d[2 * k] = v.x;
                d[2 * k + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 10; ++k) d[k] = 0u;
        }
    };
    // G = 1: the next tile's descriptors load while this tile builds (one dependent round trip
    // fewer per tile; +10 VGPRs)
    constexpr bool kPf = G == 1 && HALO_TXB_DESC_PREFETCH;
    uint32_t dn[10];
    if constexpr (kPf) load_desc(((blockIdx.x * kBlock + threadIdx.x) >> 6) * kTile + lane, dn);
    for (uint32_t tw = (blockIdx.x * kBlock + threadIdx.x) >> 6; tw < p.n_tiles * S; tw += nw) {
        const uint32_t t = tw / S, part = tw % S;
        const uint32_t first = t * kTile, i = first + lane;
        uint32_t d[10];
        if constexpr (kPf) {
#pragma unroll
            for (int k = 0; k < 10; ++k) d[k] = dn[k];
            load_desc((t + nw) * kTile + lane, dn);
        } else if constexpr (G == 1 && HALO_TXB_DESC_LDS) {
            // the tile's 64 descriptors as 320 consecutive 8-byte words, lane l taking words l,
            // l + 64, ... (each load instruction reads 512 contiguous bytes instead of 64 words 40 B
            // apart), through the wave's header rows (free until the headers are written below)
            const uint2* src = reinterpret_cast<const uint2*>(p.desc + first);
            const uint32_t words = (p.n - first < kTile ? p.n - first : kTile) * 5u;
            uint32_t* scratch = &s_hdr[wv][0];
#pragma unroll
            for (uint32_t k = 0; k < 5; ++k) {
                const uint32_t w = 64u * k + lane;
                const uint2 v = w < words ? src[w] : make_uint2(0u, 0u);
                scratch[2 * w] = v.x;
                scratch[2 * w + 1] = v.y;
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < 10; ++k) d[k] = scratch[10 * lane + k];
            __builtin_amdgcn_wave_barrier();  // read before the header rows are written
        } else {
            load_desc(i, d);
        }
        uint32_t flen = 0;
        const uint32_t code = i < p.n ? verdict(d[2], d[9], p.stride, flen) : HALO_TX_B_PROTO;
        const bool rej = i < p.n && code != HALO_TX_B_OK;
        const uint64_t bal = __ballot(rej);
        if (lane == 0 && part == 0) {
            p.ws[1 + t] = (uint32_t)__popcll(bal);  // rejections in this tile
            if (bal) p.ws[0] = p.seq;
        }
        const uint32_t before =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        // iphId++ then use (ipv4.go:103-104); rejections in earlier tiles settled by launches 2/3
        const uint32_t mine = (i < p.n && !rej) ? 0x80000000u | ((base + 1u + i - before) & 0xFFFFu) : 0u;
        uint32_t hv[16];  // this lane's descriptor's header (Ethernet layout, or the loopback bytes from 14 on)
        {
            const Frame f = decode(d, p.payload);
            const uint32_t id = mine & 0xFFFFu;
            uint32_t e[18];
            eth_header(f, id, ipv4_cksum(f, id, (p.flags & HALO_RX_CSUM_ENABLE) != 0), p, e);
            const bool l3 = f.mode == HALO_TX_BUILD_LOOPBACK;
            if (__builtin_amdgcn_ballot_w64(l3) == 0) {  // wave-uniform: no loopback packet, no shift
#pragma unroll
                for (int k = 0; k < 16; ++k) hv[k] = k >= 14 ? 0u : e[k];
            } else {
#pragma unroll
                for (int k = 0; k < 16; ++k) hv[k] = k >= 14 ? 0u : l3 ? ((e[k + 3] >> 16) | (e[k + 4] << 16)) : e[k];
            }
        }
        if constexpr (G == 1) {
            // a frame of <= 64 B is built in registers and staged in LDS; longer ones read their
            // header from LDS and store as they build
            uint32_t* row = &s_hdr[wv][kRow * lane];
            uint32_t staged = 0;
            if (mine >> 31) {
                const Frame f = decode(d, p.payload);
                if (HALO_TXB_SMALL && f.flen <= 64u) {
                    uint32_t o[16];
                    // (the lanes here: this tile's small frames; uniform over them in the common batch)
                    // (flen <= 64: hdr_end, plen and base < 256; proto sets the checksum field)
                    const uint32_t sig = f.hdr_end | (f.plen << 8) | (f.base << 16) | (f.proto << 24);
                    const uint32_t sig0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)sig);
                    if (HALO_TXB_SMALL_UNIFORM && __builtin_amdgcn_ballot_w64(sig != sig0) == 0)
                        build_small<true>(p, f, hv, p.desc + i, o);
                    else
                        build_small<false>(p, f, hv, p.desc + i, o);
#pragma unroll
                    for (int k = 0; k < 16; ++k) row[k] = o[k];
                    staged = (f.flen + 3u) >> 2;
                } else {
#pragma unroll
                    for (int k = 0; k < 16; ++k) row[k] = hv[k];
                    build_frame<G, U>(p, f, row, 0, p.frames + (uint64_t)i * p.stride);
                }
            }
            s_ndw[wv][lane] = staged;
            __builtin_amdgcn_wave_barrier();
            // the staged frames, four lanes per frame: lane 4g + c stores chunk c of frame 16s + g,
            // so one store instruction writes 16 frames' chunks side by side
#pragma unroll
            for (uint32_t st = 0; st < 4; ++st) {
                const uint32_t fl = 16 * st + (lane >> 2), c = lane & 3u;
                const uint32_t nd = s_ndw[wv][fl];
                if (4 * c < nd) {
                    const uint32_t* src = &s_hdr[wv][kRow * fl + 4 * c];
                    uint32_t* o = reinterpret_cast<uint32_t*>(p.frames + (uint64_t)(first + fl) * p.stride) + 4 * c;
                    if (4 * c + 4 <= nd) {
                        *reinterpret_cast<uint4*>(o) = make_uint4(src[0], src[1], src[2], src[3]);
                    } else {
#pragma unroll
                        for (uint32_t q = 0; q < 3; ++q)
                            if (4 * c + q < nd) o[q] = src[q];
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();  // the region is rewritten for the next tile
        } else {
            // this wave's frames (steps congruent to `part` mod S) at compact LDS slots
            constexpr uint32_t F = 64u / G;  // frames per step
            const uint32_t my_step = lane / F;
            const uint32_t slot = (my_step / S) * F + lane % F;
            if (my_step % S == part) {
#pragma unroll
                for (int k = 0; k < 16; ++k) s_hdr[wv][kRow * slot + k] = hv[k];
                // the wave's descriptors through its own LDS region (no block barrier), so that they
                // are not live in registers across the build steps
#pragma unroll
                for (int k = 0; k < 10; ++k) s_desc[wv][10 * slot + k] = d[k];
                s_meta[wv][slot] = mine;
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll 1
            for (uint32_t step = 0; step < (uint32_t)G / S; ++step) {
                const uint32_t sl = step * F + g;                // this group's frame's LDS slot
                const uint32_t fl = (step * S + part) * F + g;  // ... and its lane in the tile
                const uint32_t meta = s_meta[wv][sl];
                if (meta >> 31) {  // uniform over the group
                    uint32_t dd[10];
#pragma unroll
                    for (int k = 0; k < 10; ++k) dd[k] = s_desc[wv][10 * sl + k];
                    if constexpr (G >= 16 && HALO_TXB_BIG_PATH)
                        build_big<G, U>(p, decode(dd, p.payload), &s_hdr[wv][kRow * sl], j,
                                        p.frames + (uint64_t)(first + fl) * p.stride);
                    else
                        build_frame<G, U>(p, decode(dd, p.payload), &s_hdr[wv][kRow * sl], j,
                                          p.frames + (uint64_t)(first + fl) * p.stride);
                }
            }
            __builtin_amdgcn_wave_barrier();  // the region is rewritten for the next tile
        }
        if (part == 0 && i < p.n) {  // after the build: these stores do not hold up the payload loads
            p.lens[i] = code == HALO_TX_B_OK ? (uint16_t)flen : (uint16_t)0;
            if (p.result) p.result[i] = (uint8_t)code;
        }
    }
}

// Launch 1 for frames of more than 64 chunks (HALO_TXB_PAIR, the default): one wave per pair of
// frames, 32 lanes each (build_big), no grid-stride loop — the dispatcher walks the batch in order
// the way the size-matched probe's blocks do. A wave that owns a 64-frame tile for 32 dependent
// steps keeps 4096 streams 97 KB apart open at once for 256k frames; the same bytes moved by a
// no-work probe with that structure ran 0.184-0.202 ms against 0.145 for the streaming probe
// (tools/exp/tx_layout_sweep.py, profiles/r04/r4l). Each wave still decides its tile's 64
// descriptors (their dwords 2 and 9 only: 512 B, shared by the tile's 32 waves through the L2) for
// the rank of its two frames among the tile's rejections; the wave holding the tile's first pair
// writes the tile's rejection count for launches 2 and 3.
#ifndef HALO_TXB_PAIR
#define HALO_TXB_PAIR 1
#endif
#ifndef HALO_TXB_PAIR_XCD
#define HALO_TXB_PAIR_XCD 1
#endif
template <int U>
__global__ void __launch_bounds__(kBlock) tx_build_pair_kernel(const BuildParams p) {
    __shared__ uint32_t s_hdr[kBlock / 64][2 * 16];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    // XCD-aware order (HALO_TXB_PAIR_XCD): blocks are dealt round-robin over the 8 XCDs, and the 8
    // blocks of a tile all read the tile's descriptor block — in dispatch order once per XCD, 1.19x
    // the algorithmic reads (r4p). Within each run of 64 blocks (8 tiles), block b takes tile
    // b % 8 of the run, part (b / 8) % 8: a tile stays on one XCD, and the batch is still walked
    // in order 8 tiles at a time. (Giving each XCD a contiguous eighth of the batch instead cut the
    // reads to 1.0002x but ran 2-3 % slower: r4q.)
    const uint32_t lb = HALO_TXB_PAIR_XCD == 2 ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)
                      : HALO_TXB_PAIR_XCD == 1 ? (blockIdx.x & ~63u) | ((blockIdx.x & 7u) << 3) | ((blockIdx.x >> 3) & 7u)
                                               : blockIdx.x;
    const uint32_t pair = lb * (kBlock / 64) + wv;
    if (2ull * pair >= p.n) return;  // wave-uniform
    const uint32_t g = lane >> 5, j = lane & 31u;
    const uint32_t i = 2 * pair + g, t = (2 * pair) / kTile, il = t * kTile + lane;
    const uint32_t base_id = *p.ip_id;
    // this group's descriptor first: its loads go out with the tile's verdict loads below
    uint32_t d[10];
    if (i < p.n) {
        const uint2* src = reinterpret_cast<const uint2*>(p.desc + i);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint2 v = src[k];
            d[2 * k] = v.x;
            d[2 * k + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 10; ++k) d[k] = 0u;
    }
    uint32_t d2 = 0, d9 = 0, flen_l = 0;
    if (il < p.n) {
        const uint32_t* dw = reinterpret_cast<const uint32_t*>(p.desc + il);
        d2 = dw[2];
        d9 = dw[9];
    }
    const uint32_t code_l = il < p.n ? verdict(d2, d9, p.stride, flen_l) : HALO_TX_B_PROTO;
    const uint64_t bal = __ballot(il < p.n && code_l != HALO_TX_B_OK);
    if (lane == 0 && (pair % (kTile / 2)) == 0) {
        p.ws[1 + t] = (uint32_t)__popcll(bal);  // rejections in tile t
        if (bal) p.ws[0] = p.seq;
    }
    const uint32_t fl = i % kTile;
    const uint32_t code = (uint32_t)__shfl((int)code_l, (int)fl, 64), flen = (uint32_t)__shfl((int)flen_l, (int)fl, 64);
    const uint32_t before = (uint32_t)__popcll(bal & ((1ull << fl) - 1ull));
    const bool build = i < p.n && code == HALO_TX_B_OK;
    const uint32_t id = (base_id + 1u + i - before) & 0xFFFFu;  // iphId++ then use (ipv4.go:103-104)
    const Frame f = decode(d, p.payload);
    if (j == 0 && build) {  // the frame's header dwords 0..15 (Ethernet layout, or the loopback bytes)
        uint32_t e[18];
        eth_header(f, id, ipv4_cksum(f, id, (p.flags & HALO_RX_CSUM_ENABLE) != 0), p, e);
        const bool l3 = f.mode == HALO_TX_BUILD_LOOPBACK;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            s_hdr[wv][16 * g + k] = k >= 14 ? 0u : l3 ? ((e[k + 3] >> 16) | (e[k + 4] << 16)) : e[k];
    }
    __builtin_amdgcn_wave_barrier();
    if (build) build_big<32, U>(p, f, &s_hdr[wv][16 * g], j, p.frames + (uint64_t)i * p.stride);
    if (j == 0 && i < p.n) {
        p.lens[i] = build ? (uint16_t)flen : (uint16_t)0;
        if (p.result) p.result[i] = (uint8_t)code;
    }
}

// Launch 2: the new iphId, and only after a rejection the renumbering of the frames behind it. A
// tile that saw a rejection stores this launch's sequence number (p.seq) in ws[0] beside its count
// in ws[1 + t]. The common case — no tile did — is one load per block and one iphId update: round 3
// ran a one-block settle launch and a renumber launch after every build, ~6 us of launch gaps per
// step (a 64 B build is 23 us of kernel; r4t). A stale or uninitialised ws[0] equal to p.seq only by
// chance takes the full path, which recomputes everything from the tile counts and is exact anyway.
// Full path: every block scans the tile counts 1024 at a time (exclusive prefix in LDS) and patches
// the frames of its own tiles (t = block mod grid) that were numbered too high by the rejections in
// earlier tiles: identification and, with checksums on, the IPv4 header checksum (RFC 1624
// incremental update of the value BuildIpv4Pkt computed); block 0 writes the new iphId.
__global__ void __launch_bounds__(1024) tx_finish_kernel(const BuildParams p) {
    __shared__ uint32_t s_part[1024 / 64];
    __shared__ uint32_t s_carry;
    __shared__ uint32_t s_pre[1024];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    if (p.ws[0] != p.seq) {  // no rejection in this launch
        if (blockIdx.x == 0 && tid == 0) *p.ip_id = (uint16_t)(*p.ip_id + p.n);  // one iphId++ per built packet
        return;
    }
    const bool csum = (p.flags & HALO_RX_CSUM_ENABLE) != 0;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t t0 = 0; t0 < p.n_tiles; t0 += 1024) {
        const uint32_t t = t0 + tid;
        const uint32_t v = t < p.n_tiles ? p.ws[1 + t] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) s_part[wave] = x;
        __syncthreads();
        uint32_t off = s_carry;
        for (uint32_t w = 0; w < wave; ++w) off += s_part[w];
        s_pre[tid] = off + x - v;  // rejections before tile t
        __syncthreads();
        // this block's tiles of the pass, one wave per tile, lane = frame of the tile
        const uint32_t r0 = (blockIdx.x + gridDim.x - t0 % gridDim.x) % gridDim.x;
        for (uint32_t r = r0 + wave * gridDim.x; r < 1024 && t0 + r < p.n_tiles; r += 16 * gridDim.x) {
            const uint32_t back = s_pre[r];
            const uint32_t i = (t0 + r) * kTile + lane;
            if (back == 0u || i >= p.n || p.lens[i] == 0) continue;
            const uint32_t mode = (reinterpret_cast<const uint32_t*>(p.desc + i)[9] >> 16) & 0xFFu;
            uint8_t* ip = p.frames + (uint64_t)i * p.stride + (mode == HALO_TX_BUILD_LOOPBACK ? 0u : 14u);
            const uint32_t old_id = ((uint32_t)ip[4] << 8) | ip[5];
            const uint32_t new_id = (old_id - back) & 0xFFFFu;
            ip[4] = (uint8_t)(new_id >> 8);
            ip[5] = (uint8_t)new_id;
            if (csum) {  // HC' = ~(~HC + ~m + m')
                const uint32_t hc = ((uint32_t)ip[10] << 8) | ip[11];
                const uint32_t nc = (~fold16((~hc & 0xFFFFu) + (~old_id & 0xFFFFu) + new_id)) & 0xFFFFu;
                ip[10] = (uint8_t)(nc >> 8);
                ip[11] = (uint8_t)nc;
            }
        }
        if (tid == 0) {
            uint32_t tot = 0;
            for (uint32_t w = 0; w < 1024 / 64; ++w) tot += s_part[w];
            s_carry += tot;
        }
        __syncthreads();  // s_pre and s_part are rewritten by the next pass
    }
    if (blockIdx.x == 0 && tid == 0) *p.ip_id = (uint16_t)(*p.ip_id + p.n - s_carry);
}

}  // namespace
}  // namespace halo

extern "C" HALO_API uint64_t halo_tx_build_workspace(uint32_t n) {
    return 4ull * (1ull + ((uint64_t)n + halo::kTile - 1) / halo::kTile);
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
        (reinterpret_cast<uintptr_t>(d_workspace) & 3u) || (reinterpret_cast<uintptr_t>(d_ip_id) & 1u))
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
    static std::atomic<uint32_t> launches{0};
    do p.seq = launches.fetch_add(1, std::memory_order_relaxed) + 1u; while (p.seq == 0u);
    hipStream_t s = static_cast<hipStream_t>(stream);
    // a wave per tile of 64 descriptors, grid-stride: up to 8 resident 4-wave blocks per CU
#ifndef HALO_TXB_MAX_BLOCKS
#define HALO_TXB_MAX_BLOCKS (HALO_TXB_G1_WAVES * 256u)  // waves x 1024 SIMDs / 4 per block: one resident round
#endif
    // lanes per frame and chunks per lane from the largest frame expected (a frame needs
    // ceil(flen / 16) chunks; longer ones than G * U chunks take extra rounds)
    const uint32_t h = max_payload_hint ? max_payload_hint : 1472u;
    const uint32_t chunks = (h + 42u + 15u) / 16u;  // UDP / ICMP headers; TCP frames 12 B longer
    const uint32_t split = chunks > 32 ? halo::kSplit<16> : 1u;  // waves per tile (G >= 16)
    const uint32_t waves = p.n_tiles * split, blocks = (waves + 3) / 4, cap = HALO_TXB_MAX_BLOCKS * split;
    const dim3 grid(blocks < cap ? blocks : cap), blk(halo::kBlock);
    if (chunks <= 4) hipLaunchKernelGGL((halo::tx_build_kernel<1, 4>), grid, blk, 0, s, p);
    else if (chunks <= 16) hipLaunchKernelGGL((halo::tx_build_kernel<4, 4>), grid, blk, 0, s, p);
    else if (chunks <= 32) hipLaunchKernelGGL((halo::tx_build_kernel<8, 4>), grid, blk, 0, s, p);
    else if (chunks <= 64) hipLaunchKernelGGL((halo::tx_build_kernel<16, 4>), grid, blk, 0, s, p);
// lanes x chunks per round for frames > 64 chunks: 32 x 3 (227 us for 256k x 1514 B) against
// 16 x 6 303, 16 x 3 242, 8 x 4 277, 64 x 2 305, 32 x 2 244 (profiles/r02/txb/ab_big_frame_G_U_sweep.log)
#ifndef HALO_TXB_BIG_G
#define HALO_TXB_BIG_G 32
#define HALO_TXB_BIG_U 3
#endif
    else if (HALO_TXB_PAIR)
        hipLaunchKernelGGL((halo::tx_build_pair_kernel<HALO_TXB_BIG_U>),
                           dim3((uint32_t)(((uint64_t)n + 511u) / 512u * 64u)), blk, 0, s, p);  // runs of 8 tiles
    else hipLaunchKernelGGL((halo::tx_build_kernel<HALO_TXB_BIG_G, HALO_TXB_BIG_U>), grid, blk, 0, s, p);
    // Launch 2 (one word in the common case) costs the same with 1, 8 or 64 blocks (25.2 / 25.2 /
    // 25.0 us per 64 B call, profiles/r05/r5j): the gap between two dependent dispatches, not the
    // grid. 64 keeps the renumbering after a rejection wide.
#ifndef HALO_TXB_FINISH_BLOCKS
#define HALO_TXB_FINISH_BLOCKS 64u
#endif
    hipLaunchKernelGGL(halo::tx_finish_kernel, dim3(p.n_tiles < HALO_TXB_FINISH_BLOCKS ? p.n_tiles : HALO_TXB_FINISH_BLOCKS),
                       dim3(1024), 0, s, p);
    return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
}
