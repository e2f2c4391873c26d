// rx_parse.hip — the hot path: batched Ethernet -> IPv4 -> UDP/TCP/ICMP parse and
// 16-bit one's-complement Internet checksum verification on gfx950 (MI355X).
//
// Restates, per frame and bit-exactly:
//   protocol.GetCheckSum        protocol/utils.go:11-31
//   protocol.ParseEthFrm        protocol/ethernet.go:29-55
//   protocol.ParseIpv4Pkt       protocol/ipv4.go:48-86
//   protocol.ParseUdpPkt        protocol/udp.go:21-49
//   protocol.ParseTcpPkt        protocol/tcp.go:36-70
//   protocol.ParseIcmpPkt       protocol/icmp.go:33-63
//   protocol.NatGetSrcDstPort   protocol/ipv4.go:229-246
//   NetIf.RxEthernet / RxIpv4 branch inputs  engine/ethernet_engine.go:22, ipv4_engine.go:24,31
//
// Execution shape (DESIGN.md "Kernels"): a group of G lanes of one 64-wide wavefront owns a
// frame; 64/G frames per wave. Lane j of the group loads dwords [4j, 4j+4) + k*4G of the frame
// with one 16-byte load per step, so a wave-instruction covers 64/G frames' consecutive bytes
// (coalesced). The 48-byte header (dwords 0..11) sits in group lanes 0..2 after the first load
// and is broadcast to the group (DPP quad_perm / row_newbcast for G = 4 / 16, v_readlane for
// G = 64, ds_bpermute otherwise); every lane then runs the header checks redundantly (no
// divergence, no second broadcast). Only the L4 segment sum needs a cross-lane reduction
// (DPP butterflies). G = 1 (small frames): each lane owns a whole frame, reads its header with
// its own three 16-byte loads and needs no cross-lane traffic at all. Mixed sizes packed in
// memory (IMIX) take the byte-stream kernel (rx_stream_kernel below): a lane per frame for the
// header, the whole wave for one coalesced pass over the window's bytes, and every L4 sum as a
// difference of a running prefix.
//
// Checksum arithmetic (DESIGN.md "Checksum in the little-endian domain"): the frame is summed
// as little-endian dwords. A one's-complement sum of byte-swapped 16-bit words is the byte
// swap of the sum (RFC 1071 §2B); swapping maps 0xFFFF to itself, and 2^16 == 1 (mod 0xFFFF),
// so "GetCheckSum(region) == 0" <=> fold16(sum of the LE dwords of the region) == 0xFFFF.
// Every region on the path starts at an even frame offset (14, 26, 34), so region edges fall
// on half-dwords and an odd trailing byte lands in the low byte of its half, which is the
// HIGH byte of its big-endian word: exactly protocol/utils.go:21-24.
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>

#include "device_util.h"
#include "flow_key.h"
#include "halo_common.h"
#include "route_view.h"

namespace halo {
namespace {

// NT: a non-temporal store. The byte-stream kernel's records take it (HALO_RX_STREAM_NT_STORES):
// IMIX 1.272 -> 1.244 / 1.240 ms on one box (profiles/r06/r6c/ab_nt.log); the lane kernel's do
// not (1M x 64 B 21.5 -> 22.2 us in the same A/B; §15.4).
#ifndef HALO_RX_STREAM_NT_STORES
#define HALO_RX_STREAM_NT_STORES 1
#endif
#ifndef HALO_RX_NT_STORES  // every other record store (measurement knob)
#define HALO_RX_NT_STORES 0
#endif
template <bool NT = (HALO_RX_NT_STORES != 0)>
__device__ __forceinline__ void store16(uint4* dst, uint4 v) {
    if constexpr (NT) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store((u32x4){v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(dst));
    } else {
        *dst = v;
    }
}

// Byte offset of the IPv4 header in the buffer: 14 in an Ethernet frame, 0 for a LoChan packet
// (HALO_RX_L3_START). Both are even, so every region stays on half-dword boundaries.
template <bool L3>
constexpr uint32_t kIpOff = L3 ? 0u : 14u;

// Accumulate the L4-segment bytes [kIpOff + 20, seg_end) held in dwords [d0, d0+4).
template <bool L3>
__device__ __forceinline__ void acc_segment(const uint32_t (&w)[4], uint32_t d0, uint32_t seg_end, uint64_t& c) {
    constexpr uint32_t kSeg = kIpOff<L3> + 20u;  // 34 (dword 8, high half) or 20 (dword 5)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t d = d0 + j;
        const int32_t rel = (int32_t)seg_end - (int32_t)(4u * d);  // segment bytes left in this dword
        uint32_t keep = rel >= 4 ? 0xFFFFFFFFu : (rel <= 0 ? 0u : ((1u << (rel * 8)) - 1u));
        keep &= d >= (kSeg + 3u) / 4u ? 0xFFFFFFFFu : ((kSeg & 2u) && d == kSeg / 4u ? 0xFFFF0000u : 0u);
        c += (uint64_t)(w[j] & keep);
    }
}

// Lane-per-frame form of acc_segment (G = 1): the end mask from one clamped shift (v_med3 + a
// 64-bit shift) instead of two compares and selects, and each dword's two 16-bit halves added into
// a u32 with one v_dot2_u32_u16 instead of a 64-bit add. A halves sum keeps the value mod 0xFFFF
// (2^16 == 1) and is zero exactly when the masked bytes are, which is all fold16 looks at; it stays
// below 2^32 for any frame (<= 2254 dwords x 2 x 0xFFFF). e8 = 8 * seg_end.
#ifndef HALO_RX_LANE_DOT2
#define HALO_RX_LANE_DOT2 1
#endif
template <bool L3>
__device__ __forceinline__ void acc_segment_dot2(const uint32_t (&w)[4], uint32_t d0, int32_t e8, uint32_t& h) {
    constexpr uint32_t kSeg = kIpOff<L3> + 20u;
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 one = {1, 1};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t d = d0 + j;
        const int32_t r8 = e8 - (int32_t)(32u * d);
        const int32_t sh = r8 < 0 ? 0 : (r8 > 32 ? 32 : r8);  // segment bits left in this dword
        uint32_t keep = (uint32_t)~(~0ull << sh);
        keep &= d >= (kSeg + 3u) / 4u ? 0xFFFFFFFFu : ((kSeg & 2u) && d == kSeg / 4u ? 0xFFFF0000u : 0u);
        h = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w[j] & keep), one, h, false);
    }
}

// Group form (G > 1): the halves sum (v_dot2_u32_u16, as acc_segment_dot2) of the segment bytes in
// dwords [d0, d0+4). A chunk wholly inside the segment needs no mask, and whether every lane's chunk
// is is one wave-uniform test, so the common case costs four v_dot2 per chunk; only a wave whose
// chunk meets the segment's start or end (FIRST: round 0's header chunk) takes the masked path.
template <bool L3, bool FIRST = false>
__device__ __forceinline__ void acc_chunk(const uint32_t (&w)[4], uint32_t d0, uint32_t seg_end, uint32_t& hs) {
    constexpr uint32_t kSeg = kIpOff<L3> + 20u;
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 one = {1, 1};
    const bool inside = 4u * d0 >= kSeg && 4u * d0 + 16u <= seg_end;
    if (!FIRST && __builtin_amdgcn_ballot_w64(!inside) == 0) {  // wave-uniform: no masks
#pragma unroll
        for (int j = 0; j < 4; ++j) hs = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w[j]), one, hs, false);
        return;
    }
    acc_segment_dot2<L3>(w, d0, (int32_t)(8u * seg_end), hs);
}

struct Verdict {
    uint32_t status, flags, ethertype, ip_proto, ip_total_len, src_ip, dst_ip, sport, dport;
    uint32_t pay_off, pay_len, l4_aux, l4_seq, l4_ack;
    uint32_t seg_end;   // end of the L4 segment whose sum is needed (0: none)
    uint32_t l4_extra;  // pseudo-header + header-field part of the L4 sum, LE domain
    bool check_l4;      // L4 checksum decides the verdict after the reduction
};

#define HB(b) ((h[(b) >> 2] >> (((b)&3) * 8)) & 0xFFu)

// Frames failing ParseEthFrm's length check (or, for LoChan packets, ParseIpv4Pkt's) are never
// read: the reference looks at no byte of them.
template <bool L3>
__device__ __forceinline__ bool len_readable(uint32_t L, uint32_t flags) {
    const bool jumbo = (flags & HALO_RX_JUMBO_EXT) != 0;
    if constexpr (L3) return L >= 20u && L <= (jumbo ? kIpMaxJumbo : kIpMax);
    return L >= kEthMin && L <= (jumbo ? kEthMaxJumbo : kEthMax);
}

// Header checks, in reference order, up to (not including) the L4 checksum. h = buffer dwords
// 0..11: an Ethernet frame (IPv4 header at byte 14) or, with L3, a LoChan packet (at byte 0).
template <bool L3>
__device__ __forceinline__ Verdict parse_header(const uint32_t (&h)[12], uint32_t L, bool present,
                                                const RxParams& p) {
    constexpr uint32_t O = kIpOff<L3>;
    Verdict v;
    v.status = HALO_RX_OK; v.flags = 0; v.ethertype = kEthUnknown; v.ip_proto = kIpUnknown;
    v.ip_total_len = 0; v.src_ip = 0; v.dst_ip = 0; v.sport = 0; v.dport = 0;
    v.pay_off = 0; v.pay_len = 0; v.l4_aux = 0; v.l4_seq = 0; v.l4_ack = 0;
    v.seg_end = 0; v.l4_extra = 0; v.check_l4 = false;
    const bool jumbo = (p.flags & HALO_RX_JUMBO_EXT) != 0;
    const bool csum = (p.flags & HALO_RX_CSUM_ENABLE) != 0;
    const uint32_t ip_max = jumbo ? kIpMaxJumbo : kIpMax;
    const uint32_t l4_max = jumbo ? kL4MaxJumbo : kL4Max;

    uint32_t iplen;
    if constexpr (L3) {  // a LoChan packet: IPv4 only, no Ethernet layer (engine/engine.go:361)
        v.ethertype = kEthIpv4;
        iplen = L;
    } else {
        // ---- ParseEthFrm (protocol/ethernet.go:29-55)
        const uint32_t eth_max = jumbo ? kEthMaxJumbo : kEthMax;
        if (!present || L < kEthMin || L > eth_max) { v.status = HALO_RX_ETH_LEN; return v; }
        const uint32_t et = bswap16(h[3] & 0xFFFFu);
        if (et != kEthIeee8023 && et != kEthIpv4 && et != kEthArp && et != kEthIpv6) {
            v.status = HALO_RX_ETH_TYPE; return v;
        }
        v.ethertype = et;
        v.pay_off = 14; v.pay_len = L - 14;
        // RxEthernet's filter (engine/ethernet_engine.go:22)
        const uint32_t dm_lo = h[0], dm_hi = h[1] & 0xFFFFu;
        if ((dm_lo == p.mac_lo && dm_hi == p.mac_hi) || (dm_lo == 0xFFFFFFFFu && dm_hi == 0xFFFFu))
            v.flags |= HALO_RX_F_MAC_MATCH;
        if (et != kEthIpv4) return v;
        iplen = L - 14;
    }

    // ---- ParseIpv4Pkt (protocol/ipv4.go:48-86) on pkt = frm[14:L] (or the LoChan packet)
    if ((L3 && !present) || iplen < 20 || iplen > ip_max) { v.status = HALO_RX_IP_LEN; return v; }
    if (HB(O + 0) != 0x45u) { v.status = HALO_RX_IP_VER; return v; }
    if ((HB(O + 6) != 0x40u && HB(O + 6) != 0x00u) || HB(O + 7) != 0x00u) { v.status = HALO_RX_IP_FRAG; return v; }
    const uint32_t proto = HB(O + 9);
    if (proto != kIpIcmp && proto != kIpTcp && proto != kIpUdp) { v.status = HALO_RX_IP_PROTO; return v; }
    // pseudo-header src+dst (IP bytes 12..19), LE domain; sum_a = the rest of the IP header
    const uint32_t sum_b = L3 ? hsum(h[3]) + hsum(h[4]) : (h[6] >> 16) + hsum(h[7]) + (h[8] & 0xFFFFu);
    if (csum) {
        const uint32_t sum_a = L3 ? hsum(h[0]) + hsum(h[1]) + hsum(h[2])
                                  : (h[3] >> 16) + hsum(h[4]) + hsum(h[5]) + (h[6] & 0xFFFFu);
        if (fold16(sum_a + sum_b) != 0xFFFFu) { v.status = HALO_RX_IP_HDR_CKSUM; return v; }
    }
    const uint32_t total_len = L3 ? bswap16(h[0] >> 16) : bswap16(h[4] & 0xFFFFu);
    // pkt[20:totalLen] (protocol/ipv4.go:84): Go panics below 20 and reads stale bytes or
    // panics past len(pkt); both are reported as build-defined statuses.
    if (total_len < 20) { v.status = HALO_RX_IP_TOTLEN_UNDERFLOW; return v; }
    if (total_len > iplen) { v.status = HALO_RX_IP_TOTLEN_OVERRUN; return v; }
    v.ip_proto = proto;
    v.ip_total_len = total_len;
    v.src_ip = (HB(O + 12) << 24) | (HB(O + 13) << 16) | (HB(O + 14) << 8) | HB(O + 15);
    v.dst_ip = (HB(O + 16) << 24) | (HB(O + 17) << 16) | (HB(O + 18) << 8) | HB(O + 19);
    if (HB(O + 19) == 255u) v.flags |= HALO_RX_F_IP_BCAST;
    if (v.dst_ip == p.own_ip) v.flags |= HALO_RX_F_DST_IS_OWN;
    // NatGetSrcDstPort (protocol/ipv4.go:229-246) on the untrimmed packet: (0, 0) below 26 B,
    // which only a LoChan packet can be (an Ethernet frame's IPv4 part is >= 28 B)
    if (L3 && iplen < 26) {
        v.sport = v.dport = 0;
    } else if (proto == kIpIcmp) {
        v.sport = v.dport = (HB(O + 24) << 8) | HB(O + 25);
    } else {
        v.sport = (HB(O + 20) << 8) | HB(O + 21);
        v.dport = (HB(O + 22) << 8) | HB(O + 23);
    }
    v.pay_off = O + 20; v.pay_len = total_len - 20;

    // ---- L4 pre-checksum checks on pkt = ipPayload (len = totalLen - 20)
    const uint32_t l4len = total_len - 20;
    const uint32_t seg_end = total_len + O;
    if (proto == kIpUdp) {        // protocol/udp.go:21-49
        if (l4len < 8 || l4len > l4_max) { v.status = HALO_RX_L4_LEN; return v; }
        if (csum) {  // pseudo length = the UDP header's own length field (udp.go:30,38)
            v.check_l4 = true; v.seg_end = seg_end;
            v.l4_extra = sum_b + 0x1100u + (L3 ? h[6] & 0xFFFFu : h[9] >> 16);  // IP bytes 24..25
        }
    } else if (proto == kIpTcp) { // protocol/tcp.go:36-70
        if (l4len < 20 || l4len > l4_max) { v.status = HALO_RX_L4_LEN; return v; }
        if (csum) {  // pseudo length = len(pkt) (tcp.go:54-59)
            v.check_l4 = true; v.seg_end = seg_end;
            v.l4_extra = sum_b + 0x0600u + bswap16(l4len);
        }
    } else {                      // ICMP, protocol/icmp.go:33-63: checksum ALWAYS verified
        if (l4len < 8 || l4len > l4_max) { v.status = HALO_RX_L4_LEN; return v; }
        const uint32_t type = HB(O + 20);
        if (type != kIcmpRequest && type != kIcmpReply && type != kIcmpTtl) { v.status = HALO_RX_ICMP_TYPE; return v; }
        if (HB(O + 21) != 0u) { v.status = HALO_RX_ICMP_CODE; return v; }
        v.check_l4 = true; v.seg_end = seg_end; v.l4_extra = 0;
    }
    return v;
}

// L4 outputs once the whole chain succeeded.
template <bool L3>
__device__ __forceinline__ void finish_l4(const uint32_t (&h)[12], Verdict& v) {
    constexpr uint32_t S = kIpOff<L3> + 20u;  // L4 segment start
    const uint32_t l4len = v.ip_total_len - 20;
    if (v.ip_proto == kIpUdp) {
        v.pay_off = S + 8; v.pay_len = l4len - 8;                       // udp.go:47
    } else if (v.ip_proto == kIpTcp) {
        v.l4_aux = HB(S + 13);                                         // tcp.go:50
        v.l4_seq = (HB(S + 4) << 24) | (HB(S + 5) << 16) | (HB(S + 6) << 8) | HB(S + 7);
        v.l4_ack = (HB(S + 8) << 24) | (HB(S + 9) << 16) | (HB(S + 10) << 8) | HB(S + 11);
        const uint32_t hl = HB(S + 12) >> 4;                           // tcp.go:49 (words used as bytes)
        v.pay_off = S + hl; v.pay_len = l4len - hl;                    // tcp.go:68
    } else {
        v.l4_aux = HB(S);                                              // icmp.go:38
        v.l4_seq = (HB(S + 4) << 24) | (HB(S + 5) << 16) | (HB(S + 6) << 8) | HB(S + 7);
        v.pay_off = S + 8; v.pay_len = l4len - 8;                       // icmp.go:62
    }
}
#undef HB

// LAYOUT 0: ragged (u32 dword offsets + u16 lengths); 1: strided with per-frame lengths;
// 2: strided, one length; 3: ragged LoChan packets (HALO_RX_L3_START).
template <int LAYOUT>
constexpr bool kL3 = LAYOUT == 3;

template <int LAYOUT>
__device__ __forceinline__ void frame_at(const RxParams& p, uint64_t i, const uint8_t*& frame, uint32_t& L) {
    if constexpr (LAYOUT == 0 || LAYOUT == 3) {
        frame = p.bytes + ((uint64_t)p.offsets_dw[i] << 2);
        L = p.lens[i];
    } else if constexpr (LAYOUT == 1) {
        frame = p.bytes + i * p.stride;
        L = p.lens[i];
    } else {
        frame = p.bytes + i * p.stride;
        L = p.len;
    }
}

// Per-block status histogram: OK frames are counted per lane, the rest in LDS.
struct Hist {
    uint32_t* s;  // __shared__ [HALO_RX_STATUS_COUNT]
    uint32_t ok;
    // status threads: the key word the launch queue's tree most likely has (flush_hist), loaded when
    // the block starts so that its latency hides under the frame loads instead of ending the block
    unsigned long long key;
    __device__ __forceinline__ void add(uint32_t status) {
        if (status == HALO_RX_OK) ++ok;
        else atomicAdd(&s[status], 1u);
    }
};

// The launch's HSA queue and the tree-set slot its key is looked up from first.
__device__ __forceinline__ unsigned long long launch_queue() {
    return (unsigned long long)(uintptr_t)(const void*)__builtin_amdgcn_queue_ptr();
}
__device__ __forceinline__ uint32_t tree_slot0(unsigned long long q) {
    return ((uint32_t)(q >> 6) ^ (uint32_t)(q >> 17)) & (kHistTrees - 1u);
}
__device__ __forceinline__ Hist hist_open(const RxParams& p, uint32_t* s_hist) {
    Hist h{s_hist, 0, 0};
    if (p.hist && threadIdx.x < HALO_RX_STATUS_COUNT)
        h.key = reinterpret_cast<const unsigned long long*>(p.hist)[tree_slot0(launch_queue())];
    return h;
}

// 16-byte chunks per lane issued before the header is parsed (a lane-per-frame lane needs its
// first 64 bytes). Eight for groups would let a 570 B frame finish in one round trip, but costs
// ~55 VGPRs (occupancy 5 -> 3) and lost more than it gained; kept as a knob.
#ifndef HALO_RX_R0_G8
#define HALO_RX_R0_G8 4  // measurement knob: round-0 chunk rows of the 8-lane kernel
#endif
template <int G>
constexpr int kRound0 = G == 8 ? HALO_RX_R0_G8 : 4;
// One frame's state between "fetch" (addresses + round-0 loads issued) and "finish".
// Later-round loads of the widest groups (jumbo frames) are non-temporal: 9000 B frames 6.08-6.10
// -> 5.76 ms; for 1500 B on 8 lanes the same hint costs 12 % (290-296 -> 332 us), IMIX 2 %
// (profiles/r03/r3y/ab_nt.log: HALO_RX_LATER_NT_G 16 / off / 8, two rounds on one box).
#ifndef HALO_RX_LATER_NT_G
#define HALO_RX_LATER_NT_G 16
#endif
#ifndef HALO_RX_GROUP_XCD
#define HALO_RX_GROUP_XCD 8  // runs of this many blocks per XCD in the 4- and 8-lane kernels (0/1: off)
#endif
template <int G, int R0 = kRound0<G>>
struct FrameState {
    static constexpr int kR0 = R0;
    const uint8_t* frame;
    uint32_t L, ndw;
    uint32_t buf[R0][4];  // round 0: chunks (u*G + gl) of 16 bytes
};

template <int LAYOUT, typename FS>
__device__ __forceinline__ void frame_meta(const RxParams& p, uint64_t i, bool present, FS& st) {
    st.frame = p.bytes;
    st.L = 0;
    if (present) frame_at<LAYOUT>(p, i, st.frame, st.L);
    st.ndw = (present && len_readable<kL3<LAYOUT>>(st.L, p.flags)) ? (st.L + 3) >> 2 : 0;
}

// Round 0: four 16-byte chunks per lane issued back to back, bounded by the frame length (the
// L4 end is not known before the header is parsed, and never exceeds the frame length).
template <int G, int R0>
__device__ __forceinline__ void frame_loads(uint32_t gl, FrameState<G, R0>& st) {
#pragma unroll
    for (int u = 0; u < R0; ++u) load4(st.frame, (u * G + gl) * 4, st.ndw, st.buf[u]);
}

// Header dwords 0..11 of the frame: the lane's own chunks (G = 1) or chunk 0 of group lanes 0..2.
template <int G, int R0>
__device__ __forceinline__ void frame_header(const FrameState<G, R0>& st, uint32_t grp_base, uint32_t (&h)[12]) {
    if constexpr (G == 1) {
#pragma unroll
        for (int j = 0; j < 12; ++j) h[j] = st.buf[j >> 2][j & 3];
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            h[j] = group_bcast<G, 0>(st.buf[0][j], grp_base);
            h[4 + j] = group_bcast<G, 1>(st.buf[0][j], grp_base);
            h[8 + j] = group_bcast<G, 2>(st.buf[0][j], grp_base);
        }
    }
}

// Verdict after the L4 segment sum (this lane's or group's partial `c`), record store and count.
// `stage` (lane-per-frame only): write the record to this wave's LDS staging slot instead of
// global memory; the wave then stores its 64 consecutive records fully coalesced.
// FUSE (compile time, so the plain parse carries none of it): 1 = hash every record's NAT flow
// key (halo_rx_parse_flow_batch_device), 2 = FindRoute of every record's dst
// (halo_rx_parse_route_batch_device).
template <int G, int FUSE = 0, bool L3 = false>
__device__ __forceinline__ void frame_store(const RxParams& p, uint64_t i, bool present, uint32_t gl,
                                            const uint32_t (&h)[12], Verdict& v, uint64_t c, Hist& hist,
                                            uint4* stage = nullptr) {
    const uint32_t c32 = group_sum<G>(fold64(c));
    if (v.status == HALO_RX_OK && v.check_l4 && fold16(c32 + v.l4_extra) != 0xFFFFu) v.status = HALO_RX_L4_CKSUM;
    if (v.status == HALO_RX_OK && v.ip_proto != kIpUnknown) finish_l4<L3>(h, v);

    if (present && gl < 2) {
        uint4 lo, hi;
        lo.x = v.status | (v.flags << 8) | (v.ethertype << 16);
        lo.y = v.ip_proto | (v.l4_aux << 8) | (v.ip_total_len << 16);
        lo.z = v.src_ip;
        lo.w = v.dst_ip;
        hi.x = v.sport | (v.dport << 16);
        hi.y = v.pay_off | (v.pay_len << 16);
        hi.z = v.l4_seq;
        hi.w = v.l4_ack;
        if (p.flags & HALO_RX_RECORD_COMPACT) {  // halo_rx_record16_t
            if (gl == 0) {
                const uint32_t et_class = v.ethertype == kEthArp ? HALO_RX_F_ET_ARP
                                        : v.ethertype == kEthIpv6 ? HALO_RX_F_ET_IPV6
                                        : v.ethertype == kEthIeee8023 ? HALO_RX_F_ET_8023 : 0u;
                const uint4 r16 =
                    make_uint4(v.status | ((v.flags | et_class) << 8) | (v.ip_proto << 16) | (v.l4_aux << 24),
                               v.src_ip, v.dst_ip, hi.x);
                if constexpr (G == 1) {
                    if (stage) stage[0] = r16;
                    else reinterpret_cast<uint4*>(p.out)[i] = r16;
                } else {
                    reinterpret_cast<uint4*>(p.out)[i] = r16;
                }
            }
        } else if (G == 1 && stage) {
            stage[0] = lo;
            stage[1] = hi;
        } else {
            uint4* rec = reinterpret_cast<uint4*>(p.out + i);
            if constexpr (G == 1) {
                rec[0] = lo;
                rec[1] = hi;
            } else {  // lane 0 writes bytes 0..15, lane 1 bytes 16..31 (per-component select: no scratch)
                const bool h1 = gl != 0;
                rec[gl] = make_uint4(h1 ? hi.x : lo.x, h1 ? hi.y : lo.y, h1 ? hi.z : lo.z, h1 ? hi.w : lo.w);
            }
        }
        if (gl == 0 && p.hist) hist.add(v.status);
        if (FUSE == 1 && gl == 0) {  // the flow key from the record's own fields (flow_key.h)
            const uint64_t fh = flowkey::nat_hash(lo.y & 0xFFu, lo.z, lo.w, hi.x & 0xFFFFu, hi.x >> 16,
                                                  p.flow_kind, p.flow_nat);
            p.flow_hash[i] = fh;
            if (p.flow_bucket) p.flow_bucket[i] = (uint32_t)(fh % p.flow_buckets);  // hashmap/hashmap.go:64
        }
        if (FUSE == 2 && gl == 0)  // FindRoute(dst) (route_view.h)
            p.route_out[i] = find_route(LpmView{p.rt_tbl24, p.rt_tbl8, p.rt_lists, p.rt_ids}, lo.w);
    }
}

// Everything after round 0 for frame i on a group of G lanes (G = 1: one lane, no cross-lane
// traffic). Every lane of a group calls it with the same i / present (other groups may be doing
// the same for other frames); `present` false means "no frame": nothing is read or written,
// but the group still executes the collective steps.
#ifndef HALO_RX_LATER_CHUNKS
#define HALO_RX_LATER_CHUNKS 8
#endif
template <int G, int FUSE = 0, int U = HALO_RX_LATER_CHUNKS, int R0 = kRound0<G>, bool L3 = false>  // U: 16-byte chunks in flight per lane per later round
__device__ __forceinline__ void frame_finish(const RxParams& p, uint64_t i, bool present, uint32_t gl,
                                             uint32_t grp_base, FrameState<G, R0>& st, Hist& hist,
                                             uint4* stage = nullptr) {
    constexpr uint32_t STEP = 4 * G;  // dwords per group per load step
    constexpr int U0 = R0;            // chunks already loaded
    uint32_t h[12];
    frame_header(st, grp_base, h);
    uint64_t c = 0;
    uint32_t hs = 0;  // group kernels: halves sum of this lane's segment dwords
    if constexpr (G > 1) {
        // Round 0 is summed before the header checks run, so its buffers are dead during them (a
        // group kernel can then issue more of the frame in round 0). The segment end is the one
        // parse_header computes (IPv4 offset + totalLen) whenever the L4 sum decides the verdict;
        // for any other frame the sum is never read.
        const uint32_t tl = L3 ? bswap16(h[0] >> 16) : bswap16(h[4] & 0xFFFFu);
        acc_chunk<L3, true>(st.buf[0], gl * 4, kIpOff<L3> + tl, hs);
#pragma unroll
        for (int u = 1; u < U0; ++u) acc_chunk<L3>(st.buf[u], (u * G + gl) * 4, kIpOff<L3> + tl, hs);
    }
    Verdict v = parse_header<L3>(h, st.L, present, p);

    // L4 segment sum over [kIpOff + 20, seg_end): round 0 from registers, then U chunks per round
    if (v.seg_end && G == 1 && HALO_RX_LANE_DOT2) {
        uint32_t hs = 0;
        const int32_t e8 = (int32_t)(8u * v.seg_end);
#pragma unroll
        for (int u = 0; u < U0; ++u) acc_segment_dot2<L3>(st.buf[u], u * 4, e8, hs);
        const uint32_t seg_dw = (v.seg_end + 3) >> 2;
        for (uint32_t r0 = U0 * STEP; r0 < seg_dw; r0 += U * STEP) {
            uint32_t x[U][4];
#pragma unroll
            for (int u = 0; u < U; ++u) load4(st.frame, r0 + u * 4, seg_dw, x[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) acc_segment_dot2<L3>(x[u], r0 + u * 4, e8, hs);
        }
        c = hs;
    } else if (v.seg_end && G == 1) {
#pragma unroll
        for (int u = 0; u < U0; ++u) acc_segment<L3>(st.buf[u], u * 4, v.seg_end, c);
        const uint32_t seg_dw = (v.seg_end + 3) >> 2;
        for (uint32_t r0 = U0 * STEP; r0 < seg_dw; r0 += U * STEP) {
            uint32_t x[U][4];
#pragma unroll
            for (int u = 0; u < U; ++u) load4(st.frame, r0 + u * 4, seg_dw, x[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) acc_segment<L3>(x[u], r0 + u * 4, v.seg_end, c);
        }
    } else if constexpr (G > 1) {
        // later rounds: the group's loop bound is wave-uniform in practice (one length per batch),
        // and a group with no segment (or a frame not present) loads nothing
        const uint32_t seg_dw = v.seg_end ? (v.seg_end + 3) >> 2 : 0u;
        for (uint32_t r0 = U0 * STEP; r0 < seg_dw; r0 += U * STEP) {
            uint32_t x[U][4];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (G >= HALO_RX_LATER_NT_G) load4_nt(st.frame, r0 + (u * G + gl) * 4, seg_dw, x[u]);
                else load4(st.frame, r0 + (u * G + gl) * 4, seg_dw, x[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc_chunk<L3>(x[u], r0 + (u * G + gl) * 4, v.seg_end, hs);
        }
        c = hs;
    }
    frame_store<G, FUSE, L3>(p, i, present, gl, h, v, c, hist, stage);
}

// The whole chain for frame i on a group of G lanes: R0 chunks per lane in round 0, U per later round.
template <int G, int LAYOUT, int FUSE, int R0, int U>
__device__ __forceinline__ void process_frame(const RxParams& p, uint64_t i, bool present, uint32_t gl,
                                              uint32_t grp_base, Hist& hist) {
    FrameState<G, R0> st;
    frame_meta<LAYOUT>(p, i, present, st);
    frame_loads(gl, st);
    frame_finish<G, FUSE, U, R0, kL3<LAYOUT>>(p, i, present, gl, grp_base, st, hist);
}

// The block's counts reach the caller's counters through a two-level tree of partial histograms
// (p.hist, hist_trees) instead of device-scope atomics on the caller's 14 counters: those serialise
// at the memory side, ~10 ns each, and 16384 one-wave blocks cost 170 us on a 21 us launch (bench
// r4b). Every word of the tree is a 64-bit (arrivals << 40 | count) pair, one per status: block b
// adds (1 << 40 | its count) to status k of level-1 slot b % 1024 (16 blocks per slot for 1M
// frames), and the add that brings the arrivals to the slot's block count returns the slot's final
// count, so that thread alone moves it on — to level-2 slot (b % 1024) / 32, whose last arrival
// adds it to the caller's counter (at most 32 x 14 atomics on them per launch) — and zeroes the word
// for the next launch on the queue. Each word carries its own completion, so no fence is needed: a
// __threadfence per block (agent-scope release / acquire, L2 writeback and invalidate across the
// XCDs on gfx950) cost 0.55 ms per 1M-frame launch (bench r4i), and a separate finalize launch
// ~10 us (r4e). Every block of a kernel that counts calls this once, with the whole block.
// The tree is the one of the launch's HSA queue (halo_common.h): the words assume one launch at a
// time per tree, and the dispatch packet's barrier bit is what guarantees it.
#ifndef HALO_HIST_HDR
#define HALO_HIST_HDR 0  // measurement knob: 1 = every block re-reads its dispatch packet's barrier bit
#endif
// key0: the word at the queue's first probe slot as block thread 0 read it when the block started
// (Hist::key). A key never changes once set, so a stale copy can only read 0, and then the CAS
// (performed at memory) returns the real key.
// Called by the 64 lanes of wave 0 (every kernel that counts has blocks of whole waves, >= 64
// threads). Lane j reads probe slot k0 + j (kHistTrees == 64: every slot in one round trip); the
// first slot in probe order holding this queue's key is the tree; otherwise the slots read as free
// are claimed in probe order by lane 0, one CAS each, until one is this queue's. A queue that finds
// every key held by others (or poisoned) returns nullptr after that one round trip (16 serial probes
// before round 6).
static_assert(kHistTrees == 64, "one probe slot per lane of a wave");
__device__ __forceinline__ unsigned long long* launch_tree(uint32_t* set_u32, unsigned long long key0) {
#if HALO_HIST_HDR
    // 100 us per 1M-frame launch: the packet lives in host memory (bench_hist, profiles/r05)
    const uint16_t hdr = *static_cast<const uint16_t*>((const void*)__builtin_amdgcn_dispatch_ptr());
    if (!((hdr >> 8) & 1u)) return nullptr;  // HSA_PACKET_HEADER_BARRIER
#endif
    unsigned long long* set = reinterpret_cast<unsigned long long*>(set_u32);
    const unsigned long long q = launch_queue();
    const uint32_t k0 = tree_slot0(q), lane = threadIdx.x & 63u;
    const unsigned long long k0key =
        ((unsigned long long)(uint32_t)__shfl((int)(uint32_t)(key0 >> 32), 0, 64) << 32) |
        (uint32_t)__shfl((int)(uint32_t)key0, 0, 64);
    if (k0key == q) return set + kHistKeyWords + (uint64_t)k0 * kHistWords;  // uniform
    const unsigned long long key = set[(k0 + lane) & (kHistTrees - 1u)];
    const uint64_t mine = __ballot(key == q);
    if (mine) return set + kHistKeyWords + (uint64_t)((k0 + (uint32_t)__builtin_ctzll(mine)) & (kHistTrees - 1u)) * kHistWords;
    uint64_t free_slots = __ballot(key == 0);
    while (free_slots) {  // uniform
        const uint32_t k = (k0 + (uint32_t)__builtin_ctzll(free_slots)) & (kHistTrees - 1u);
        unsigned long long got = 0;
        if (lane == 0) {  // claim it (device scope: a native compare-and-swap, no retry loop)
            __hip_atomic_compare_exchange_strong(set + k, &got, q, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
        }
        got = ((unsigned long long)(uint32_t)__shfl((int)(uint32_t)(got >> 32), 0, 64) << 32) |
              (uint32_t)__shfl((int)(uint32_t)got, 0, 64);
        if (got == 0 || got == q) return set + kHistKeyWords + (uint64_t)k * kHistWords;  // claimed now / by a sibling block
        free_slots &= free_slots - 1;  // another queue's key (our read was stale): the next free slot
    }
    return nullptr;  // every key taken by another queue, or poisoned (hist_trees: no barrier bits)
}

__device__ __forceinline__ void flush_hist(const RxParams& p, Hist& hist) {
    if (!p.hist) return;
    const uint32_t t = threadIdx.x;
    uint32_t ok = hist.ok;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) ok += __shfl_xor(ok, m, 64);
    if ((threadIdx.x & 63u) == 0 && ok) atomicAdd(&hist.s[HALO_RX_OK], ok);
    __syncthreads();
    if (t >= 64) return;
    unsigned long long* tree = launch_tree(p.hist, hist.key);  // wave 0: one probe round trip for the block
    if (t >= HALO_RX_STATUS_COUNT) return;
    const uint32_t s = blockIdx.x & (kHistSlots - 1u), g = gridDim.x;
    if (!tree) {  // no tree this launch can own alone: straight into the caller's counters
        if (hist.s[t]) atomicAdd(&p.hist_out[t], hist.s[t]);
        return;
    }
    // What it costs is a fixed tail per launch, not a per-block price (two-level tree: 1M frames
    // +2.7 us, 4M +2.4, 16M +1.4; counting, the LDS adds and the barrier alone +0.4): the last
    // block's chain of dependent round trips. Arrivals in one word with only the statuses a block saw
    // ran 0.6 us slower; one level of 64 / 256 / 1024 slots strided over the grid ran +0.3 / +1.3 / +9
    // us (their completers all finish at the end and queue on one counter, ~10 ns an add). Runs of
    // consecutive blocks complete through the launch instead. DESIGN.md §14.5.
    constexpr unsigned long long kOne = 1ull << 40, kCount = kOne - 1;
#ifndef HALO_HIST_RUNS
#define HALO_HIST_RUNS 16  // 0: off. 1M x 64 B: +1.8-2.0 us against +2.1-2.4 for the two-level tree;
#endif                     // runs of 8: +5.6, of 32: +1.8-2.0 (profiles/r05/r5zz2)
    if (HALO_HIST_RUNS && g <= kHistSlots * (uint32_t)(HALO_HIST_RUNS ? HALO_HIST_RUNS : 1)) {  // uniform
        // Grids up to 16384 blocks: slot = a run of 16 consecutive blocks. Workgroups are dispatched
        // in order, so the runs complete one after another through the launch instead of all at its
        // end, and each completer adds straight into the caller's counters (one level: the adds
        // arrive spread out, not queued on one counter at the tail).
        constexpr uint32_t R = HALO_HIST_RUNS ? HALO_HIST_RUNS : 1;
        const uint32_t r = blockIdx.x / R;
        unsigned long long* w = tree + r * kHistStride + t;
        const unsigned long long add = kOne | hist.s[t];
        const unsigned long long now1 = atomicAdd(w, add) + add;
        if ((now1 >> 40) != (g - r * R < R ? g - r * R : R)) return;
        atomicExch(w, 0ull);
        if (now1 & kCount) atomicAdd(&p.hist_out[t], (uint32_t)(now1 & kCount));
        return;
    }
    unsigned long long* l1 = tree + s * kHistStride + t;
    unsigned long long now = atomicAdd(l1, kOne | hist.s[t]) + (kOne | hist.s[t]);
    if ((now >> 40) != g / kHistSlots + (g % kHistSlots > s)) return;
    atomicExch(l1, 0ull);
    const uint32_t used = g < kHistSlots ? g : kHistSlots, first = s & ~(kHistFan - 1u);
    unsigned long long* l2 = tree + (kHistSlots + s / kHistFan) * kHistStride + t;
    now = atomicAdd(l2, kOne | (now & kCount)) + (kOne | (now & kCount));
    if ((now >> 40) != (used - first < kHistFan ? used - first : kHistFan)) return;
    atomicExch(l2, 0ull);
    if (now & kCount) atomicAdd(&p.hist_out[t], (uint32_t)(now & kCount));
}

// Uniform batches: G lanes per frame for every frame (G in {1,4,8,16}); 64/G frames per wave.
template <int G, int LAYOUT, int FUSE, int R0 = kRound0<G>, int U = HALO_RX_LATER_CHUNKS>
__device__ __forceinline__ void group_kernel_body(const RxParams& p) {
    constexpr uint32_t FPW = 64 / G;  // frames per wave
    __shared__ uint32_t s_hist[HALO_RX_STATUS_COUNT];
    if (threadIdx.x < HALO_RX_STATUS_COUNT) s_hist[threadIdx.x] = 0;
    __syncthreads();
    Hist hist = hist_open(p, s_hist);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp_base = lane & ~(uint32_t)(G - 1);
    // frame indices fit in 32 bits (n is a u32): 32-bit loop state keeps the SGPR budget low
    // Blocks are dealt round-robin over the 8 XCDs, so neighbouring waves sit on different XCDs and
    // the 128-byte line two neighbouring frames share is fetched into two L2s: 1500 B frames read
    // 1.033x their bytes. Runs of R consecutive blocks per XCD, the XCDs taking runs in turn, keep
    // all but one wave boundary in 4R inside one L2 and still sweep the batch in order: R = 8 reads
    // 1.013x at the same time (r5p/r5q: R = 4 / 8 / 16 / 64 read 1.017 / 1.013 / 1.012 / 1.011x; one
    // contiguous range per XCD read 1.011x but ran 4 % slower). Not for 16 lanes per frame: jumbo
    // frames share a line in 9000 B and ran 0.5 % slower with it.
    uint32_t lblock = blockIdx.x;
    if constexpr (G <= 8 && HALO_RX_GROUP_XCD > 1) {
        constexpr uint32_t R = HALO_RX_GROUP_XCD;
        const uint32_t b = blockIdx.x, grp = b / (8 * R);
        if ((grp + 1) * 8 * R <= gridDim.x) lblock = grp * 8 * R + (b & 7u) * R + (b >> 3) % R;
    }
    const uint32_t wave = (lblock * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t base = wave * FPW; base < p.n; base += nwaves * FPW) {
        const uint32_t i = base + lane / G;
        process_frame<G, LAYOUT, FUSE, R0, U>(p, i, i < p.n, gl, grp_base, hist);
    }
    flush_hist(p, hist);
}

// Lane per frame. The build lands at 76 VGPRs = 6 waves per SIMD; forcing 7 (72 VGPRs) or 8
// (64, with scratch spills) was not faster (profiles/r01/ab_r2o_lane_waves.log: 22.2 / 27.8 µs vs
// 21.9 µs on config 2), so the knob HALO_RX_LANE_WAVES stays off. A wave's 64 records are
// consecutive: they are staged in LDS and written with fully coalesced 16-byte stores (a lane
// writing its own 32 B record at a 32 B stride stored the same bytes 25 % slower:
// profiles/r01/probe_store_patterns.log).
// One wave's window of 64 consecutive frames, a lane each (frames base .. base + 63): parse, stage
// the 64 records in the wave's LDS (s_rec_w: 128 x 16 B) and store them fully coalesced.
template <int LAYOUT, int FUSE>
__device__ __forceinline__ void lane_window_finish(const RxParams& p, uint32_t base, uint32_t lane, FrameState<1>& st,
                                                   uint4* s_rec_w, Hist& hist);
template <int LAYOUT, int FUSE>
__device__ __forceinline__ void lane_window(const RxParams& p, uint32_t base, uint32_t lane, uint4* s_rec_w,
                                           Hist& hist) {
    const uint32_t i = base + lane;
    FrameState<1> st;
    frame_meta<LAYOUT>(p, i, i < p.n, st);
    frame_loads<1>(0, st);
    lane_window_finish<LAYOUT, FUSE>(p, base, lane, st, s_rec_w, hist);
}

#ifndef HALO_RX_LANE_WAVES
#define HALO_RX_LANE_WAVES 0
#endif
// Prefetching the next group's address/length in waves that loop: no gain at 1M (22.0 vs 22.1
// us) and 3 % slower at 16M; with capped grids 2-11 % slower (profiles/r02/ab_lane_prefetch.log).
#ifndef HALO_RX_LANE_PREFETCH
#define HALO_RX_LANE_PREFETCH 0
#endif
// Threads per block of the lane kernel (64, 128 or 256) and 16-byte chunks per lane in its later
// load rounds (frames > 64 B only). One-wave blocks with 4.5 KB of LDS padding (22 blocks =
// 5.5 waves per SIMD resident, against 6 by registers) beat 256-thread blocks at every size
// measured: 1M x 64 B 22.2 -> 21.5 us, 16M x 64 B 321 -> 313 us, 128 B 49.8 -> 49.3 us
// (profiles/r02/lane_ab/: fewer frame bytes in flight per CU stream faster
// from HBM; occupancy 8 (LATER 4: 60 VGPRs) was 2-8 % slower, 4 waves 2-9 % slower).
#ifndef HALO_RX_LANE_BLOCK
#define HALO_RX_LANE_BLOCK 64
#endif
#ifndef HALO_RX_LANE_LATER
#define HALO_RX_LANE_LATER HALO_RX_LATER_CHUNKS
#endif
// A/B knobs: dynamic LDS bytes per lane-kernel block (caps resident blocks per CU, i.e. the
// frame bytes in flight), and XCD-contiguous block order (blocks b, b+8, ... share an XCD; with
// the remap each XCD's blocks take one contiguous range of the batch).
#ifndef HALO_RX_LANE_LDS_PAD
#define HALO_RX_LANE_LDS_PAD 4608
#endif
#ifndef HALO_RX_LANE_XCD
#define HALO_RX_LANE_XCD 0
#endif
template <int LAYOUT, int FUSE>
__device__ __forceinline__ void lane_window_finish(const RxParams& p, uint32_t base, uint32_t lane, FrameState<1>& st,
                                                   uint4* s_rec_w, Hist& hist) {
    const bool compact = (p.flags & HALO_RX_RECORD_COMPACT) != 0;
    const uint32_t i = base + lane;
    frame_finish<1, FUSE, HALO_RX_LANE_LATER, kRound0<1>, kL3<LAYOUT>>(p, i, i < p.n, 0, lane, st, hist,
                                                                     &s_rec_w[compact ? lane : 2 * lane]);
    __builtin_amdgcn_wave_barrier();
    const uint32_t nrec = p.n - base < 64 ? p.n - base : 64;  // records of this wave
    if (compact) {
        if (lane < nrec) store16(reinterpret_cast<uint4*>(p.out) + base + lane, s_rec_w[lane]);
    } else {
        uint4* out4 = reinterpret_cast<uint4*>(p.out) + 2ull * base;
        if (lane < 2 * nrec) store16(out4 + lane, s_rec_w[lane]);
        if (64 + lane < 2 * nrec) store16(out4 + 64 + lane, s_rec_w[64 + lane]);
    }
    __builtin_amdgcn_wave_barrier();
}

template <int LAYOUT, int FUSE>
__global__ void __launch_bounds__(HALO_RX_LANE_BLOCK) __attribute__((amdgpu_num_sgpr(80)))
#if HALO_RX_LANE_WAVES
__attribute__((amdgpu_waves_per_eu(HALO_RX_LANE_WAVES)))
#endif
rx_lane_kernel(const RxParams p) {
    __shared__ uint32_t s_hist[HALO_RX_STATUS_COUNT];
    __shared__ uint4 s_rec[HALO_RX_LANE_BLOCK / 64][128];  // per wave: 64 records of 32 B
    if (threadIdx.x < HALO_RX_STATUS_COUNT) s_hist[threadIdx.x] = 0;
    __syncthreads();
    Hist hist = hist_open(p, s_hist);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = threadIdx.x >> 6;
#if HALO_RX_LANE_XCD
    const uint32_t nb = gridDim.x, per = nb >> 3, rem = nb & 7u, xcd = blockIdx.x & 7u;
    const uint32_t lblock = (xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per) + (blockIdx.x >> 3);
    const uint32_t wave = (lblock * blockDim.x + threadIdx.x) >> 6;
#else
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
#endif
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
#if HALO_RX_LANE_PREFETCH
    // the next group's address and length load while this group is parsed (waves that loop)
    FrameState<1> nx;
    frame_meta<LAYOUT>(p, wave * 64 + lane, wave * 64 + lane < p.n, nx);
#endif
    for (uint32_t base = wave * 64; base < p.n; base += nwaves * 64) {
#if HALO_RX_LANE_PREFETCH
        const uint32_t i = base + lane;
        FrameState<1> st;
        st.frame = nx.frame; st.L = nx.L; st.ndw = nx.ndw;
        frame_loads<1>(0, st);
        frame_meta<LAYOUT>(p, i + nwaves * 64, i + nwaves * 64 < p.n, nx);
        lane_window_finish<LAYOUT, FUSE>(p, base, lane, st, s_rec[w], hist);
#else
        lane_window<LAYOUT, FUSE>(p, base, lane, s_rec[w], hist);
#endif
    }
    flush_hist(p, hist);
}

// Several batches in one launch (halo_rx_parse_batches_device): the batch stream of the reference's
// unbounded poll loop (engine/engine.go:344-351) handed over K batches at a time. A 1M-frame launch
// spends a fixed ramp and tail filling and draining 256 CUs — config 2 ran at 0.62 of 8 TB/s while
// the same kernel reached 0.74 on 16M frames — so the K batches' 64-frame windows are
// one grid: window w belongs to the batch whose cumulative window count first exceeds w (a
// wave-uniform scan over <= kMultiMax kernel arguments), and each wave runs the lane kernel's window
// code on that batch's arrays. Records, histogram and read contract are those of K separate launches.
constexpr uint32_t kMultiMax = 32;
struct MultiParams {
    RxParams p;  // the shared fields (flags, netif, histogram); per-batch arrays below
    uint32_t k;
    uint32_t win_end[kMultiMax];  // windows of batches 0..b
    uint32_t n[kMultiMax];
    const uint8_t* bytes[kMultiMax];
    const uint32_t* offsets_dw[kMultiMax];
    const uint16_t* lens[kMultiMax];
    halo_rx_result_t* out[kMultiMax];
};

template <int LAYOUT>
__global__ void __launch_bounds__(HALO_RX_LANE_BLOCK) rx_lane_multi_kernel(const MultiParams mp) {
    __shared__ uint32_t s_hist[HALO_RX_STATUS_COUNT];
    __shared__ uint4 s_rec[HALO_RX_LANE_BLOCK / 64][128];
    if (threadIdx.x < HALO_RX_STATUS_COUNT) s_hist[threadIdx.x] = 0;
    __syncthreads();
    Hist hist = hist_open(mp.p, s_hist);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const uint32_t total = mp.win_end[mp.k - 1];
    for (uint32_t win = wave; win < total; win += nwaves) {
        uint32_t b = 0;
        while (win >= mp.win_end[b]) ++b;  // k <= 32, uniform across the wave
        RxParams p = mp.p;
        p.bytes = mp.bytes[b];
        p.offsets_dw = mp.offsets_dw[b];
        p.lens = mp.lens[b];
        p.out = mp.out[b];
        p.n = mp.n[b];
        const uint32_t base = (win - (b ? mp.win_end[b - 1] : 0u)) * 64u;
        lane_window<LAYOUT, 0>(p, base, lane, s_rec[w], hist);
    }
    flush_hist(mp.p, hist);
}

// The resident small-poll consumer (RingServiceCtl, halo_common.h), kSvcGroups workgroups of
// kSvcWaves waves. In each group wave 0 waits for a request: all its lanes load the request line
// (one 64-byte read of pinned host memory, system scope), s_sleep between tries, bounded by the
// stop flag and an idle timeout on the 100 MHz real-time counter, so every wave reaches the exit.
// A new req_seq whose check matches the fields of the same read is taken (the fields arrive with
// the sequence number: no second round trip); an acquire fence, then the group's waves parse their
// 64-frame windows (window k goes to group k % kSvcGroups, spreading a 1k-frame request over 8
// CUs' memory pipelines) with the lane kernel's window code; after a block barrier thread 0 fences
// and publishes the group's done_seq slot. Measured on one box (profiles/r03/r3j/ab_svc.log, 1 /
// 1000 frames per poll): 1 group x 16 waves 17.5 us at 1000; 8 x 8 9.2 / 11.8-12.6 us; 16 x 4
// 10.3 / 13.2-13.9; 32 x 2 16.5 / 20.4. Rejected: each group also reading its window's lengths
// with the request (offsets derived in-wave, no metadata read after the request: 11.5 / 13.3-13.6,
// the wider poll read cost more than the read it saved), and four poll reads in flight per group
// (profiles/r03/r3h: 25.9 us at 1000: the reads queued ahead of the frame reads).
// Idle exit is one decision for the grid: the first group whose timer runs out sets *quit (device
// memory) and every other group leaves at its next empty read of the request line, so a request
// that races the exit finds the whole kernel gone (the host relaunches within microseconds) rather
// than some groups alive for another 20 ms. Requests whose flags carry
// HALO_RX_L3_START (a LoChan drain through a host context) take the L3 layout.
__global__ void __launch_bounds__(64 * kSvcWaves) ring_service_kernel(RingServiceCtl* ctl, const uint8_t* data,
                                                                      const uint32_t* off, const uint16_t* len,
                                                                      uint32_t* quit_all, uint32_t last,
                                                                      uint64_t idle_ticks) {
    __shared__ uint32_t s_cmd[12];  // seq, exit, n, flags, mac_lo, mac_hi, own_ip, out_lo, out_hi, uni_off/stride/len
    __shared__ uint32_t s_hist[HALO_RX_STATUS_COUNT];
    __shared__ uint4 s_rec[kSvcWaves][128];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, g = blockIdx.x;
    uint32_t* line = reinterpret_cast<uint32_t*>(ctl);
    if (threadIdx.x < HALO_RX_STATUS_COUNT) s_hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) __hip_atomic_store(&ctl->alive[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint64_t t_idle = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (w == 0) {
            uint32_t v, seq, quit = 0;
            for (;;) {
                v = __hip_atomic_load(&line[lane & 15u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                seq = __builtin_amdgcn_readlane(v, 0);
                if (seq != last) {
                    const uint32_t ck = svc_check(seq, __builtin_amdgcn_readlane(v, 1), __builtin_amdgcn_readlane(v, 2),
                                                  __builtin_amdgcn_readlane(v, 3), __builtin_amdgcn_readlane(v, 4),
                                                  __builtin_amdgcn_readlane(v, 5), __builtin_amdgcn_readlane(v, 6),
                                                  __builtin_amdgcn_readlane(v, 7), __builtin_amdgcn_readlane(v, 10),
                                                  __builtin_amdgcn_readlane(v, 11), __builtin_amdgcn_readlane(v, 12));
                    if (ck == __builtin_amdgcn_readlane(v, 9)) break;
                }
                const uint32_t others = __hip_atomic_load(quit_all, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__builtin_amdgcn_readlane(v, 8) || others) {
                    quit = 1;
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t_idle > idle_ticks) {
                    if (lane == 0) __hip_atomic_store(quit_all, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    quit = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0) {
                s_cmd[0] = seq;
                s_cmd[1] = quit;
                s_cmd[2] = __builtin_amdgcn_readlane(v, 1);
                s_cmd[3] = __builtin_amdgcn_readlane(v, 2);
                s_cmd[4] = __builtin_amdgcn_readlane(v, 3);
                s_cmd[5] = __builtin_amdgcn_readlane(v, 4);
                s_cmd[6] = __builtin_amdgcn_readlane(v, 5);
                s_cmd[7] = __builtin_amdgcn_readlane(v, 6);
                s_cmd[8] = __builtin_amdgcn_readlane(v, 7);
                s_cmd[9] = __builtin_amdgcn_readlane(v, 10);
                s_cmd[10] = __builtin_amdgcn_readlane(v, 11);
                s_cmd[11] = __builtin_amdgcn_readlane(v, 12);
                if (!quit) ctl->t_seen[g] = __builtin_amdgcn_s_memrealtime();
            }
            // the request's off / len / frames are read after the request was seen
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        }
        __syncthreads();
        if (s_cmd[1]) break;
        RxParams p{};
        p.bytes = data;
        p.offsets_dw = off;
        p.lens = len;
        p.n = s_cmd[2];
        p.flags = s_cmd[3];
        p.mac_lo = s_cmd[4];
        p.mac_hi = s_cmd[5];
        p.own_ip = s_cmd[6];
        p.out = reinterpret_cast<halo_rx_result_t*>((uint64_t)s_cmd[7] | ((uint64_t)s_cmd[8] << 32));
        Hist hist{s_hist, 0, 0};  // the consumer keeps no histogram
        if (s_cmd[11]) {  // one length, consecutive records: the strided layout, no array reads
            p.bytes = data + 4ull * s_cmd[9];
            p.stride = 4ull * s_cmd[10];
            p.len = s_cmd[11];
            for (uint32_t base = (w * kSvcGroups + g) * 64; base < p.n; base += kSvcGroups * kSvcWaves * 64)
                lane_window<2, 0>(p, base, lane, s_rec[w], hist);
        } else if (p.flags & HALO_RX_L3_START) {
            for (uint32_t base = (w * kSvcGroups + g) * 64; base < p.n; base += kSvcGroups * kSvcWaves * 64)
                lane_window<3, 0>(p, base, lane, s_rec[w], hist);
        } else {
            for (uint32_t base = (w * kSvcGroups + g) * 64; base < p.n; base += kSvcGroups * kSvcWaves * 64)
                lane_window<0, 0>(p, base, lane, s_rec[w], hist);
        }
        __syncthreads();  // every record of this group stored
        if (threadIdx.x == 0) {
            ctl->t_done[g] = __builtin_amdgcn_s_memrealtime();
            __threadfence_system();
            __hip_atomic_store(&ctl->done_seq[g], s_cmd[0], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        last = s_cmd[0];
        t_idle = __builtin_amdgcn_s_memrealtime();
        __syncthreads();  // s_cmd is rewritten by the next wait
    }
    if (threadIdx.x == 0) __hip_atomic_store(&ctl->alive[g], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// G lanes per frame (G in {4, 8, 16}); VGPR-limited occupancy, so no SGPR cap.
#ifndef HALO_RX_GROUP_WAVES
#define HALO_RX_GROUP_WAVES 5
#endif
// A/B knobs: threads per block and dynamic LDS padding per block (caps resident blocks per CU).
#ifndef HALO_RX_GROUP_BLOCK
#define HALO_RX_GROUP_BLOCK 256
#endif
#ifndef HALO_RX_GROUP_LDS_PAD
#define HALO_RX_GROUP_LDS_PAD 0
#endif
template <int G, int LAYOUT, int FUSE>
__global__ void __launch_bounds__(HALO_RX_GROUP_BLOCK) __attribute__((amdgpu_waves_per_eu(HALO_RX_GROUP_WAVES)))
rx_group_kernel(const RxParams p) {
    static_assert(G == 4 || G == 8 || G == 16, "G must be 4, 8 or 16");
    group_kernel_body<G, LAYOUT, FUSE>(p);
}

// Mixed sizes (IMIX): each wave takes a window of 256 consecutive frames (four per lane), sorts
// them by size class into LDS (ballot ranks; the frame address and length travel with the
// entry, so nothing is re-loaded), then runs one pass per class with the lanes-per-frame that
// the uniform sweep found best for that size: <= 128 B (and frames failing the length check)
// lane per frame, <= 1024 B 4 lanes, <= 4096 B 8 lanes, longer 16 lanes. Every pass keeps all
// groups busy with frames of one class, so no lane waits behind a longer neighbour.
#ifndef HALO_RX_MIX_WINDOW
#define HALO_RX_MIX_WINDOW 256
#endif
constexpr uint32_t kMixWindow = HALO_RX_MIX_WINDOW;  // frames per wave window (a multiple of 64)
constexpr int kMixPer = (int)(kMixWindow / 64);      // frames per lane in the classification
#ifndef HALO_RX_MIX_MAX_G
#define HALO_RX_MIX_MAX_G 16  // 8: frames > 4096 B take the 8-lane pass (no 16-lane pass compiled)
#endif

// Later-round chunks per lane in the mix passes: just enough for each class's size range in one
// later round trip (<= 128 B: 64 + 4*16 B; 570 B on 4 lanes: 256 + 5*64 B; 1500 B on 8 lanes:
// 512 + 8*128 B), so the short classes' passes do not hold the buffers the long ones need.
// IMIX 1.60 -> 1.58 ms, 570 B 150 -> 147 us (profiles/r01/ab_r43_mix_later_small.log, 5 vs 6
// chunks for 570 B: ab_r43_mix_later_g4.log).
#ifndef HALO_RX_MIX_LATER_SMALL
#define HALO_RX_MIX_LATER_SMALL 1
#endif
#ifndef HALO_RX_MIX_LATER_G4
#define HALO_RX_MIX_LATER_G4 5
#endif
template <int G>
constexpr int kMixLater = !HALO_RX_MIX_LATER_SMALL ? HALO_RX_LATER_CHUNKS
                        : G == 1 ? 4 : G == 4 ? HALO_RX_MIX_LATER_G4 : HALO_RX_LATER_CHUNKS;

// Round-0 chunks per lane in the mix passes (HALO_RX_MIX_ROUND0=1): 570 B on 4 lanes in one round
// trip (9 x 64 B >= 576 B), 1500 B on 8 lanes in one (12 x 128 B >= 1536 B). Off: the bigger round
// 0 spills at occupancy 4 (IMIX 2.06 ms) and at occupancy 3 is slower still than two round trips
// (IMIX 1.69 ms, 570 B 173 us; profiles/r01/ab_r43_mix_round0_rejected.log).
#ifndef HALO_RX_MIX_ROUND0
#define HALO_RX_MIX_ROUND0 0
#endif
template <int G>
constexpr int kMixRound0 = !HALO_RX_MIX_ROUND0 ? kRound0<G> : G == 4 ? 9 : G == 8 && HALO_RX_MIX_ROUND0 >= 2 ? 12 : kRound0<G>;

template <int G, int FUSE, bool L3>
__device__ __forceinline__ void mix_pass(const RxParams& p, uint32_t e_begin, uint32_t e_end, uint32_t lane,
                                         const uint64_t* s_ptr, const uint32_t* s_idx, const uint16_t* s_len,
                                         uint32_t len_max, Hist& hist) {
    constexpr uint32_t FPW = 64 / G;
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp_base = lane & ~(uint32_t)(G - 1);
    for (uint32_t e0 = e_begin; e0 < e_end; e0 += FPW) {
        const uint32_t e = e0 + lane / G;
        const bool has = e < e_end;
        FrameState<G, kMixRound0<G>> st;
        st.frame = has ? reinterpret_cast<const uint8_t*>(s_ptr[e]) : p.bytes;
        st.L = has ? s_len[e] : 0u;
        st.ndw = (has && st.L >= (L3 ? 20u : kEthMin) && st.L <= len_max) ? (st.L + 3) >> 2 : 0;
        frame_loads(gl, st);
        frame_finish<G, FUSE, kMixLater<G>, kMixRound0<G>, L3>(p, has ? s_idx[e] : 0u, has, gl, grp_base, st, hist);
    }
}

template <int LAYOUT, int FUSE>
#ifndef HALO_RX_MIX_WAVES
#define HALO_RX_MIX_WAVES 4
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HALO_RX_MIX_WAVES))) rx_mix_kernel(const RxParams p) {
    __shared__ uint32_t s_hist[HALO_RX_STATUS_COUNT];
    __shared__ uint64_t s_ptr[4][kMixWindow];
    __shared__ uint32_t s_idx[4][kMixWindow];
    __shared__ uint16_t s_len[4][kMixWindow];
    if (threadIdx.x < HALO_RX_STATUS_COUNT) s_hist[threadIdx.x] = 0;
    __syncthreads();
    Hist hist = hist_open(p, s_hist);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = threadIdx.x >> 6;
    constexpr bool L3 = kL3<LAYOUT>;
    const bool jumbo = (p.flags & HALO_RX_JUMBO_EXT) != 0;
    const uint32_t len_max = L3 ? (jumbo ? kIpMaxJumbo : kIpMax) : (jumbo ? kEthMaxJumbo : kEthMax);
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t base = wave * kMixWindow; base < p.n; base += nwaves * kMixWindow) {
        // classify: frame base + 64k + lane, k < kMixPer
        const uint8_t* fp[kMixPer];
        uint32_t fl[kMixPer], cls[kMixPer];
#pragma unroll
        for (int k = 0; k < kMixPer; ++k) {
            const uint32_t i = base + 64 * k + lane;
            fp[k] = p.bytes;
            fl[k] = 0;
            if (i < p.n) frame_at<LAYOUT>(p, i, fp[k], fl[k]);
            cls[k] = i >= p.n ? 4u
                   : (fl[k] <= 128 || fl[k] > len_max) ? 0u
                   : fl[k] <= 1024 ? 1u : (HALO_RX_MIX_MAX_G < 16 || fl[k] <= 4096) ? 2u : 3u;
        }
        // counting sort by class: one ballot live at a time
        uint32_t pos[kMixPer];
        uint32_t start[5];
        uint32_t run = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            start[c] = run;
#pragma unroll
            for (int k = 0; k < kMixPer; ++k) {
                const uint64_t b = __ballot(cls[k] == (uint32_t)c);
                if (cls[k] == (uint32_t)c)
                    pos[k] = run + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
                run += (uint32_t)__popcll(b);
            }
        }
        start[4] = run;
#pragma unroll
        for (int k = 0; k < kMixPer; ++k) {
            if (cls[k] < 4u) {
                s_ptr[w][pos[k]] = reinterpret_cast<uint64_t>(fp[k]);
                s_idx[w][pos[k]] = base + 64 * k + lane;
                s_len[w][pos[k]] = (uint16_t)fl[k];
            }
        }
        const uint32_t st0 = start[0], st1 = start[1], st2 = start[2], st3 = start[3], nall = start[4];
        __builtin_amdgcn_wave_barrier();
        mix_pass<1, FUSE, L3>(p, st0, st1, lane, s_ptr[w], s_idx[w], s_len[w], len_max, hist);
        mix_pass<4, FUSE, L3>(p, st1, st2, lane, s_ptr[w], s_idx[w], s_len[w], len_max, hist);
        mix_pass<8, FUSE, L3>(p, st2, st3, lane, s_ptr[w], s_idx[w], s_len[w], len_max, hist);
        if constexpr (HALO_RX_MIX_MAX_G >= 16)
            mix_pass<16, FUSE, L3>(p, st3, nall, lane, s_ptr[w], s_idx[w], s_len[w], len_max, hist);
        __builtin_amdgcn_wave_barrier();
    }
    flush_hist(p, hist);
}

// ---- Byte-stream kernel (ragged batches of mixed sizes, DESIGN.md §4.3 "stream").
// A wave takes a window of 64 consecutive frames, one per lane. Each lane reads its frame's
// 48-byte header and runs the header checks (as the lane kernel). The L4 segment sums then come
// from ONE coalesced pass over the window's bytes: the wave streams [min segment start, max
// segment end) in 4 KB steps (64 contiguous bytes per lane), and a running prefix P of the
// 16-bit halves of every dword gives each frame's sum as P(end) - P(start). Halves sums keep the
// sum's value mod 0xFFFF and its zero-ness, which is all fold16 looks at; the u32 difference is
// exact for any segment (< 2^32 whatever the prefix wraps to). So every byte of a window is
// fetched once, in full 128-byte lines, whatever the sizes, and no lane waits on a longer
// neighbour. The step's bytes and its prefix at each 16-byte sub-chunk go to LDS; a lane whose
// segment starts or ends in the step reads its prefix back from there. A window whose frames are
// not dense in memory (span > 2 x their segment bytes + 8 KB, or a 4 KB page of the span holding
// no frame byte: window_pages_covered) sums each frame on its own lane.
constexpr uint32_t kStreamStep = 4096;  // bytes per wave per step: 64 lanes x 64 B

template <typename Op>
__device__ __forceinline__ uint32_t wave_allreduce(uint32_t x, Op op) {
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppHalfMirror, 0xF, 0xF, false));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppMirror, 0xF, 0xF, false));
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 0), r1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 16);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 32), r3 = (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
    return op(op(r0, r1), op(r2, r3));
}

// Exclusive prefix sum of x over the wave (lane order) and the wave total: row scans over DPP
// row_shr, row totals by v_readlane.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t lane, uint32_t& total) {
    uint32_t v = x;
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15), r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47), r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
    total = r0 + r1 + r2 + r3;
    const uint32_t row = lane >> 4;
    const uint32_t off = row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r0 + r1 : r0 + r1 + r2;
    return v + off - x;
}

// one dword's two 16-bit halves added to acc (v_dot2_u32_u16)
__device__ __forceinline__ uint32_t halves_acc(uint32_t w, uint32_t acc) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 one = {1, 1};
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w), one, acc, false);
}

// P at step byte r, counting nb (0..4) bytes of the dword holding r: the sub-chunk's base plus
// the halves of its dwords below r's and of the low nb bytes of r's own.
__device__ __forceinline__ uint32_t stream_prefix(const uint32_t* s_base, const uint4* s_x, uint32_t r, uint32_t nb) {
    const uint32_t k = r >> 4, j = (r >> 2) & 3u;
    const uint4 q = s_x[k];
    const uint32_t part = nb >= 4 ? 0xFFFFFFFFu : (1u << (8 * nb)) - 1u;
    uint32_t acc = s_base[k];
    acc = halves_acc(q.x & (j > 0 ? 0xFFFFFFFFu : part), acc);
    acc = halves_acc(q.y & (j > 1 ? 0xFFFFFFFFu : j == 1 ? part : 0u), acc);
    acc = halves_acc(q.z & (j > 2 ? 0xFFFFFFFFu : j == 2 ? part : 0u), acc);
    return halves_acc(q.w & (j == 3 ? part : 0u), acc);
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Stream origin alignment (bytes; the first step starts at the window's lowest byte rounded
// down to it). Measured and removed (profiles/r02/stream/stream1-3.log): software-pipelining the
// step loads (+16 VGPRs: 570 B 132 -> 156 us), issuing the next step's loads before this step's
// lookups, and prefetching the next window's addresses / headers (neutral or slower).
#ifndef HALO_RX_STREAM_ALIGN
#define HALO_RX_STREAM_ALIGN 128
#endif

// This lane's 64 bytes of the step at s0 (sub-chunk u at s0 + 1024u + 16 lane, so each load
// instruction reads 1 KB contiguous): always four 16-byte loads, no branch, so the load counter
// stays exact across steps. Positions are 16-byte aligned in memory and a window streams only
// when every page of [lo, hi) holds a frame dword (window_pages_covered), so every block in
// [lo, hi) is readable; a sub-chunk wholly outside reads the nearest such block instead. Bytes
// outside the frames are never inside a segment or header, and P differences cancel them.
__device__ __forceinline__ void stream_load(uint64_t B, uint32_t s0, uint32_t lane, uint32_t lo, uint32_t hi,
                                            uint32_t (&x)[4][4]) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(16)));
    const uint32_t first = lo & ~15u, last = (hi - 1u) & ~15u;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        uint32_t a = s0 + 1024u * u + 16 * lane;
        a = a < first ? first : a > last ? last : a;
        const u32x4 q = *(const __attribute__((address_space(1))) u32x4*)(B + a);
        x[u][0] = q.x; x[u][1] = q.y; x[u][2] = q.z; x[u][3] = q.w;
    }
}

// The read contract of include/halo_rx.h: no kernel reads a page that holds no frame byte. The
// stream reads every 16-byte block in [lo, hi) (clamped to it), so a window streams only when
// every 4 KB page of [lo, hi) holds a readable dword of one of its frames (member lanes `in`,
// frame dwords [ps, ps + nb)); pg0 = the stream base's offset in its page, so (position + pg0)
// >> 12 counts real pages. Pages are checked 32 at a time: each member lane ORs in the pages its
// frame touches, and the wave's union must be all of them. A window with a page-sized hole
// (frames in two allocations addressed from one base, or a sparse layout the 2x density test
// lets through) sums its frames lane by lane, reading nothing outside them.
__device__ __forceinline__ bool window_pages_covered(bool in, uint32_t ps, uint32_t nb, uint32_t lo, uint32_t hi,
                                                     uint32_t pg0) {
    const uint32_t P0 = (lo + pg0) >> 12;
    const uint32_t np = ((hi - 1u + pg0) >> 12) - P0 + 1u;
    const uint32_t a = in ? ((ps + pg0) >> 12) - P0 : 1u, b = in ? ((ps + nb - 1u + pg0) >> 12) - P0 : 0u;
    const auto uor = [](uint32_t x, uint32_t y) { return x | y; };
    for (uint32_t w0 = 0; w0 < np; w0 += 32) {
        const uint32_t w1 = np - 1u < w0 + 31u ? np - 1u : w0 + 31u;
        const uint32_t lb = a > w0 ? a : w0, hb = b < w1 ? b : w1;
        const uint32_t m = lb <= hb ? ((2u << (hb - lb)) - 1u) << (lb - w0) : 0u;
        if (wave_allreduce(m, uor) != (2u << (w1 - w0)) - 1u) return false;
    }
    return true;
}

// A/B knobs: threads per block and dynamic LDS padding per block.
#ifndef HALO_RX_STREAM_BLOCK
#define HALO_RX_STREAM_BLOCK 256
#endif
#ifndef HALO_RX_STREAM_LDS_PAD
#define HALO_RX_STREAM_LDS_PAD 0
#endif
#ifndef HALO_RX_STREAM_WAVES
#define HALO_RX_STREAM_WAVES 6
#endif
#ifndef HALO_RX_STREAM_PIPE  // 1: the next step's loads issued before this step is summed
#define HALO_RX_STREAM_PIPE 0
#endif
#ifndef HALO_RX_STREAM_HDR
#define HALO_RX_STREAM_HDR 1
#endif

// One stream step's 64 bytes of this lane: their 16-byte sub-chunk prefixes (P at each sub-chunk
// start; carry = P at the step start) and the bytes, to the wave's LDS.
__device__ __forceinline__ void stream_sum(const uint32_t (&x)[4][4], uint32_t lane, uint32_t& carry,
                                           uint32_t* s_base, uint4* s_x) {
    uint32_t s[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
        s[u] = halves_acc(x[u][3], halves_acc(x[u][2], halves_acc(x[u][1], halves_acc(x[u][0], 0u))));
    uint32_t total;
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // sub-chunk k = 64u + lane in stream order
        s_base[u * 64 + lane] = carry + wave_excl_scan(s[u], lane, total);
        carry += total;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) s_x[u * 64 + lane] = make_uint4(x[u][0], x[u][1], x[u][2], x[u][3]);
    wave_lds_sync();
}

// HDR (chosen per call: checksums on): the headers come out of the stream too. Each lane copies
// its frame's 48 header bytes from the step buffer as the stream passes them, and its segment end
// follows from the IPv4 total length (the parse's seg_end = O + totalLen) as soon as that field
// has passed; the header checks run once after the stream. Every byte of a dense window is then
// fetched from HBM exactly once. Without HDR (checksums off: only ICMP frames have a segment),
// the lane reads its header first and the stream covers only the windows' segments.
// Mixed-size batches (IMIX) take the stream kernel in one-wave blocks with 1.5 KB of LDS padding
// (22 blocks = 5.5 waves per SIMD resident): IMIX 1.27 -> 1.25 ms; uniform batches keep 256-thread
// blocks, which the 570 B line prefers (127 vs 133 us; profiles/r02/ab_stream_group_block_uncapped.log).
#ifndef HALO_RX_STREAM_MIXED_BLOCK
#define HALO_RX_STREAM_MIXED_BLOCK 64
#endif
#ifndef HALO_RX_STREAM_MIXED_LDS_PAD
#define HALO_RX_STREAM_MIXED_LDS_PAD 1536
#endif
template <int LAYOUT, int FUSE, bool HDR, int BLK = HALO_RX_STREAM_BLOCK>
__global__ void __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(HALO_RX_STREAM_WAVES)))
rx_stream_kernel(const RxParams p) {
    constexpr int kW = BLK / 64;
    __shared__ uint32_t s_hist[HALO_RX_STATUS_COUNT];
    __shared__ uint4 s_x[kW][kStreamStep / 16];       // per wave: the step's bytes (records at the end)
    __shared__ uint32_t s_base[kW][kStreamStep / 16];  // per wave: P at each 16-byte sub-chunk
    if (threadIdx.x < HALO_RX_STATUS_COUNT) s_hist[threadIdx.x] = 0;
    __syncthreads();
    Hist hist = hist_open(p, s_hist);
    constexpr bool L3 = kL3<LAYOUT>;
    constexpr uint32_t O = kIpOff<L3>;
    constexpr uint32_t kSeg = O + 20u;        // L4 segment start in the frame (34 or 20)
    constexpr uint32_t kTlDw = (O + 2u) / 4u;  // the header dword holding the IPv4 total length
    constexpr uint32_t kNone = 0xFFFFFFFFu;    // a position no step holds
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = threadIdx.x >> 6;
    const bool compact = (p.flags & HALO_RX_RECORD_COMPACT) != 0;
    const bool aligned = (reinterpret_cast<uint64_t>(p.bytes) & 3u) == 0;  // positions are dword-exact
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const auto umin = [](uint32_t a, uint32_t b) { return a < b ? a : b; };
    const auto umax = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
    const auto uadd = [](uint32_t a, uint32_t b) { return a + b; };
    for (uint32_t wbase = wave * 64; wbase < p.n; wbase += nwaves * 64) {
        const uint32_t i = wbase + lane;
        const bool present = i < p.n;
        FrameState<1, 3> st;
        frame_meta<LAYOUT>(p, i, present, st);
        uint32_t h[12];
        Verdict v;
        uint64_t c = 0;
        bool done = false;  // wave-uniform: the window went through the stream
        if constexpr (HDR) {
            const bool rd = st.ndw != 0;
            const uint64_t rds = __ballot(rd);
            if (rds && aligned) {
                // positions relative to a base 2^30 below the first readable frame's 128-byte line
                const uint32_t first = (uint32_t)__builtin_ctzll(rds);
                const uint64_t fa = reinterpret_cast<uint64_t>(st.frame);
                const uint64_t ref = (((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(fa >> 32), first) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fa, first)) & ~127ull;
                const uint64_t B = ref - (1ull << 30);
                const uint64_t d64 = fa - B;
                const uint32_t ps = (uint32_t)d64;
                const uint32_t lo = wave_allreduce(rd ? ps : kNone, umin);
                const uint32_t hi = wave_allreduce(rd ? ps + 4 * st.ndw : 0u, umax);
                const uint32_t sum = wave_allreduce(rd ? st.L : 0u, uadd);
                const uint32_t G0 = lo & ~(uint32_t)(HALO_RX_STREAM_ALIGN - 1);
                const uint32_t span = hi - G0;
                if (!__ballot(rd && d64 >= (1ull << 31)) && span <= 2 * sum + 8192u &&
                    window_pages_covered(rd, ps, 4 * st.ndw, lo, hi, (uint32_t)B & 4095u)) {
#pragma unroll
                    for (int j = 0; j < 12; ++j) h[j] = 0;
                    const uint32_t pa = ps + kSeg;
                    uint32_t pb = kNone;  // the segment's last byte, once the total length has passed
                    uint32_t PA = 0, PB = 0, carry = 0;
                    const uint32_t nsteps = (span + kStreamStep - 1) / kStreamStep;
#if HALO_RX_STREAM_PIPE
                    uint32_t x[4][4];
                    stream_load(B, G0, lane, lo, hi, x);
#endif
                    for (uint32_t t = 0; t < nsteps; ++t) {
                        const uint32_t s0 = G0 + t * kStreamStep;
#if HALO_RX_STREAM_PIPE
                        uint32_t xn[4][4];  // the next step's bytes (past the window: a clamped re-read)
                        stream_load(B, s0 + kStreamStep, lane, lo, hi, xn);
                        stream_sum(x, lane, carry, s_base[w], s_x[w]);
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int k = 0; k < 4; ++k) x[u][k] = xn[u][k];
#else
                        uint32_t x[4][4];
                        stream_load(B, s0, lane, lo, hi, x);
                        stream_sum(x, lane, carry, s_base[w], s_x[w]);
#endif
                        const uint32_t* xw = reinterpret_cast<const uint32_t*>(s_x[w]);
                        const uint32_t r0 = ps - s0;  // header start in this step (wraps below it)
                        if (__ballot(rd && (r0 < kStreamStep || r0 + 48u < 48u + kStreamStep))) {
#pragma unroll
                            for (int j = 0; j < 12; ++j) {
                                const uint32_t r = r0 + 4u * j;
                                const uint32_t wv = xw[(r >> 2) & (kStreamStep / 4 - 1)];
                                if (rd && r < kStreamStep && (uint32_t)j < st.ndw) h[j] = wv;
                            }
                            if (rd && pb == kNone && r0 + 4u * kTlDw < kStreamStep && kTlDw < st.ndw) {
                                const uint32_t tl = L3 ? bswap16(h[0] >> 16) : bswap16(h[kTlDw] & 0xFFFFu);
                                pb = (tl >= 20u && O + tl <= st.L) ? ps + O + tl - 1u : kNone - 1u;
                            }
                        }
                        const uint32_t ra = pa - s0, rb = pb - s0;
                        if (rd && ra < kStreamStep) PA = stream_prefix(s_base[w], s_x[w], ra, ra & 3u);
                        if (rd && rb < kStreamStep) PB = stream_prefix(s_base[w], s_x[w], rb, (rb & 3u) + 1u);
                        wave_lds_sync();
                    }
                    v = parse_header<L3>(h, st.L, present, p);
                    if (v.seg_end) c = (uint32_t)(PB - PA);
                    done = true;
                }
            }
        }
        if (!done) {
            frame_loads(0u, st);
            frame_header(st, lane, h);
            v = parse_header<L3>(h, st.L, present, p);
            const bool seg = v.seg_end != 0;
            const uint64_t segs = __ballot(seg);
            bool streamed = false;
            if (!HDR && segs && aligned) {
                // positions relative to a base 2^30 below the first segment frame's 128-byte line
                const uint32_t first = (uint32_t)__builtin_ctzll(segs);
                const uint64_t fa = reinterpret_cast<uint64_t>(st.frame);
                const uint64_t ref = (((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(fa >> 32), first) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fa, first)) & ~127ull;
                const uint64_t B = ref - (1ull << 30);
                const uint64_t d64 = fa - B;
                const uint32_t ps = (uint32_t)d64;
                const uint32_t pa = ps + kSeg, pe = ps + v.seg_end;  // the segment is [pa, pe)
                const uint32_t S = wave_allreduce(seg ? pa : kNone, umin);
                const uint32_t E = wave_allreduce(seg ? pe : 0u, umax);
                const uint32_t lo = wave_allreduce(seg ? ps : kNone, umin);
                const uint32_t hi = wave_allreduce(seg ? ps + 4 * st.ndw : 0u, umax);
                const uint32_t sum = wave_allreduce(seg ? v.seg_end - kSeg : 0u, uadd);
                const uint32_t G0 = S & ~(uint32_t)(HALO_RX_STREAM_ALIGN - 1);
                const uint32_t span = E - G0;
                if (!__ballot(seg && d64 >= (1ull << 31)) && span <= 2 * sum + 8192u &&
                    window_pages_covered(seg, ps, 4 * st.ndw, lo, hi, (uint32_t)B & 4095u)) {
                    uint32_t PA = 0, PB = 0, carry = 0;
                    const uint32_t ea = pe - 1;  // the segment's last byte
                    const uint32_t nsteps = (span + kStreamStep - 1) / kStreamStep;
#if HALO_RX_STREAM_PIPE
                    uint32_t x[4][4];
                    stream_load(B, G0, lane, lo, hi, x);
#endif
                    for (uint32_t t = 0; t < nsteps; ++t) {
                        const uint32_t s0 = G0 + t * kStreamStep;
#if HALO_RX_STREAM_PIPE
                        uint32_t xn[4][4];  // the next step's bytes (past the window: a clamped re-read)
                        stream_load(B, s0 + kStreamStep, lane, lo, hi, xn);
                        stream_sum(x, lane, carry, s_base[w], s_x[w]);
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int k = 0; k < 4; ++k) x[u][k] = xn[u][k];
#else
                        uint32_t x[4][4];
                        stream_load(B, s0, lane, lo, hi, x);
                        stream_sum(x, lane, carry, s_base[w], s_x[w]);
#endif
                        const uint32_t ra = pa - s0, rb = ea - s0;
                        if (seg && ra < kStreamStep) PA = stream_prefix(s_base[w], s_x[w], ra, ra & 3u);
                        if (seg && rb < kStreamStep) PB = stream_prefix(s_base[w], s_x[w], rb, (rb & 3u) + 1u);
                        wave_lds_sync();
                    }
                    c = (uint32_t)(PB - PA);
                    streamed = true;
                }
            }
            if (seg && !streamed) {  // not dense (or unaligned data): this lane sums its own segment
                const uint32_t seg_dw = (v.seg_end + 3) >> 2;
                for (uint32_t d0 = (kSeg / 4) & ~3u; d0 < seg_dw; d0 += 4) {
                    uint32_t x[4];
                    load4(st.frame, d0, seg_dw, x);
                    acc_segment<L3>(x, d0, v.seg_end, c);
                }
            }
        }
        uint4* stage = reinterpret_cast<uint4*>(s_x[w]);
        frame_store<1, FUSE, L3>(p, i, present, 0, h, v, c, hist, &stage[compact ? lane : 2 * lane]);
        wave_lds_sync();
        const uint32_t nrec = p.n - wbase < 64 ? p.n - wbase : 64;
        constexpr bool kNt = HALO_RX_STREAM_NT_STORES != 0;
        if (compact) {
            if (lane < nrec) store16<kNt>(reinterpret_cast<uint4*>(p.out) + wbase + lane, stage[lane]);
        } else {
            uint4* out4 = reinterpret_cast<uint4*>(p.out) + 2ull * wbase;
            if (lane < 2 * nrec) store16<kNt>(out4 + lane, stage[lane]);
            if (64 + lane < 2 * nrec) store16<kNt>(out4 + 64 + lane, stage[64 + lane]);
        }
        wave_lds_sync();
    }
    flush_hist(p, hist);
}

// Grid cap, in 4-wave blocks (the lane kernel scales it to its block size). Effectively no cap:
// a launch takes one wave per 64 frames (per frame group) and lets the dispatcher refill CUs as
// waves finish. The round-1 cap of 16384 blocks made waves loop over several groups in big batches,
// and a looping wave serialises its round trips: lifting it took 16M x 64 B 314 -> 294 us,
// 128M x 64 B 2.74 -> 2.32 ms, IMIX 1.32 -> 1.28 ms, jumbo 6.20 -> 6.14 ms, 1500 B within noise
// (profiles/r02/ab_grid_cap_raised.log).
#ifndef HALO_RX_MAX_BLOCKS
#define HALO_RX_MAX_BLOCKS 4194304ull
#endif
#ifndef HALO_RX_LANE_MAX_BLOCKS
#define HALO_RX_LANE_MAX_BLOCKS HALO_RX_MAX_BLOCKS
#endif
#ifndef HALO_RX_HIST_HALVE_MAX  // lane-kernel grids up to this many blocks are halved when a histogram is kept
#define HALO_RX_HIST_HALVE_MAX 16384u
#endif
constexpr int kVariantMix = -1, kVariantStream = 2, kVariantStreamMixed = 3;

uint32_t grid_for(uint64_t n, uint32_t frames_per_wave, uint64_t max_blocks = HALO_RX_MAX_BLOCKS,
                  uint32_t waves_per_block = 4) {
    const uint64_t waves = (n + frames_per_wave - 1) / frames_per_wave;
    uint64_t blocks = (waves + waves_per_block - 1) / waves_per_block;
    const uint64_t kMaxBlocks = max_blocks;
    return (uint32_t)(blocks > kMaxBlocks ? kMaxBlocks : blocks);
}

template <int LAYOUT, int FUSE = 0>
hipError_t launch_variant(const RxParams& p, int variant, hipStream_t s) {
    const dim3 block(256);
    switch (variant) {
        case 1: {
            constexpr uint32_t wpb = HALO_RX_LANE_BLOCK / 64;
            uint32_t grid = grid_for(p.n, 64, HALO_RX_LANE_MAX_BLOCKS * 4 / wpb, wpb);
            // with a status histogram, batches up to 1M frames take half the waves, two frame groups
            // each: half the arrivals in the histogram tree, whose tail is a fixed cost per launch
            // (1M x 64 B: +2.1 instead of +2.7 us, 8192 blocks; 4096 gave no gain, profiles/r05/r5zm)
            if (p.hist && grid <= HALO_RX_HIST_HALVE_MAX) grid = (grid + 1) / 2;
            hipLaunchKernelGGL((rx_lane_kernel<LAYOUT, FUSE>), dim3(grid),
                               dim3(HALO_RX_LANE_BLOCK), HALO_RX_LANE_LDS_PAD, s, p);
            break;
        }
        case kVariantStream: {
            constexpr uint32_t wpb = HALO_RX_STREAM_BLOCK / 64;
            const dim3 g(grid_for(p.n, 64, HALO_RX_MAX_BLOCKS * 4 / wpb, wpb)), b(HALO_RX_STREAM_BLOCK);
            if (HALO_RX_STREAM_HDR && (p.flags & HALO_RX_CSUM_ENABLE))
                hipLaunchKernelGGL((rx_stream_kernel<LAYOUT, FUSE, true>), g, b, HALO_RX_STREAM_LDS_PAD, s, p);
            else
                hipLaunchKernelGGL((rx_stream_kernel<LAYOUT, FUSE, false>), g, b, HALO_RX_STREAM_LDS_PAD, s, p);
            break;
        }
        case kVariantStreamMixed: {
            constexpr int BLK = HALO_RX_STREAM_MIXED_BLOCK;
            constexpr uint32_t wpb = BLK / 64;
            const dim3 g(grid_for(p.n, 64, HALO_RX_MAX_BLOCKS * 4 / wpb, wpb)), b(BLK);
            if (HALO_RX_STREAM_HDR && (p.flags & HALO_RX_CSUM_ENABLE))
                hipLaunchKernelGGL((rx_stream_kernel<LAYOUT, FUSE, true, BLK>), g, b, HALO_RX_STREAM_MIXED_LDS_PAD, s, p);
            else
                hipLaunchKernelGGL((rx_stream_kernel<LAYOUT, FUSE, false, BLK>), g, b, HALO_RX_STREAM_MIXED_LDS_PAD, s, p);
            break;
        }
        case 4: case 8: case 16: {
            constexpr uint32_t wpb = HALO_RX_GROUP_BLOCK / 64;
            const dim3 b(HALO_RX_GROUP_BLOCK);
            const uint64_t cap = HALO_RX_MAX_BLOCKS * 4 / wpb;
            if (variant == 4)
                hipLaunchKernelGGL((rx_group_kernel<4, LAYOUT, FUSE>), dim3(grid_for(p.n, 16, cap, wpb)), b, HALO_RX_GROUP_LDS_PAD, s, p);
            else if (variant == 8)
                hipLaunchKernelGGL((rx_group_kernel<8, LAYOUT, FUSE>), dim3(grid_for(p.n, 8, cap, wpb)), b, HALO_RX_GROUP_LDS_PAD, s, p);
            else
                hipLaunchKernelGGL((rx_group_kernel<16, LAYOUT, FUSE>), dim3(grid_for(p.n, 4, cap, wpb)), b, HALO_RX_GROUP_LDS_PAD, s, p);
            break;
        }
        default: hipLaunchKernelGGL((rx_mix_kernel<LAYOUT, FUSE>), dim3(grid_for(p.n, kMixWindow)), block, 0, s, p); break;
    }
    return hipGetLastError();
}

// Kernel variant (from the sweeps in profiles/r01/tune_*.log and
// profiles/r02/stream/): a variant named in the call's flags wins; frames all <= 64 B go lane
// per frame; frames packed densely in memory (ragged layouts, or strided with little slack)
// up to 1 KB, or of mixed sizes, take the byte-stream kernel; longer uniform frames take 8 or 16
// lanes per frame; mixed sizes that are not dense take the size-class mix kernel.
int pick_variant(uint32_t max_len, bool uniform, bool dense, uint32_t flags) {
    switch ((flags & HALO_RX_VARIANT_MASK) >> HALO_RX_VARIANT_SHIFT) {
        case HALO_RX_VARIANT_LANE: return 1;
        case HALO_RX_VARIANT_G4: return 4;
        case HALO_RX_VARIANT_G8: return 8;
        case HALO_RX_VARIANT_G16: return 16;
        case HALO_RX_VARIANT_MIX: return kVariantMix;
        case HALO_RX_VARIANT_STREAM: return kVariantStream;
        default: break;
    }
    if (flags & HALO_RX_UNIFORM_LEN) uniform = max_len != 0;
    if (max_len != 0 && max_len <= 64) return 1;
    if (!uniform) return dense ? kVariantStreamMixed : kVariantMix;
    if (max_len <= 1024) return dense ? kVariantStream : max_len <= 128 ? 1 : 4;
    if (max_len <= 4096) return 8;
    return 16;
}

int launch_parse(const RxParams& p_in, int layout, uint32_t max_len, bool uniform, hipStream_t s) {
    // ragged batches are taken as packed back to back (the stream kernel checks each window and
    // sums a sparse one frame by frame); strided frames of one length are dense when the stride
    // wastes < 1/4; strided frames with their own lengths may be anything below the stride
    RxParams p = p_in;
    p.hist_out = p.hist;
    if (p.hist && !(p.hist = hist_trees(stream_device(s), s))) return HALO_E_NOMEM;  // counts go through a tree
    const bool dense = layout == 0 || layout == 3 || (layout == 2 && p.stride <= max_len + max_len / 4 + 64);
    const int v = pick_variant(max_len, uniform, dense, p.flags);
    hipError_t e;
    switch (layout) {
        case 0:  // ragged: the only layout with the fused passes
            e = p.flow_hash ? launch_variant<0, 1>(p, v, s)
              : p.route_out ? launch_variant<0, 2>(p, v, s) : launch_variant<0, 0>(p, v, s);
            break;
        case 1: e = launch_variant<1>(p, v, s); break;
        case 3: e = launch_variant<3>(p, v, s); break;  // LoChan packets: plain parse only
        default: e = launch_variant<2>(p, v, s); break;
    }
    return e == hipSuccess ? HALO_OK : HALO_E_HIP;
}

int fill_common(RxParams& p, uint32_t n, uint32_t flags, const halo_rx_netif_t* netif,
                halo_rx_result_t* d_out, uint32_t* d_hist) {
    if (!netif || !d_out) return HALO_E_INVAL;
    if (flags & ~(HALO_RX_CSUM_ENABLE | HALO_RX_JUMBO_EXT | HALO_RX_RECORD_COMPACT | HALO_RX_UNIFORM_LEN |
                  HALO_RX_L3_START | HALO_RX_VARIANT_MASK))
        return HALO_E_INVAL;
    if (((flags & HALO_RX_VARIANT_MASK) >> HALO_RX_VARIANT_SHIFT) > HALO_RX_VARIANT_STREAM) return HALO_E_INVAL;
    if (reinterpret_cast<uintptr_t>(d_out) & 15u) return HALO_E_INVAL;
    p.n = n;
    p.flags = flags;
    p.mac_lo = (uint32_t)netif->mac[0] | ((uint32_t)netif->mac[1] << 8) | ((uint32_t)netif->mac[2] << 16) |
               ((uint32_t)netif->mac[3] << 24);
    p.mac_hi = (uint32_t)netif->mac[4] | ((uint32_t)netif->mac[5] << 8);
    p.own_ip = netif->ip;
    p.out = d_out;
    p.hist = d_hist;
    return HALO_OK;
}

}  // namespace

int stream_device(hipStream_t s) {
    int dev = -1;
    if (s != nullptr && s != hipStreamPerThread) {
        if (hipStreamGetDevice(s, &dev) == hipSuccess) return dev;
        (void)hipGetLastError();
        return -1;
    }
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return dev;
}

namespace {
std::mutex g_trees_mu;
uint32_t* g_trees[64];      // a device's set: made once, never freed (graphs hold its address)
bool g_no_barriers[64];     // the probe found a dispatch without the barrier bit: keys stay poisoned

// Writes its own AQL packet header (the barrier bit is bit 8) to *out.
__global__ void dispatch_header_probe(unsigned long long* out) {
    if (threadIdx.x == 0) *out = *static_cast<const volatile uint16_t*>((const void*)__builtin_amdgcn_dispatch_ptr());
}

// flush_hist relies on every dispatch carrying the barrier bit (the runtime's in-order streams do:
// profiles/r05/queue_probe.log) instead of re-reading the packet in every block, which costs 4x the
// launch. Checked once per device on the null stream and a fresh stream; without the bit the keys
// are poisoned, and every launch adds straight into the caller's counters (slow, exact).
bool barrier_bits_set(unsigned long long* scratch) {
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return false;
    hipLaunchKernelGGL(dispatch_header_probe, dim3(1), dim3(64), 0, nullptr, scratch);
    hipLaunchKernelGGL(dispatch_header_probe, dim3(1), dim3(64), 0, st, scratch + 1);
    unsigned long long h[2] = {0, 0};
    const bool ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(st) == hipSuccess &&
                    hipStreamSynchronize(nullptr) == hipSuccess &&
                    hipMemcpy(h, scratch, sizeof h, hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipStreamDestroy(st);
    return ok && ((h[0] >> 8) & 1u) && ((h[1] >> 8) & 1u);
}
}  // namespace

uint32_t* hist_trees(int device, hipStream_t capture_probe) {
    if (device < 0 || device >= 64) return nullptr;
    std::lock_guard<std::mutex> g(g_trees_mu);
    uint32_t*& p = g_trees[device];
    if (p) return p;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(capture_probe, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
        (void)hipGetLastError();
        return nullptr;  // no allocation inside a capture: halo_rx_init(device) makes the set beforehand
    }
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != device && hipSetDevice(device) != hipSuccess) return nullptr;
    void* m = nullptr;
    bool ok = hipMalloc(&m, kHistSetBytes) == hipSuccess;
    const bool barriers = ok && barrier_bits_set(static_cast<unsigned long long*>(m) + kHistKeyWords);
    ok = ok && hipMemsetAsync(m, 0, kHistSetBytes, nullptr) == hipSuccess &&
         (barriers || hipMemsetAsync(m, 0xFF, 8ull * kHistTrees, nullptr) == hipSuccess) &&
         hipStreamSynchronize(nullptr) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        if (m) (void)hipFree(m);
        m = nullptr;
    }
    if (cur != device) (void)hipSetDevice(cur);
    g_no_barriers[device] = ok && !barriers;
    p = static_cast<uint32_t*>(m);
    return p;
}

namespace {
// Writes the key words of `device`'s set (g_trees_mu held): all 0 (free), all ~0 (poisoned), or
// ids no queue has for all but the first `free_keys` slots.
int write_keys(int device, int fill, uint32_t free_keys) {
    uint32_t* set = g_trees[device];
    if (!set) return HALO_E_NOMEM;
    unsigned long long k[kHistKeyWords];
    for (uint32_t j = 0; j < kHistKeyWords; ++j)
        k[j] = fill == 0 ? 0ull : fill == 1 ? ~0ull : (j < free_keys ? 0ull : 0x40ull * (j + 1));  // not a queue address
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return HALO_E_NODEV;
    if (cur != device && hipSetDevice(device) != hipSuccess) return HALO_E_NODEV;
    const bool ok = hipMemcpy(set, k, sizeof k, hipMemcpyHostToDevice) == hipSuccess;
    if (cur != device) (void)hipSetDevice(cur);
    return ok ? HALO_OK : HALO_E_HIP;
}
}  // namespace

int hist_trees_reset_keys(int device) {
    if (device < 0 || device >= 64) return HALO_E_NODEV;
    std::lock_guard<std::mutex> g(g_trees_mu);
    if (!g_trees[device]) return HALO_OK;
    return write_keys(device, g_no_barriers[device] ? 1 : 0, 0);
}

int hist_keys_debug(int device, int op, uint32_t arg) {
    if (device < 0 || device >= 64) return HALO_E_NODEV;
    if (op == 3) return hist_trees_reset_keys(device);
    if (!hist_trees(device, nullptr)) return HALO_E_NOMEM;
    std::lock_guard<std::mutex> g(g_trees_mu);
    if (op == 1) return write_keys(device, 1, 0);
    if (op == 2) return arg > kHistTrees ? HALO_E_INVAL : write_keys(device, 2, arg);
    if (op != 0) return HALO_E_INVAL;
    unsigned long long k[kHistKeyWords];
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return HALO_E_NODEV;
    if (cur != device && hipSetDevice(device) != hipSuccess) return HALO_E_NODEV;
    const bool ok = hipMemcpy(k, g_trees[device], sizeof k, hipMemcpyDeviceToHost) == hipSuccess;
    if (cur != device) (void)hipSetDevice(cur);
    if (!ok) return HALO_E_HIP;
    int claimed = 0;
    for (uint32_t j = 0; j < kHistTrees; ++j) claimed += k[j] != 0 && k[j] != ~0ull;
    return claimed;
}
}  // namespace halo

extern "C" HALO_API int halo_rx_parse_batch_device(const uint8_t* d_bytes, const uint32_t* d_offsets_dw,
                                                   const uint16_t* d_lens, uint32_t n, uint32_t flags,
                                                   const halo_rx_netif_t* netif, uint32_t max_len_hint,
                                                   halo_rx_result_t* d_out, uint32_t* d_status_hist,
                                                   halo_stream_t stream) {
    halo::RxParams p{};
    int rc = halo::fill_common(p, n, flags, netif, d_out, d_status_hist);
    if (rc) return rc;
    if (n == 0) return HALO_OK;
    if (!d_bytes || !d_offsets_dw || !d_lens) return HALO_E_INVAL;
    if ((rc = halo::check_device())) return rc;
    p.bytes = d_bytes;
    p.offsets_dw = d_offsets_dw;
    p.lens = d_lens;
    return halo::launch_parse(p, (flags & HALO_RX_L3_START) ? 3 : 0, max_len_hint, false,
                              static_cast<hipStream_t>(stream));
}

extern "C" HALO_API int halo_rx_parse_flow_batch_device(const uint8_t* d_bytes, const uint32_t* d_offsets_dw,
                                                        const uint16_t* d_lens, uint32_t n, uint32_t flags,
                                                        const halo_rx_netif_t* netif, uint32_t max_len_hint,
                                                        halo_rx_result_t* d_out, uint32_t* d_status_hist,
                                                        uint32_t flow_kind, uint32_t nat_type, uint64_t* d_hash,
                                                        uint32_t bucket_count, uint32_t* d_bucket,
                                                        halo_stream_t stream) {
    if (flow_kind > HALO_FLOW_NAT_WAN || !d_hash || (reinterpret_cast<uintptr_t>(d_hash) & 7u)) return HALO_E_INVAL;
    if (d_bucket && bucket_count == 0) return HALO_E_INVAL;
    halo::RxParams p{};
    int rc = halo::fill_common(p, n, flags, netif, d_out, d_status_hist);
    if (rc) return rc;
    if (flags & HALO_RX_L3_START) return HALO_E_INVAL;  // LoChan packets: plain ragged parse only
    if (n == 0) return HALO_OK;
    if (!d_bytes || !d_offsets_dw || !d_lens) return HALO_E_INVAL;
    if ((rc = halo::check_device())) return rc;
    p.bytes = d_bytes;
    p.offsets_dw = d_offsets_dw;
    p.lens = d_lens;
    p.flow_hash = d_hash;
    p.flow_bucket = d_bucket;
    p.flow_buckets = bucket_count;
    p.flow_kind = flow_kind;
    p.flow_nat = nat_type;
    return halo::launch_parse(p, 0, max_len_hint, false, static_cast<hipStream_t>(stream));
}

extern "C" HALO_API int halo_rx_parse_route_batch_device(const uint8_t* d_bytes, const uint32_t* d_offsets_dw,
                                                         const uint16_t* d_lens, uint32_t n, uint32_t flags,
                                                         const halo_rx_netif_t* netif, uint32_t max_len_hint,
                                                         halo_rx_result_t* d_out, uint32_t* d_status_hist,
                                                         const halo_route_table_t* table, uint32_t* d_route_ids,
                                                         halo_stream_t stream) {
    halo::RouteViewLock lk(table);  // until the fused kernel is enqueued
    halo::LpmView v{};
    if (halo::route_view(table, &v) || !d_route_ids) return HALO_E_INVAL;
    halo::RxParams p{};
    int rc = halo::fill_common(p, n, flags, netif, d_out, d_status_hist);
    if (rc) return rc;
    if (flags & HALO_RX_L3_START) return HALO_E_INVAL;  // LoChan packets: plain ragged parse only
    if (n == 0) return HALO_OK;
    if (!d_bytes || !d_offsets_dw || !d_lens) return HALO_E_INVAL;
    if ((rc = halo::check_device())) return rc;
    p.bytes = d_bytes;
    p.offsets_dw = d_offsets_dw;
    p.lens = d_lens;
    p.rt_tbl24 = v.tbl24;
    p.rt_tbl8 = v.tbl8;
    p.rt_lists = v.lists;
    p.rt_ids = v.ids;
    p.route_out = d_route_ids;
    return halo::launch_parse(p, 0, max_len_hint, false, static_cast<hipStream_t>(stream));
}

extern "C" HALO_API int halo_rx_parse_strided_device(const uint8_t* d_bytes, uint64_t stride,
                                                     const uint16_t* d_lens, uint32_t len, uint32_t n,
                                                     uint32_t flags, const halo_rx_netif_t* netif,
                                                     halo_rx_result_t* d_out, uint32_t* d_status_hist,
                                                     halo_stream_t stream) {
    halo::RxParams p{};
    int rc = halo::fill_common(p, n, flags, netif, d_out, d_status_hist);
    if (rc) return rc;
    if (flags & HALO_RX_L3_START) return HALO_E_INVAL;  // LoChan packets: plain ragged parse only
    if (n == 0) return HALO_OK;
    if (!d_bytes || (stride & 3u) || (n > 1 && stride == 0)) return HALO_E_INVAL;
    if (!d_lens && n > 1 && len > stride) return HALO_E_INVAL;
    if ((rc = halo::check_device())) return rc;
    p.bytes = d_bytes;
    p.lens = d_lens;
    p.stride = stride;
    p.len = len;
    // with per-frame lengths only the stride bounds them (mixed sizes possible)
    const uint32_t max_len = d_lens ? (uint32_t)(stride < 65535 ? stride : 65535) : len;
    return halo::launch_parse(p, d_lens ? 1 : 2, max_len, d_lens == nullptr, static_cast<hipStream_t>(stream));
}

extern "C" HALO_API int halo_rx_parse_batches_device(const halo_rx_batch_desc_t* batches, uint32_t k, uint32_t flags,
                                                     const halo_rx_netif_t* netif, uint32_t max_len_hint,
                                                     uint32_t* d_status_hist, halo_stream_t stream) {
    if (!batches || k == 0 || k > halo::kMultiMax) return HALO_E_INVAL;
    halo::MultiParams mp{};
    uint64_t windows = 0;
    uint32_t live = 0;
    for (uint32_t j = 0; j < k; ++j) {
        const halo_rx_batch_desc_t& d = batches[j];
        if (d.n == 0) {
            mp.win_end[j] = (uint32_t)windows;
            continue;
        }
        int rc = halo::fill_common(mp.p, d.n, flags, netif, d.d_out, d_status_hist);
        if (rc) return rc;
        if (!d.d_bytes || !d.d_offsets_dw || !d.d_lens) return HALO_E_INVAL;
        windows += (d.n + 63u) / 64u;
        mp.win_end[j] = (uint32_t)windows;
        mp.n[j] = d.n;
        mp.bytes[j] = d.d_bytes;
        mp.offsets_dw[j] = d.d_offsets_dw;
        mp.lens[j] = d.d_lens;
        mp.out[j] = d.d_out;
        ++live;
    }
    if (!live) return netif ? HALO_OK : HALO_E_INVAL;
    int rc = halo::check_device();
    if (rc) return rc;
    const uint32_t v = (flags & HALO_RX_VARIANT_MASK) >> HALO_RX_VARIANT_SHIFT;
    const bool lane = v == HALO_RX_VARIANT_LANE || (v == HALO_RX_VARIANT_AUTO && max_len_hint && max_len_hint <= 64);
    if (!lane) {  // the larger-frame kernels are per batch: one launch each, in order, on `stream`
        for (uint32_t j = 0; j < k && rc == HALO_OK; ++j)
            if (batches[j].n)
                rc = halo_rx_parse_batch_device(batches[j].d_bytes, batches[j].d_offsets_dw, batches[j].d_lens,
                                                batches[j].n, flags, netif, max_len_hint, batches[j].d_out,
                                                d_status_hist, stream);
        return rc;
    }
    mp.k = k;
    mp.p.n = 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    mp.p.hist_out = d_status_hist;
    if (d_status_hist && !(mp.p.hist = halo::hist_trees(halo::stream_device(s), s))) return HALO_E_NOMEM;
    constexpr uint32_t wpb = HALO_RX_LANE_BLOCK / 64;
    const dim3 grid(halo::grid_for(windows * 64u, 64, HALO_RX_LANE_MAX_BLOCKS * 4 / wpb, wpb));
    if (flags & HALO_RX_L3_START)
        hipLaunchKernelGGL(halo::rx_lane_multi_kernel<3>, grid, dim3(HALO_RX_LANE_BLOCK), HALO_RX_LANE_LDS_PAD, s, mp);
    else
        hipLaunchKernelGGL(halo::rx_lane_multi_kernel<0>, grid, dim3(HALO_RX_LANE_BLOCK), HALO_RX_LANE_LDS_PAD, s, mp);
    return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
}

namespace halo {
int launch_ring_service(RingServiceCtl* d_ctl, const uint8_t* d_data, const uint32_t* d_off, const uint16_t* d_len,
                        uint32_t* d_quit, uint32_t last, uint32_t idle_us, hipStream_t s) {
    if (hipMemsetAsync(d_quit, 0, sizeof(uint32_t), s) != hipSuccess) return HALO_E_HIP;
    hipLaunchKernelGGL(ring_service_kernel, dim3(kSvcGroups), dim3(64 * kSvcWaves), 0, s, d_ctl, d_data, d_off, d_len,
                       d_quit, last, (uint64_t)idle_us * 100u);  // s_memrealtime: 100 MHz
    return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
}
}  // namespace halo
