// rx_cpu.cc — libhalo_rx_cpu.so: halo_rx_parse_batch_cpu (include/halo_rx_cpu.h), the receive
// parse-and-verify chain on the calling core. No HIP, and nothing in libhalo_rx.so calls it: it is
// the explicit CPU entry point of SURVEY.md §8b for polls too small to pay a GPU round trip, not a
// fallback for a missing device.
//
// Per frame, in reference order (the same verdicts and record fields as rx_parse.hip's
// parse_header / finish_l4 / frame_store):
//   ParseEthFrm        protocol/ethernet.go:29-55   length caps, EtherType whitelist
//   RxEthernet filter  engine/ethernet_engine.go:22 dst MAC == own || broadcast
//   ParseIpv4Pkt       protocol/ipv4.go:48-86       len, 0x45, DF|0, protocol, header checksum, totalLen
//   NatGetSrcDstPort   protocol/ipv4.go:229-246     ports (ICMP: the echo id twice)
//   ParseUdpPkt        protocol/udp.go:21-49        pseudo length = the UDP length field
//   ParseTcpPkt        protocol/tcp.go:36-70        pseudo length = len(pkt); payload at the
//                                                   data-offset nibble used as bytes
//   ParseIcmpPkt       protocol/icmp.go:33-63       type, code, checksum always verified
//   GetCheckSum        protocol/utils.go:11-31
//
// Checksums: every region starts at an even offset of the bytes GetCheckSum is given (the IPv4
// header, the pseudo header + segment), so the sum of the region's little-endian 16-bit words is
// the byte swap of GetCheckSum's big-endian sum (RFC 1071 §2B), and "GetCheckSum == 0" is "the
// folded little-endian sum is 0xFFFF" (0xFFFF is its own swap). The region is read 8 bytes at a
// time and each u64 adds as its two u32 halves (2^16 == 1 mod 0xFFFF); an odd last byte lands in
// the low byte of its little-endian word, the high byte of GetCheckSum's (utils.go:21-24).
#include <stdint.h>
#include <string.h>

#include "halo_limits.h"
#include "halo_rx.h"
#include "halo_rx_cpu.h"

namespace {

using namespace halo;

inline uint32_t be16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }
inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
inline uint32_t le16(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }

// Little-endian word sum of [p, p + n), up to a multiple of 0xFFFF (see the header comment).
inline uint64_t sum_le(const uint8_t* p, uint32_t n) {
    uint64_t a = 0, b = 0;
    uint32_t i = 0;
    for (; i + 16 <= n; i += 16) {
        uint64_t w0, w1;
        memcpy(&w0, p + i, 8);
        memcpy(&w1, p + i + 8, 8);
        a += (w0 & 0xFFFFFFFFu) + (w0 >> 32);
        b += (w1 & 0xFFFFFFFFu) + (w1 >> 32);
    }
    if (i + 8 <= n) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        a += (w & 0xFFFFFFFFu) + (w >> 32);
        i += 8;
    }
    if (i + 4 <= n) {
        uint32_t w;
        memcpy(&w, p + i, 4);
        b += w;
        i += 4;
    }
    if (i + 2 <= n) {
        a += le16(p + i);
        i += 2;
    }
    if (i < n) b += p[i];
    return a + b;
}

inline bool sums_to_ones(uint64_t s) {
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return s == 0xFFFFu;
}

struct Own {
    uint32_t mac_lo, mac_hi;  // own MAC bytes 0..3 / 4..5, little-endian packed
    uint32_t ip;
    bool csum, jumbo;
};

// One frame (or, with L3, one LoChan packet starting at its IPv4 header) -> its record.
template <bool L3>
inline void parse_one(const uint8_t* f, uint32_t L, const Own& own, halo_rx_result_t& r) {
    r = halo_rx_result_t{};
    r.status = HALO_RX_OK;
    r.ethertype = kEthUnknown;
    r.ip_proto = kIpUnknown;
    const uint8_t* p;  // the IPv4 packet
    uint32_t iplen;
    if (L3) {  // engine/engine.go:361: the channel carries IPv4 packets only
        r.ethertype = kEthIpv4;
        p = f;
        iplen = L;
    } else {
        if (L < kEthMin || L > (own.jumbo ? kEthMaxJumbo : kEthMax)) {
            r.status = HALO_RX_ETH_LEN;
            return;
        }
        const uint32_t et = be16(f + 12);
        if (et != kEthIeee8023 && et != kEthIpv4 && et != kEthArp && et != kEthIpv6) {
            r.status = HALO_RX_ETH_TYPE;
            return;
        }
        r.ethertype = (uint16_t)et;
        r.payload_off = 14;
        r.payload_len = (uint16_t)(L - 14);
        uint32_t dm_lo;
        memcpy(&dm_lo, f, 4);
        const uint32_t dm_hi = le16(f + 4);
        if ((dm_lo == own.mac_lo && dm_hi == own.mac_hi) || (dm_lo == 0xFFFFFFFFu && dm_hi == 0xFFFFu))
            r.flags |= HALO_RX_F_MAC_MATCH;
        if (et != kEthIpv4) return;
        p = f + 14;
        iplen = L - 14;
    }
    const uint32_t O = L3 ? 0u : 14u;
    if (iplen < 20 || iplen > (own.jumbo ? kIpMaxJumbo : kIpMax)) {
        r.status = HALO_RX_IP_LEN;
        return;
    }
    if (p[0] != 0x45) {
        r.status = HALO_RX_IP_VER;
        return;
    }
    if ((p[6] != 0x40 && p[6] != 0x00) || p[7] != 0x00) {
        r.status = HALO_RX_IP_FRAG;
        return;
    }
    const uint32_t proto = p[9];
    if (proto != kIpIcmp && proto != kIpTcp && proto != kIpUdp) {
        r.status = HALO_RX_IP_PROTO;
        return;
    }
    if (own.csum && !sums_to_ones(sum_le(p, 20))) {
        r.status = HALO_RX_IP_HDR_CKSUM;
        return;
    }
    const uint32_t total = be16(p + 2);
    if (total < 20) {  // pkt[20:totalLen] (ipv4.go:84): Go panics
        r.status = HALO_RX_IP_TOTLEN_UNDERFLOW;
        return;
    }
    if (total > iplen) {  // ... or reads past len(pkt)
        r.status = HALO_RX_IP_TOTLEN_OVERRUN;
        return;
    }
    r.ip_proto = (uint8_t)proto;
    r.ip_total_len = (uint16_t)total;
    r.src_ip = be32(p + 12);
    r.dst_ip = be32(p + 16);
    if (p[19] == 255) r.flags |= HALO_RX_F_IP_BCAST;
    if (r.dst_ip == own.ip) r.flags |= HALO_RX_F_DST_IS_OWN;
    if (L3 && iplen < 26) {  // NatGetSrcDstPort: (0, 0) below 26 bytes
    } else if (proto == kIpIcmp) {
        r.sport = r.dport = (uint16_t)be16(p + 24);
    } else {
        r.sport = (uint16_t)be16(p + 20);
        r.dport = (uint16_t)be16(p + 22);
    }
    r.payload_off = (uint16_t)(O + 20);
    r.payload_len = (uint16_t)(total - 20);

    const uint8_t* s = p + 20;  // the L4 segment, len = totalLen - 20
    const uint32_t l4 = total - 20;
    const uint32_t l4_max = own.jumbo ? kL4MaxJumbo : kL4Max;
    // pseudo-header addresses, little-endian words
    const uint64_t addr = (uint64_t)le16(p + 12) + le16(p + 14) + le16(p + 16) + le16(p + 18);
    if (proto == kIpUdp) {
        if (l4 < 8 || l4 > l4_max) {
            r.status = HALO_RX_L4_LEN;
            return;
        }
        // fake header: src, dst, 0x00 0x11, the UDP length field (udp.go:34-38)
        if (own.csum && !sums_to_ones(sum_le(s, l4) + addr + 0x1100u + le16(s + 4))) {
            r.status = HALO_RX_L4_CKSUM;
            return;
        }
        r.payload_off = (uint16_t)(O + 28);
        r.payload_len = (uint16_t)(l4 - 8);
    } else if (proto == kIpTcp) {
        if (l4 < 20 || l4 > l4_max) {
            r.status = HALO_RX_L4_LEN;
            return;
        }
        // fake header: src, dst, 0x00 0x06, len(pkt) (tcp.go:54-59)
        if (own.csum && !sums_to_ones(sum_le(s, l4) + addr + 0x0600u + ((l4 >> 8) | ((l4 & 0xFFu) << 8)))) {
            r.status = HALO_RX_L4_CKSUM;
            return;
        }
        const uint32_t hl = s[12] >> 4;  // tcp.go:49: words used as bytes
        r.l4_aux = s[13];
        r.l4_seq = be32(s + 4);
        r.l4_ack = be32(s + 8);
        r.payload_off = (uint16_t)(O + 20 + hl);
        r.payload_len = (uint16_t)(l4 - hl);
    } else {
        if (l4 < 8 || l4 > l4_max) {
            r.status = HALO_RX_L4_LEN;
            return;
        }
        if (s[0] != kIcmpRequest && s[0] != kIcmpReply && s[0] != kIcmpTtl) {
            r.status = HALO_RX_ICMP_TYPE;
            return;
        }
        if (s[1] != 0) {
            r.status = HALO_RX_ICMP_CODE;
            return;
        }
        if (!sums_to_ones(sum_le(s, l4))) {  // icmp.go:53, whatever CheckSumEnable says
            r.status = HALO_RX_L4_CKSUM;
            return;
        }
        r.l4_aux = s[0];
        r.l4_seq = be32(s + 4);
        r.payload_off = (uint16_t)(O + 28);
        r.payload_len = (uint16_t)(l4 - 8);
    }
}

// The 16-byte record of a full one (HALO_RX_RECORD_COMPACT, include/halo_rx.h): the EtherType as
// its class in flags bits 4-5, as rx_parse.hip's frame_store packs it.
inline halo_rx_record16_t compact(const halo_rx_result_t& r) {
    halo_rx_record16_t c;
    const uint32_t et_class = r.ethertype == kEthArp ? HALO_RX_F_ET_ARP
                            : r.ethertype == kEthIpv6 ? HALO_RX_F_ET_IPV6
                            : r.ethertype == kEthIeee8023 ? HALO_RX_F_ET_8023 : HALO_RX_F_ET_IPV4;
    c.status = r.status;
    c.flags = (uint8_t)(r.flags | et_class);
    c.ip_proto = r.ip_proto;
    c.l4_aux = r.l4_aux;
    c.src_ip = r.src_ip;
    c.dst_ip = r.dst_ip;
    c.sport = r.sport;
    c.dport = r.dport;
    return c;
}

template <bool L3, bool COMPACT>
void parse_all(const uint8_t* bytes, const uint64_t* offsets, const uint16_t* lens, uint32_t n, const Own& own,
               void* out, uint32_t* hist) {
    constexpr uint32_t kAhead = 8;  // frames prefetched ahead of the one being parsed
    for (uint32_t i = 0; i < n; ++i) {
        if (i + kAhead < n) __builtin_prefetch(bytes + offsets[i + kAhead]);
        halo_rx_result_t r;
        parse_one<L3>(bytes + offsets[i], lens[i], own, r);
        if (COMPACT) static_cast<halo_rx_record16_t*>(out)[i] = compact(r);
        else static_cast<halo_rx_result_t*>(out)[i] = r;
        if (hist) ++hist[r.status];
    }
}

}  // namespace

extern "C" HALO_API int halo_rx_parse_batch_cpu(const uint8_t* bytes, const uint64_t* offsets, const uint16_t* lens,
                                                uint32_t n, uint32_t flags, const halo_rx_netif_t* netif,
                                                halo_rx_result_t* out, uint32_t* status_hist) {
    if (!netif) return HALO_E_INVAL;
    if (flags & ~(HALO_RX_CSUM_ENABLE | HALO_RX_JUMBO_EXT | HALO_RX_RECORD_COMPACT | HALO_RX_UNIFORM_LEN |
                  HALO_RX_L3_START | HALO_RX_VARIANT_MASK))
        return HALO_E_INVAL;
    if (n == 0) return HALO_OK;
    if (!bytes || !offsets || !lens || !out) return HALO_E_INVAL;
    Own own;
    memcpy(&own.mac_lo, netif->mac, 4);
    own.mac_hi = le16(netif->mac + 4);
    own.ip = netif->ip;
    own.csum = (flags & HALO_RX_CSUM_ENABLE) != 0;
    own.jumbo = (flags & HALO_RX_JUMBO_EXT) != 0;
    const bool l3 = (flags & HALO_RX_L3_START) != 0, c16 = (flags & HALO_RX_RECORD_COMPACT) != 0;
    if (l3 && c16) parse_all<true, true>(bytes, offsets, lens, n, own, out, status_hist);
    else if (l3) parse_all<true, false>(bytes, offsets, lens, n, own, out, status_hist);
    else if (c16) parse_all<false, true>(bytes, offsets, lens, n, own, out, status_hist);
    else parse_all<false, false>(bytes, offsets, lens, n, own, out, status_hist);
    return HALO_OK;
}

extern "C" HALO_API const char* halo_rx_cpu_version(void) { return "halo_rx_cpu 1.0 (host, no HIP)"; }
