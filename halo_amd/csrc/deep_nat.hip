// deep_nat.hip — IcmpTtlDeepNat on gfx950 (SURVEY.md §8f row f2's family): the forward path's
// NAT rewrite of the packet an ICMP time-exceeded message quotes, engine/icmp_engine.go:55-86,
// called by Ipv4RouteForward on every received Ethernet payload before its own DNAT
// (engine/ipv4_engine.go:111-130):
//   ParseIpv4Pkt(ethPayload)            protocol/ipv4.go:48-86   (ICMP only)
//   ParseIcmpPkt(ipv4Payload)           protocol/icmp.go:33-63   (ICMP_TTL only)
//   quote = icmpPayload, >= 28 bytes; NatGetSrcDstPort(quote)    protocol/ipv4.go:229-246
//   NatGetFlowByWan(...)                engine/ipv4_engine.go:554-581 (the caller's NAT table)
//   NatChangeSrc(quote, LanHost)        protocol/ipv4.go:249-275 (ReCalc* of the quoted packet)
//   NatChangeDst(ethPayload, LanHost, 0) protocol/ipv4.go:277-302 (ReCalcIcmpCheckSum over the
//                                        UNTRIMMED payload, padding included, :164-174)
// ICMP errors are a slow path (a router sends them at a limited rate), so the shape is simple:
// one 64-lane wave per frame, the frame staged in the wave's LDS region, header logic evaluated
// redundantly by every lane (uniform), byte edits by lane 0, and each GetCheckSum a wave-parallel
// sum of the LDS dwords of its region in the little-endian domain (every region starts at an
// even frame offset: 34, 42, 62), as rx_parse.hip.
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "halo_common.h"

namespace halo {
namespace {

constexpr uint32_t kWaves = 4, kFrameDw = 384;  // 1536 B per wave: frames past 1514 B never qualify

struct NatParams {
    uint8_t* bytes;
    const uint32_t* offsets_dw;
    const uint16_t* lens;
    const halo_tx_deep_nat_t* nat;  // null: checks and quote records only, frames untouched
    halo_rx_result_t* quote;
    uint8_t* applied;
    uint32_t n, flags;
};

__device__ __forceinline__ uint32_t rd8(const uint8_t* b, uint32_t at) { return b[at]; }
__device__ __forceinline__ uint32_t rd16(const uint8_t* b, uint32_t at) { return ((uint32_t)b[at] << 8) | b[at + 1]; }
__device__ __forceinline__ uint32_t rd32(const uint8_t* b, uint32_t at) { return (rd16(b, at) << 16) | rd16(b, at + 2); }

// One's-complement sum (big-endian value, folded to 16 bits) of frame bytes [lo, hi), lo even,
// as GetCheckSum's accumulation (protocol/utils.go:11-28): every lane sums its dwords of the
// region in the little-endian domain, the wave reduces, one byte swap at the end.
__device__ __forceinline__ uint32_t wave_sum_be(const uint32_t* buf, uint32_t lo, uint32_t hi, uint32_t lane) {
    uint64_t s = 0;
    for (uint32_t k = (lo >> 2) + lane; 4 * k < hi; k += 64) {
        const int32_t a = (int32_t)lo - (int32_t)(4 * k), b = (int32_t)hi - (int32_t)(4 * k);
        const uint32_t mb = b >= 4 ? 0xFFFFFFFFu : (1u << (8 * b)) - 1u;
        const uint32_t ma = a <= 0 ? 0xFFFFFFFFu : ~((1u << (8 * a)) - 1u);
        s += buf[k] & ma & mb;
    }
    uint32_t x = fold64(s);
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) x += (uint32_t)__shfl_xor((int)x, m, 64);
    return bswap16(fold16(x));
}

__device__ __forceinline__ uint32_t not16(uint32_t s) { return (~s) & 0xFFFFu; }

__global__ void __launch_bounds__(64 * kWaves) deep_nat_kernel(const NatParams p) {
    __shared__ uint32_t s_buf[kWaves][kFrameDw];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * kWaves + w;
    if (i >= p.n) return;  // whole waves only
    uint32_t* buf = s_buf[w];
    uint8_t* b = reinterpret_cast<uint8_t*>(buf);
    const bool en = (p.flags & HALO_RX_CSUM_ENABLE) != 0;
    uint8_t* frame = p.bytes + ((uint64_t)p.offsets_dw[i] << 2);
    const uint32_t L = p.lens[i];
    // ---- the checks of IcmpTtlDeepNat up to its flow lookup (status as ora_icmp_quote)
    uint32_t st = HALO_RX_OK;
    if (L < 14) st = HALO_RX_ETH_LEN;
    else if (L - 14 < 20 || L - 14 > kIpMax) st = HALO_RX_IP_LEN;  // ipv4.go:49
    const uint32_t ndw = st == HALO_RX_OK ? (L + 3) >> 2 : 0;
    for (uint32_t k = lane; k < ndw; k += 64) buf[k] = reinterpret_cast<const uint32_t*>(frame)[k];
    __builtin_amdgcn_wave_barrier();
    const uint32_t P = 14, plen = L - 14;  // pkt = ethPayload = frame[14:L]
    uint32_t total_len = 0;
    if (st == HALO_RX_OK) {
        if (rd8(b, P) != 0x45u) st = HALO_RX_IP_VER;
        else if ((rd8(b, P + 6) != 0x40u && rd8(b, P + 6) != 0u) || rd8(b, P + 7) != 0u) st = HALO_RX_IP_FRAG;
        else if (rd8(b, P + 9) != kIpIcmp && rd8(b, P + 9) != kIpTcp && rd8(b, P + 9) != kIpUdp) st = HALO_RX_IP_PROTO;
    }
    if (st == HALO_RX_OK && en && not16(wave_sum_be(buf, P, P + 20, lane)) != 0u) st = HALO_RX_IP_HDR_CKSUM;
    if (st == HALO_RX_OK) {
        total_len = rd16(b, P + 2);
        if (total_len < 20) st = HALO_RX_IP_TOTLEN_UNDERFLOW;  // Go: slice panic (ipv4.go:84)
        else if (total_len > plen) st = HALO_RX_IP_TOTLEN_OVERRUN;
        else if (rd8(b, P + 9) != kIpIcmp) st = HALO_RX_IP_PROTO;  // icmp_engine.go:61-63
    }
    if (st == HALO_RX_OK) {  // ParseIcmpPkt on ipv4Payload = pkt[20:totalLen]
        const uint32_t il = total_len - 20, t = rd8(b, P + 20);
        if (il < 8 || il > kL4Max) st = HALO_RX_L4_LEN;
        else if (t != kIcmpRequest && t != kIcmpReply && t != kIcmpTtl) st = HALO_RX_ICMP_TYPE;
        else if (rd8(b, P + 21) != 0u) st = HALO_RX_ICMP_CODE;
        else if (not16(wave_sum_be(buf, P + 20, P + total_len, lane)) != 0u) st = HALO_RX_L4_CKSUM;
        else if (t != kIcmpTtl) st = HALO_RX_ICMP_TYPE;  // icmp_engine.go:71-73
        else if (total_len - 28 < 28) st = HALO_RX_L4_LEN;  // len(icmpPayload) < 28 (:74-76)
    }
    const uint32_t Q = P + 28;  // icmpPayload = ipv4Payload[8:], the quoted packet
    const uint32_t qlen = st == HALO_RX_OK ? total_len - 28 : 0;
    if (p.quote && lane == 0) {
        uint32_t proto = 0xFFu, remote = 0, wan = 0, rport = 0, wport = 0;
        if (st == HALO_RX_OK) {
            proto = rd8(b, Q + 9);
            remote = rd32(b, Q + 16);
            wan = rd32(b, Q + 12);
            if (proto == kIpIcmp) wport = rport = rd16(b, Q + 24);
            else if (proto == kIpTcp || proto == kIpUdp) { wport = rd16(b, Q + 20); rport = rd16(b, Q + 22); }
        }
        uint4* r = reinterpret_cast<uint4*>(p.quote + i);
        r[0] = make_uint4(st | (0x0800u << 16), proto, remote, wan);
        r[1] = make_uint4(rport | (wport << 16), 0u, 0u, 0u);
    }
    const bool apply = st == HALO_RX_OK && p.nat && p.nat[i].found;
    if (p.applied && lane == 0) p.applied[i] = apply ? 1u : 0u;
    if (!apply) return;
    const uint32_t lan_ip = p.nat[i].lan_ip, lan_port = p.nat[i].lan_port;
    auto put16 = [&](uint32_t at, uint32_t v) {
        if (lane == 0) { b[at] = (uint8_t)(v >> 8); b[at + 1] = (uint8_t)v; }
    };
    auto put32 = [&](uint32_t at, uint32_t v) { put16(at, v >> 16); put16(at + 2, v & 0xFFFFu); };
    auto sync = [&] { __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); };
    // ReCalcIpv4CheckSum (ipv4.go:148-161) of the IPv4 header at frame byte h
    auto recalc_ipv4 = [&](uint32_t h) {
        put16(h + 10, 0u);
        sync();
        if (en) put16(h + 10, not16(wave_sum_be(buf, h, h + 20, lane)));
        sync();
    };
    // ---- NatChangeSrc(icmpPayload, LanHostIpAddr, LanHostPort) (ipv4.go:249-275), len = qlen >= 28
    put32(Q + 12, lan_ip);
    sync();
    recalc_ipv4(Q);
    const uint32_t qp = rd8(b, Q + 9);
    if (qp == kIpIcmp) {  // ReCalcIcmpCheckSum: len >= 24
        put16(Q + 24, lan_port);
        put16(Q + 22, 0u);
        sync();
        put16(Q + 22, not16(wave_sum_be(buf, Q + 20, Q + qlen, lane)));
    } else if (qp == kIpTcp || qp == kIpUdp) {  // ReCalcTcpCheckSum (guard 38) / ReCalcUdpCheckSum (guard 28)
        put16(Q + 20, lan_port);
        const uint32_t guard = qp == kIpTcp ? 38u : 28u, at = qp == kIpTcp ? 36u : 26u;
        if (qlen >= guard) {
            put16(Q + at, 0u);
            sync();
            if (en) {  // pseudo header from the quoted header as it now is; its totalLen - 20, 16 bits
                const uint32_t pseudo = rd16(b, Q + 12) + rd16(b, Q + 14) + rd16(b, Q + 16) + rd16(b, Q + 18) + qp +
                                        ((rd16(b, Q + 2) - 20u) & 0xFFFFu);
                put16(Q + at, not16(fold16(pseudo + wave_sum_be(buf, Q + 20, Q + qlen, lane))));
            }
        }
    }
    sync();
    // ---- NatChangeDst(ethPayload, LanHostIpAddr, 0) (ipv4.go:277-302), len = plen (untrimmed)
    put32(P + 16, lan_ip);
    sync();
    recalc_ipv4(P);
    put16(P + 24, 0u);  // the ICMP "port": the time-exceeded message's unused bytes 4..5
    put16(P + 22, 0u);
    sync();
    put16(P + 22, not16(wave_sum_be(buf, P + 20, P + plen, lane)));  // pkt[20:], padding included
    sync();
    // ---- the rewritten bytes back (frame dwords 3 .. the last; bytes past L in its dword unchanged)
    for (uint32_t k = 3 + lane; k < ndw; k += 64) reinterpret_cast<uint32_t*>(frame)[k] = buf[k];
}

}  // namespace
}  // namespace halo

extern "C" HALO_API int halo_tx_icmp_deep_nat_batch_device(uint8_t* d_bytes, const uint32_t* d_offsets_dw,
                                                           const uint16_t* d_lens, uint32_t n,
                                                           const halo_tx_deep_nat_t* d_nat, uint32_t flags,
                                                           halo_rx_result_t* d_quote, uint8_t* d_applied,
                                                           halo_stream_t stream) {
    if (flags & ~HALO_RX_CSUM_ENABLE) return HALO_E_INVAL;
    if (n == 0) return HALO_OK;
    if (!d_bytes || !d_offsets_dw || !d_lens) return HALO_E_INVAL;
    if ((reinterpret_cast<uintptr_t>(d_quote) & 15u) || (reinterpret_cast<uintptr_t>(d_nat) & 3u)) return HALO_E_INVAL;
    int rc = halo::check_device();
    if (rc) return rc;
    halo::NatParams p{};
    p.bytes = d_bytes;
    p.offsets_dw = d_offsets_dw;
    p.lens = d_lens;
    p.nat = d_nat;
    p.quote = d_quote;
    p.applied = d_applied;
    p.n = n;
    p.flags = flags;
    const uint32_t grid = (n + halo::kWaves - 1) / halo::kWaves;
    hipLaunchKernelGGL(halo::deep_nat_kernel, dim3(grid), dim3(64 * halo::kWaves), 0,
                       static_cast<hipStream_t>(stream), p);
    return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
}
