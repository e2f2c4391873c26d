// flow_key.h — the NAT flow key of a parsed record and its XXH3-64, shared
// by the standalone flow-hash kernel (flow_hash.hip) and the rx kernels' fused pass (rx_parse.hip,
// halo_rx_parse_flow_batch_device), so the two produce the same bits by construction.
//
//   key (13 bytes, little-endian): remote ip u32 | remote port u16 | local ip u32 | local port u16
//   | proto u8 — NatFlowHash / NatWanFlowHash (engine/ipv4_engine.go:451-479) as NatGetFlowByHash /
//   NatGetFlowByWan build them (:524-581); hashed by hashcode.GetHashCodeXXH3 (hashcode/xxh3.go,
//   hashSmall for 9..16 bytes, :62-66: default secret, seed 0).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/halo_rx.h"

namespace halo {
namespace flowkey {

// secret64(24) ^ secret64(32) and secret64(40) ^ secret64(48) of hashcode/xxh3.go:27-40
constexpr uint64_t kSecLo = 0x1f67b3b7a4a44072ull ^ 0x78e5c0cc4ee679cbull;
constexpr uint64_t kSecHi = 0x2172ffcc7dd05a82ull ^ 0x8e2443f7744608b8ull;

__device__ __forceinline__ uint64_t mul_fold64(uint64_t a, uint64_t b) { return (a * b) ^ __umul64hi(a, b); }

// hashSmall for 9..16 bytes (xxh3.go:62-66) given the two overlapping 8-byte words
__device__ __forceinline__ uint64_t hash_9to16(uint64_t w_lo, uint64_t w_hi, uint32_t len) {
    const uint64_t lo = w_lo ^ kSecLo, hi = w_hi ^ kSecHi;
    uint64_t v = (uint64_t)len + __builtin_bswap64(lo) + hi + mul_fold64(lo, hi);
    v ^= v >> 37;  // avalanche (xxh3.go:238-243)
    v *= 0x165667919e3779f9ull;
    return v ^ (v >> 32);
}

// The flow key of a record (proto, IpAddrToU src/dst, ports as NatGetSrcDstPort gives them) and
// its hash. kind: HALO_FLOW_NAT_LAN / HALO_FLOW_NAT_WAN; nat_type: HALO_NAT_SYMMETRIC or other.
__device__ __forceinline__ uint64_t nat_hash(uint32_t proto, uint32_t src, uint32_t dst, uint32_t sport,
                                             uint32_t dport, uint32_t kind, uint32_t nat_type) {
    const bool wan = kind == HALO_FLOW_NAT_WAN;
    // NatGetFlowByWan(src, sport, dst, dport) / NatGetFlowByHash(dst, dport, src, sport)
    uint32_t rip = wan ? src : dst, rport = wan ? sport : dport;
    const uint32_t lip = wan ? dst : src, lport = wan ? dport : sport;
    if (nat_type != HALO_NAT_SYMMETRIC) { rip = 0; rport = 0; }  // :528-534
    if (proto == 1u) rport = 0;                                    // ICMP, :535-537
    const uint64_t w_lo = (uint64_t)rip | (uint64_t)rport << 32 | (uint64_t)(lip & 0xFFFFu) << 48;
    const uint64_t w_hi = (uint64_t)(rport >> 8) | (uint64_t)lip << 8 | (uint64_t)lport << 40 |
                          (uint64_t)proto << 56;  // key bytes 5..12
    return hash_9to16(w_lo, w_hi, 13);
}

}  // namespace flowkey
}  // namespace halo
