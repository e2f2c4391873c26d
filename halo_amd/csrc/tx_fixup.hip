// tx_fixup.hip — SURVEY.md §8f row f2 on gfx950: the forward / transmit direction of halo's
// packet path, rewritten in place over a batch of frames resident in HBM.
//
// Restates bit-exactly, per frame (pkt = frame[14:len], engine/ipv4_engine.go:31-37):
//   NatChangeDst / NatChangeSrc   protocol/ipv4.go:277-302, :249-275
//   HandleIpv4PktTtl              protocol/ipv4.go:134-145
//   ReCalcIpv4 / Icmp / Tcp / UdpCheckSum   protocol/ipv4.go:148-226
//   eth_tx software checksum fill cgo/dpdk.c:333-365 (DPDK 20.11 rte_ipv4_cksum /
//                                  rte_ipv4_udptcp_cksum, restated in oracle/halo_tx_oracle.c)
// in the order Ipv4RouteForward applies them (engine/ipv4_engine.go:108-269).
//
// Shape: the rx kernel's (rx_parse.hip) — G lanes of a wave per frame, 16-byte loads, header
// dwords 0..12 broadcast to the group. Every step only rewrites header bytes (< 52), and every
// checksum the steps ask for is a function of the FINAL packet bytes (no checksum field lies in
// another checksum's range), so the steps are first applied to a register copy of the header,
// then each needed checksum is summed once over the final bytes: header dwords from the copy,
// the rest of the frame from the loads. Sums are taken in the little-endian dword domain (see
// rx_parse.hip): the stored field, read as a little-endian half-word, is ~fold(sum) — for the
// Go functions (big-endian store of ^fold(BE sum)) and for DPDK (host-order store of
// ~rte_raw_cksum) alike. One lane per frame then writes the dirty header dwords back.
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "halo_common.h"

namespace halo {
namespace {

struct TxParams {
    uint8_t* bytes;
    const uint32_t* offsets_dw;
    const uint16_t* lens;
    const halo_tx_op_t* ops;
    uint32_t n;
    uint32_t flags;
    uint8_t* result;
};

constexpr uint32_t kGoSteps = HALO_TX_NAT_DST | HALO_TX_TTL | HALO_TX_NAT_SRC | HALO_TX_RECALC;
constexpr uint32_t kHdrDw = 13;  // header dwords 0..12 (frame bytes 0..51: up to the TCP checksum)


// byte b of the header copy / a big-endian 16-bit field at even frame offset b
#define MB(b) ((m[(b) >> 2] >> (((b)&3) * 8)) & 0xFFu)
#define SET_BE16(b, v)                                                                              \
    do {                                                                                            \
        constexpr uint32_t sh_ = ((b)&2) * 8;                                                       \
        m[(b) >> 2] = (m[(b) >> 2] & ~(0xFFFFu << sh_)) | (bswap16((uint32_t)(v)&0xFFFFu) << sh_); \
        dirty |= 1u << ((b) >> 2);                                                                  \
    } while (0)
#define SET_LE16(b, v)                                                                              \
    do {                                                                                            \
        constexpr uint32_t sh_ = ((b)&2) * 8;                                                       \
        m[(b) >> 2] = (m[(b) >> 2] & ~(0xFFFFu << sh_)) | (((uint32_t)(v)&0xFFFFu) << sh_);         \
        dirty |= 1u << ((b) >> 2);                                                                  \
    } while (0)

// bytes of dword d inside [lo, hi)
__device__ __forceinline__ uint32_t range_keep(uint32_t d, uint32_t lo, uint32_t hi) {
    const int32_t s = (int32_t)lo - (int32_t)(4u * d);
    const int32_t e = (int32_t)hi - (int32_t)(4u * d);
    const uint32_t k_hi = e >= 4 ? 0xFFFFFFFFu : (e <= 0 ? 0u : ((1u << (e * 8)) - 1u));
    const uint32_t k_lo = s <= 0 ? 0xFFFFFFFFu : (s >= 4 ? 0u : ~((1u << (s * 8)) - 1u));
    return k_hi & k_lo;
}

// [lo, hi) restricted to the header copy (dwords 3..12); sum of half-words, < 2^21
__device__ __forceinline__ uint32_t header_sum(const uint32_t (&m)[kHdrDw], uint32_t lo, uint32_t hi) {
    uint32_t s = 0;
#pragma unroll
    for (uint32_t d = 3; d < kHdrDw; ++d) s += hsum(m[d] & range_keep(d, lo, hi));
    return s;
}

// The two ranges almost every frame sums, in constant form: the IPv4 header [14, 34) (IHL 5) and
// the L4 part of the header copy [34, hi) for hi >= 52 (dword 8's high half, dwords 9..12). When
// every lane of the wave has that range (one wave-uniform test) the generic masked sum (ten
// range_keep masks) is skipped; round 2 spent ~40 % of tx_fixup's VALU there.
__device__ __forceinline__ uint32_t ip_header_sum(const uint32_t (&m)[kHdrDw], uint32_t hi) {
    const uint32_t fast = (m[3] >> 16) + hsum(m[4]) + hsum(m[5]) + hsum(m[6]) + hsum(m[7]) + (m[8] & 0xFFFFu);
    if (__builtin_amdgcn_ballot_w64(hi != 34u) == 0) return fast;
    return hi == 34u ? fast : header_sum(m, 14, hi);
}
__device__ __forceinline__ uint32_t l4_header_sum(const uint32_t (&m)[kHdrDw], uint32_t hi) {
    const uint32_t fast = (m[8] >> 16) + hsum(m[9]) + hsum(m[10]) + hsum(m[11]) + hsum(m[12]);
    if (__builtin_amdgcn_ballot_w64(hi < 4u * kHdrDw) == 0) return fast;
    return hi >= 4u * kHdrDw ? fast : header_sum(m, 34, hi);
}

// bytes [4*kHdrDw, hi) of the loaded dwords [d0, d0+4); the header part comes from the copy
__device__ __forceinline__ void acc_tail(const uint32_t (&w)[4], uint32_t d0, uint32_t hi, uint64_t& c) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t d = d0 + j;
        const int32_t rel = (int32_t)hi - (int32_t)(4u * d);
        uint32_t keep = rel >= 4 ? 0xFFFFFFFFu : (rel <= 0 ? 0u : ((1u << (rel * 8)) - 1u));
        keep = d >= kHdrDw ? keep : 0u;
        c += (uint64_t)(w[j] & keep);
    }
}

struct TxPlan {
    uint32_t ip_hi;                        // IPv4 header checksum over [14, ip_hi); 0: none
    uint32_t go_hi, go_extra, go_field;    // Go ReCalc L4 checksum over [34, go_hi) + pseudo; 0: none
    uint32_t dp_hi, dp_extra, dp_field;    // DPDK L4 checksum over [34, dp_hi) + pseudo; 0: none
    uint32_t dp_zero;                      // L4 field DPDK zeroes (before its sum, after the IPv4 sum)
    bool udp_zero_ffff;                    // DPDK: a zero UDP checksum is sent as 0xFFFF
};

// Apply the steps to the header copy; returns the checksum plan. All lanes of a group run this
// on identical inputs. `skip`/`alive`/`overrun` feed the result byte.
__device__ __forceinline__ TxPlan apply_steps(uint32_t (&m)[kHdrDw], uint32_t& dirty, uint32_t L, uint32_t steps,
                                              uint32_t dst_ip, uint32_t dst_port, uint32_t src_ip,
                                              uint32_t src_port, bool en, uint32_t& res) {
    TxPlan pl{0, 0, 0, 0, 0, 0, 0, 0, false};
    bool skip = false;
    if (L < 14) {  // no IPv4 packet: every Go step returns on its length guard
        res = (steps & kGoSteps) ? HALO_TX_R_SKIPPED : 0u;
        return pl;
    }
    const uint32_t len = L - 14;
    const uint32_t proto = MB(23);
    bool ip_go = false;   // a Go ReCalcIpv4CheckSum ran
    uint32_t l4_go = 0;   // the Go L4 recalc that ran: 1 ICMP, 6 TCP, 17 UDP

    // Go ReCalc* on the current packet (their guards; the field is (re)computed at the end)
    auto recalc_ip = [&]() { if (len < 20) skip = true; else ip_go = true; };
    auto recalc_l4 = [&]() {
        if (proto == kIpIcmp) { if (len < 24) skip = true; else l4_go = kIpIcmp; }
        else if (proto == kIpTcp) { if (len < 38) skip = true; else l4_go = kIpTcp; }
        else if (proto == kIpUdp) { if (len < 28) skip = true; else l4_go = kIpUdp; }
    };
    bool alive = true;
    if (steps & HALO_TX_NAT_DST) {  // protocol/ipv4.go:277-302
        if (len < 26) {
            skip = true;
        } else {
            SET_BE16(30, dst_ip >> 16);
            SET_BE16(32, dst_ip);
            recalc_ip();
            // ICMP: echo identifier (frame 38..39), TCP/UDP: destination port (36..37); both in
            // dword 9 (selects, not branches: branches let the compiler index m dynamically)
            const uint32_t pw = bswap16(dst_port & 0xFFFFu);
            const bool icmp = proto == kIpIcmp, tu = proto == kIpTcp || proto == kIpUdp;
            m[9] = icmp ? (m[9] & 0xFFFFu) | (pw << 16) : tu ? (m[9] & 0xFFFF0000u) | pw : m[9];
            dirty |= (icmp || tu) ? 1u << 9 : 0u;
            recalc_l4();
        }
    }
    if (steps & HALO_TX_TTL) {  // protocol/ipv4.go:134-145
        if (len < 9) {
            skip = true;
            alive = false;
        } else if (MB(22) <= 1u) {
            alive = false;
        } else {
            m[5] -= 1u << 16;  // pkt[8]-- (frame byte 22, > 1 so no borrow)
            dirty |= 1u << 5;
            recalc_ip();
        }
    }
    if (alive) {
        if (steps & HALO_TX_NAT_SRC) {  // protocol/ipv4.go:249-275
            if (len < 26) {
                skip = true;
            } else {
                SET_BE16(26, src_ip >> 16);
                SET_BE16(28, src_ip);
                recalc_ip();
                // ICMP: echo identifier (frame 38..39, dword 9), TCP/UDP: source port (34..35, dword 8)
                const uint32_t pw = bswap16(src_port & 0xFFFFu);
                const bool icmp = proto == kIpIcmp, tu = proto == kIpTcp || proto == kIpUdp;
                m[9] = icmp ? (m[9] & 0xFFFFu) | (pw << 16) : m[9];
                m[8] = tu ? (m[8] & 0xFFFFu) | (pw << 16) : m[8];
                dirty |= (icmp ? 1u << 9 : 0u) | (tu ? 1u << 8 : 0u);
                recalc_l4();
            }
        }
        if (steps & HALO_TX_RECALC) {
            recalc_ip();
            if (len >= 10) recalc_l4();
        }
    }
    res = (alive && (steps & HALO_TX_TTL) ? HALO_TX_R_TTL_ALIVE : 0u) | (skip ? HALO_TX_R_SKIPPED : 0u);

    // Go checksums: field zeroed; summed when CheckSumEnable (ICMP: always)
    if (ip_go) {
        SET_LE16(24, 0);
        if (en) pl.ip_hi = 34;
    }
    const uint32_t sum_addrs = (m[6] >> 16) + hsum(m[7]) + (m[8] & 0xFFFFu);  // pseudo src+dst
    if (l4_go == kIpIcmp) {
        SET_LE16(36, 0);
        pl.go_hi = L;
        pl.go_field = 36;
    } else if (l4_go) {
        const uint32_t f = l4_go == kIpTcp ? 50u : 40u;
        if (f == 50u) SET_LE16(50, 0);
        else SET_LE16(40, 0);
        if (en) {
            const uint32_t total_len = bswap16(m[4] & 0xFFFFu);  // frame bytes 16..17
            pl.go_hi = L;
            pl.go_field = f;
            pl.go_extra = sum_addrs + (l4_go << 8) + bswap16((total_len - 20u) & 0xFFFFu);  // Go int, 2 bytes
        }
    }

    // eth_tx software fill (cgo/dpdk.c:333-365), after everything else. Its IPv4 sum covers
    // IHL*4 bytes, which for IHL >= 7 include the UDP (>= 10: TCP) checksum field as the Go
    // steps left it; the field is zeroed only after that sum (dpdk.c:345 then :350).
    if (alive && (steps & HALO_TX_DPDK_FILL) && (m[3] & 0xFFFFu) == 0x0008u) {
        if (L < 34) {
            res |= HALO_TX_R_OVERRUN;
        } else {
            SET_LE16(24, 0);
            const uint32_t ihl4 = (MB(14) & 0xFu) * 4u;
            if (14u + ihl4 <= L) pl.ip_hi = 14u + ihl4;
            else { pl.ip_hi = 0; res |= HALO_TX_R_OVERRUN; }
            if (proto == kIpUdp || proto == kIpTcp) {
                const uint32_t f = proto == kIpUdp ? 40u : 50u;
                if (f + 2u > L) {
                    res |= HALO_TX_R_OVERRUN;  // (a Go L4 recalc cannot have run: its guard is stricter)
                } else {
                    pl.dp_zero = f;
                    if (pl.ip_hi <= f) pl.go_hi = 0;  // the Go value is overwritten unseen
                    const uint32_t l3 = bswap16(m[4] & 0xFFFFu);
                    if (l3 >= ihl4) {
                        const uint32_t l4_len = l3 - ihl4;
                        if (34u + l4_len > L) {
                            res |= HALO_TX_R_OVERRUN;
                        } else {
                            pl.dp_hi = 34u + l4_len;
                            pl.dp_field = f;
                            pl.dp_extra = sum_addrs + (proto << 8) + bswap16(l4_len);
                            pl.udp_zero_ffff = proto == kIpUdp;
                        }
                    }
                }
            }
        }
    }
    return pl;
}

template <int G>
__device__ __forceinline__ void tx_frame(const TxParams& p, uint32_t i, bool present, uint32_t gl, uint32_t grp_base) {
    constexpr uint32_t STEP = 4 * G;  // dwords per group per load step
    constexpr int U0 = 4;             // 16-byte chunks per lane in round 0 (>= the 52-byte header)
    constexpr int U = 4;
    uint8_t* frame = p.bytes;
    uint32_t L = 0;
    uint4 op = make_uint4(0, 0, 0, 0);
    if (present) {
        frame = p.bytes + ((uint64_t)p.offsets_dw[i] << 2);
        L = p.lens[i];
        op = reinterpret_cast<const uint4*>(p.ops)[i];
    }
    const uint32_t steps = op.x & 0xFFu;
    const uint32_t ndw = (present && L >= 14 && steps) ? (L + 3) >> 2 : 0;  // nothing is read for no work
    uint32_t buf[U0][4];
#pragma unroll
    for (int u = 0; u < U0; ++u) load4(frame, (u * G + gl) * 4, ndw, buf[u]);
    uint32_t m[kHdrDw];
    if constexpr (G == 1) {
#pragma unroll
        for (uint32_t j = 0; j < kHdrDw; ++j) m[j] = buf[j >> 2][j & 3];
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            m[j] = group_bcast<G, 0>(buf[0][j], grp_base);
            m[4 + j] = group_bcast<G, 1>(buf[0][j], grp_base);
            m[8 + j] = group_bcast<G, 2>(buf[0][j], grp_base);
        }
        m[12] = group_bcast<G, 3>(buf[0][0], grp_base);
    }
    uint32_t dirty = 0, res = 0;
    const TxPlan pl = apply_steps(m, dirty, L, steps, op.y,
                                  op.x >> 16, op.w, op.z & 0xFFFFu, (p.flags & HALO_RX_CSUM_ENABLE) != 0, res);

    // Sums over the final bytes: the header copy + this lane's loaded dwords past it. One pass
    // accumulates the IPv4 tail (IHL >= 10 only) and the first L4 range; the second L4 range
    // (Go value overwritten by DPDK but covered by an IHL >= 7 IPv4 sum) takes a second pass.
    const uint32_t l4a = pl.go_hi ? pl.go_hi : pl.dp_hi;        // first L4 range
    const uint32_t l4b = pl.go_hi ? pl.dp_hi : 0u;              // second (rare)
    uint64_t c_ip = 0, c_a = 0, c_b = 0;
    const uint32_t hi = pl.ip_hi > l4a ? pl.ip_hi : l4a;
    if (hi > 4 * kHdrDw) {
#pragma unroll
        for (int u = 0; u < U0; ++u) {
            if (pl.ip_hi > 4 * kHdrDw) acc_tail(buf[u], (u * G + gl) * 4, pl.ip_hi, c_ip);
            acc_tail(buf[u], (u * G + gl) * 4, l4a, c_a);
        }
        const uint32_t seg_dw = (hi + 3) >> 2;
        for (uint32_t r0 = U0 * STEP; r0 < seg_dw; r0 += U * STEP) {
            uint32_t x[U][4];
#pragma unroll
            for (int u = 0; u < U; ++u) load4(frame, r0 + (u * G + gl) * 4, seg_dw, x[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (pl.ip_hi > 4 * kHdrDw) acc_tail(x[u], r0 + (u * G + gl) * 4, pl.ip_hi, c_ip);
                acc_tail(x[u], r0 + (u * G + gl) * 4, l4a, c_a);
            }
        }
    }
    if (l4b > 4 * kHdrDw) {
        const uint32_t seg_dw = (l4b + 3) >> 2;
        for (uint32_t r0 = 0; r0 < seg_dw; r0 += U * STEP) {
            uint32_t x[U][4];
#pragma unroll
            for (int u = 0; u < U; ++u) load4(frame, r0 + (u * G + gl) * 4, seg_dw, x[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) acc_tail(x[u], r0 + (u * G + gl) * 4, l4b, c_b);
        }
    }
    const uint32_t g_ip = group_sum<G>(fold64(c_ip));
    const uint32_t g_a = group_sum<G>(fold64(c_a));
    const uint32_t g_b = l4b ? group_sum<G>(fold64(c_b)) : 0u;
    auto set_l4 = [&](uint32_t field, uint32_t v) {
        if (field == 36u) SET_LE16(36, v);
        else if (field == 40u) SET_LE16(40, v);
        else SET_LE16(50, v);
    };
    // the reference's order: Go L4 (NAT / RECALC), then the IPv4 header, then DPDK's L4
    if (pl.go_hi) {
        const uint32_t s = fold16(fold64((uint64_t)g_a + l4_header_sum(m, pl.go_hi) + pl.go_extra));
        set_l4(pl.go_field, ~s);
    }
    if (pl.ip_hi) {
        const uint32_t s = fold16(fold64((uint64_t)g_ip + ip_header_sum(m, pl.ip_hi)));
        SET_LE16(24, ~s);
    }
    if (pl.dp_zero) set_l4(pl.dp_zero, 0u);
    if (pl.dp_hi) {
        const uint32_t g = pl.go_hi ? g_b : g_a;
        const uint32_t s = fold16(fold64((uint64_t)g + l4_header_sum(m, pl.dp_hi) + pl.dp_extra));
        uint32_t f = (~s) & 0xFFFFu;
        if (pl.udp_zero_ffff && f == 0) f = 0xFFFFu;
        set_l4(pl.dp_field, f);
    }

    if constexpr (G >= 4) {
        // lane gl owns header chunk gl (dwords 4gl..4gl+3; chunk 0 is never dirty): one 16-byte
        // store per dirty chunk, so a store instruction covers 64 / G frames' chunks side by side
        if (present) {
            const uint32_t cd = gl >= 1 && gl <= 3 ? (dirty >> (4 * gl)) & 0xFu : 0u;
            if (cd) {
                uint32_t v[4];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    v[q] = gl == 1 ? m[4 + q] : gl == 2 ? m[8 + q] : (q == 0 ? m[12] : buf[0][q]);
                uint32_t* fw = reinterpret_cast<uint32_t*>(frame) + 4 * gl;
                if (16 * gl + 16 <= L) {
                    *reinterpret_cast<uint4*>(fw) = make_uint4(v[0], v[1], v[2], v[3]);
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t d = 4 * gl + q;
                        if (!((cd >> q) & 1u)) continue;
                        if (4 * d + 4 <= L) fw[q] = v[q];
                        else
                            for (uint32_t b = 4 * d; b < L; ++b) frame[b] = (uint8_t)(v[q] >> ((b & 3) * 8));
                    }
                }
            }
            if (gl == 0 && p.result) p.result[i] = (uint8_t)res;
        }
        return;
    }
    if (present && gl == 0) {
        // dirty header dwords back to the frame: 16-byte stores for dwords 4..7 and 8..11 when
        // they lie inside the frame (fewer, wider store instructions; the clean dwords among
        // them are rewritten with their own values), single dwords / bytes otherwise. Each frame's
        // stores land in one 64-byte HBM write request (TCC_EA0_WRREQ_64B: 1.016 per frame,
        // profiles/r03/r3f/tx_fixup_write_requests.json), the floor for a frame with a dirty byte;
        // writing the whole 64 bytes measured 33.4 -> 40.4 us and non-temporal stores neutral
        // (profiles/r03/r3f/ab_tx_store.log); staging the frames in LDS and storing the dirty chunks
        // (or whole lines) four lanes per frame 33.0 -> 39.4 (38.5) us (profiles/r03/r3j/ab_txc.log)
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
        __attribute__((address_space(1))) uint32_t* fw =
            (__attribute__((address_space(1))) uint32_t*)reinterpret_cast<uint32_t*>(frame);
        uint32_t rest = dirty;
#define TX_ST4(d, a, b, c, e) (*(__attribute__((address_space(1))) u32x4*)(fw + (d)) = (u32x4){a, b, c, e})
        if ((rest & 0x0F0u) && L >= 32) {
            TX_ST4(4, m[4], m[5], m[6], m[7]);
            rest &= ~0x0F0u;
        }
        if ((rest & 0xF00u) && L >= 48) {
            TX_ST4(8, m[8], m[9], m[10], m[11]);
            rest &= ~0xF00u;
        }
#undef TX_ST4
#pragma unroll
        for (uint32_t d = 3; d < kHdrDw; ++d) {
            if (rest & (1u << d)) {
                if (4 * d + 4 <= L) {
                    fw[d] = m[d];
                } else {
                    for (uint32_t b = 4 * d; b < L; ++b) frame[b] = (uint8_t)(m[d] >> ((b & 3) * 8));
                }
            }
        }
        if (p.result) p.result[i] = (uint8_t)res;
    }
}
#undef MB
#undef SET_BE16
#undef SET_LE16

// Lane-per-frame (G = 1) launch shape: one-wave blocks with 8 KB of dynamic LDS padding each,
// so 20 blocks = 5 waves per SIMD are resident instead of 6 (by registers): fewer frame bytes in
// flight per CU, 35.6 -> 33.6 us per 1M x 64 B (profiles/r02/ab_tx_block.log; 4 and 5.5 waves and
// plain one-wave blocks measured between). G > 1 keeps 256-thread blocks (not measured).
#ifndef HALO_TX_G1_BLOCK
#define HALO_TX_G1_BLOCK 64
#endif
#ifndef HALO_TX_G1_LDS_PAD
#define HALO_TX_G1_LDS_PAD 8192
#endif

template <int G>
constexpr uint32_t kTxBlock = G == 1 ? HALO_TX_G1_BLOCK : 256;
template <int G>
__global__ void __launch_bounds__(kTxBlock<G>) tx_fixup_kernel(const TxParams p) {
    constexpr uint32_t FPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane & (G - 1);
    const uint32_t grp_base = lane & ~(uint32_t)(G - 1);
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t base = wave * FPW; base < p.n; base += nwaves * FPW) {
        const uint32_t i = base + lane / G;
        tx_frame<G>(p, i, i < p.n, gl, grp_base);
    }
}

uint32_t tx_grid(uint64_t n, uint32_t frames_per_wave, uint64_t wpb) {
    const uint64_t waves = (n + frames_per_wave - 1) / frames_per_wave;
    const uint64_t blocks = (waves + wpb - 1) / wpb;
    const uint64_t kMaxBlocks = 256ull * 8 * 8 * 4 / wpb;
    return (uint32_t)(blocks > kMaxBlocks ? kMaxBlocks : blocks);
}

}  // namespace
}  // namespace halo

extern "C" HALO_API int halo_tx_fixup_batch_device(uint8_t* d_bytes, const uint32_t* d_offsets_dw,
                                                   const uint16_t* d_lens, uint32_t n,
                                                   const halo_tx_op_t* d_ops, uint32_t flags,
                                                   uint32_t max_len_hint, uint8_t* d_result,
                                                   halo_stream_t stream) {
    if (flags & ~(uint32_t)HALO_RX_CSUM_ENABLE) return HALO_E_INVAL;
    if (n == 0) return HALO_OK;
    if (!d_bytes || !d_offsets_dw || !d_lens || !d_ops) return HALO_E_INVAL;
    if (reinterpret_cast<uintptr_t>(d_bytes) & 3u || reinterpret_cast<uintptr_t>(d_ops) & 15u) return HALO_E_INVAL;
    int rc = halo::check_device();
    if (rc) return rc;
    halo::TxParams p{d_bytes, d_offsets_dw, d_lens, d_ops, n, flags, d_result};
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 block(256), block1(HALO_TX_G1_BLOCK);
    // lanes per frame from the longest frame (0: unknown -> widest); any G handles any length
    const uint32_t h = max_len_hint ? max_len_hint : 65535u;
#ifndef HALO_TX_G1_MAX
#define HALO_TX_G1_MAX 128
#endif
    if (h <= HALO_TX_G1_MAX) hipLaunchKernelGGL(halo::tx_fixup_kernel<1>, dim3(halo::tx_grid(n, 64, HALO_TX_G1_BLOCK / 64)), block1, HALO_TX_G1_LDS_PAD, s, p);
    else if (h <= 1024) hipLaunchKernelGGL(halo::tx_fixup_kernel<4>, dim3(halo::tx_grid(n, 16, 4)), block, 0, s, p);
    else if (h <= 4096) hipLaunchKernelGGL(halo::tx_fixup_kernel<8>, dim3(halo::tx_grid(n, 8, 4)), block, 0, s, p);
    else hipLaunchKernelGGL(halo::tx_fixup_kernel<16>, dim3(halo::tx_grid(n, 4, 4)), block, 0, s, p);
    return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
}
