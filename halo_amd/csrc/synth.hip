// synth.hip — seeded synthetic receive traffic, generated in HBM.
//
// Frames are built the way the reference's transmit side builds them (BuildEthFrm
// protocol/ethernet.go:58-82, BuildIpv4Pkt protocol/ipv4.go:89-131, BuildUdpPkt
// protocol/udp.go:52-91, BuildTcpPkt protocol/tcp.go:73-123, BuildIcmpPkt
// protocol/icmp.go:66-89) with randomised header fields and payload, addressed to the
// UsePcapDev NetIf (example/example.go:768-773) so the local-delivery branch and every L4
// checksum run. Every byte of frame i is a pure function of (seed, i): shards generate
// independently and the host twin in oracle/ reproduces them byte for byte.
#include <hip/hip_runtime.h>

#include "halo_common.h"

namespace halo {
namespace {

struct Synth {
    uint64_t key;
    uint32_t len, proto, mutated, total_len, hdr_end;
    uint32_t src_ip, dst_ip, ip_id, df, ttl, sport, dport, seq, ack, win;
    uint32_t mac_src_lo, mac_src_hi, mac_dst_lo, mac_dst_hi;
    uint32_t ip_csum, l4_csum;
};

__host__ __device__ inline Synth synth_fields(uint64_t seed, uint64_t index, uint32_t len, uint32_t kind,
                                              uint32_t dst_mac_lo, uint32_t dst_mac_hi, uint32_t dst_ip) {
    Synth f;
    f.key = synth_key(seed, index);
    f.len = len;
    f.proto = kind & 3u;
    f.mutated = (kind >> 7) & 1u;
    f.total_len = len - 14;
    f.hdr_end = f.proto == 1 ? 54 : 42;
    const uint64_t rm = synth_draw(f.key, kSlotMac);
    f.mac_src_lo = ((uint32_t)rm & 0xFFFFFFFCu) | 0x02u;  // locally administered unicast
    f.mac_src_hi = (uint32_t)(rm >> 32) & 0xFFFFu;
    f.mac_dst_lo = dst_mac_lo;
    f.mac_dst_hi = dst_mac_hi;
    const uint64_t ri = synth_draw(f.key, kSlotIp);
    f.src_ip = 0x0A000000u | ((uint32_t)ri & 0x00FFFFFFu);  // 10.0.0.0/8
    f.dst_ip = dst_ip;
    f.ip_id = (uint32_t)(ri >> 24) & 0xFFFFu;
    f.df = (uint32_t)(ri >> 40) & 1u;
    f.ttl = (uint32_t)((ri >> 48) % 255u) + 1u;
    const uint64_t rp = synth_draw(f.key, kSlotPorts);
    f.sport = (uint32_t)rp & 0xFFFFu;
    f.dport = (uint32_t)(rp >> 16) & 0xFFFFu;
    if (f.proto != 2) {  // UDP/TCP ports are non-zero
        if (!f.sport) f.sport = 1;
        if (!f.dport) f.dport = 1;
    }
    const uint64_t rs = synth_draw(f.key, kSlotSeq);
    f.seq = (uint32_t)rs;
    f.ack = (uint32_t)(rs >> 32);
    f.win = (uint32_t)synth_draw(f.key, kSlotWin) & 0xFFFFu;
    f.ip_csum = 0;
    f.l4_csum = 0;
    return f;
}

__host__ __device__ inline uint32_t payload_byte(const Synth& f, uint32_t b) {
    const uint32_t d = b >> 2;
    const uint64_t r = synth_draw(f.key, kSlotPayload + (d >> 1));
    const uint32_t dw = (uint32_t)(r >> (32 * (d & 1)));
    return (dw >> ((b & 3) * 8)) & 0xFFu;
}

// Byte b of the frame (checksum fields as currently set in f).
__host__ __device__ inline uint32_t frame_byte(const Synth& f, uint32_t b) {
    if (b >= f.hdr_end) return payload_byte(f, b);
    if (b < 4) return (f.mac_dst_lo >> (8 * b)) & 0xFFu;
    if (b < 6) return (f.mac_dst_hi >> (8 * (b - 4))) & 0xFFu;
    if (b < 10) return (f.mac_src_lo >> (8 * (b - 6))) & 0xFFu;
    if (b < 12) return (f.mac_src_hi >> (8 * (b - 10))) & 0xFFu;
    switch (b) {
        case 12: return 0x08; case 13: return 0x00;
        case 14: return 0x45; case 15: return 0x00;
        case 16: return f.total_len >> 8; case 17: return f.total_len & 0xFFu;
        case 18: return f.ip_id >> 8; case 19: return f.ip_id & 0xFFu;
        case 20: return f.df ? 0x40 : 0x00; case 21: return 0x00;
        case 22: return f.ttl;
        case 23: return f.proto == 0 ? kIpUdp : (f.proto == 1 ? kIpTcp : kIpIcmp);
        case 24: return f.ip_csum >> 8; case 25: return f.ip_csum & 0xFFu;
        case 26: case 27: case 28: case 29: return (f.src_ip >> (8 * (29 - b))) & 0xFFu;
        case 30: case 31: case 32: case 33: return (f.dst_ip >> (8 * (33 - b))) & 0xFFu;
        default: break;
    }
    const uint32_t l4len = f.total_len - 20;
    if (f.proto == 2) {  // ICMP echo request
        switch (b) {
            case 34: return kIcmpRequest; case 35: return 0x00;
            case 36: return f.l4_csum >> 8; case 37: return f.l4_csum & 0xFFu;
            case 38: return f.sport >> 8; case 39: return f.sport & 0xFFu;   // id
            default: return b == 40 ? f.dport >> 8 : f.dport & 0xFFu;         // seq
        }
    }
    switch (b) {
        case 34: return f.sport >> 8; case 35: return f.sport & 0xFFu;
        case 36: return f.dport >> 8; case 37: return f.dport & 0xFFu;
        default: break;
    }
    if (f.proto == 0) {  // UDP
        switch (b) {
            case 38: return l4len >> 8; case 39: return l4len & 0xFFu;
            case 40: return f.l4_csum >> 8; default: return f.l4_csum & 0xFFu;
        }
    }
    switch (b) {  // TCP, 20-byte header, ACK|PSH
        case 38: return f.seq >> 24; case 39: return (f.seq >> 16) & 0xFFu;
        case 40: return (f.seq >> 8) & 0xFFu; case 41: return f.seq & 0xFFu;
        case 42: return f.ack >> 24; case 43: return (f.ack >> 16) & 0xFFu;
        case 44: return (f.ack >> 8) & 0xFFu; case 45: return f.ack & 0xFFu;
        case 46: return 0x50; case 47: return 0x18;
        case 48: return f.win >> 8; case 49: return f.win & 0xFFu;
        case 50: return f.l4_csum >> 8; case 51: return f.l4_csum & 0xFFu;
        default: return 0x00;  // urgent pointer
    }
}

__device__ inline uint32_t frame_dword(const Synth& f, uint32_t d) {
    const uint32_t b0 = 4 * d;
    if (b0 >= f.hdr_end) {  // pure payload dword
        const uint64_t r = synth_draw(f.key, kSlotPayload + (d >> 1));
        return (uint32_t)(r >> (32 * (d & 1)));
    }
    return frame_byte(f, b0) | (frame_byte(f, b0 + 1) << 8) | (frame_byte(f, b0 + 2) << 16) |
           (frame_byte(f, b0 + 3) << 24);
}

__device__ inline uint32_t swap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// One wave per frame; lane l owns dwords l, l+64, ...
__global__ void __launch_bounds__(256) synth_kernel(uint64_t seed, uint64_t first_index, uint32_t n,
                                                     const uint16_t* lens, const uint32_t* offsets_dw,
                                                     uint64_t stride, const uint8_t* kinds, uint32_t mac_lo,
                                                     uint32_t mac_hi, uint32_t own_ip, uint8_t* bytes) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t k = wave; k < n; k += nwaves) {
        const uint32_t len = lens[k];
        Synth f = synth_fields(seed, first_index + k, len, kinds[k], mac_lo, mac_hi, own_ip);
        uint8_t* frame = bytes + (offsets_dw ? ((uint64_t)offsets_dw[k] << 2) : k * stride);
        const uint32_t ndw = (len + 3) >> 2;

        // IPv4 header checksum over bytes 14..33 with the field zeroed (BuildIpv4Pkt)
        uint32_t s = 0;
        for (uint32_t b = 14; b < 34; b += 2) s += (frame_byte(f, b) << 8) | frame_byte(f, b + 1);
        s = (s & 0xFFFFu) + (s >> 16);
        s = (s & 0xFFFFu) + (s >> 16);
        f.ip_csum = ~s & 0xFFFFu;

        // L4 segment [34, len) summed as little-endian dwords, checksum field zero
        uint64_t c = 0;
        for (uint32_t d = 8 + lane; d < ndw; d += 64) {
            uint32_t w = frame_dword(f, d);
            const int32_t rel = (int32_t)len - (int32_t)(4 * d);
            uint32_t keep = rel >= 4 ? 0xFFFFFFFFu : ((1u << (rel * 8)) - 1u);
            if (d == 8) keep &= 0xFFFF0000u;
            c += (uint64_t)(w & keep);
        }
        uint64_t t = (c & 0xFFFFFFFFull) + (c >> 32);
        uint32_t c32 = (uint32_t)((t & 0xFFFFull) + (t >> 16));
        for (int m = 1; m < 64; m <<= 1) c32 += __shfl_xor(c32, m, 64);
        const uint32_t l4len = f.total_len - 20;
        if (f.proto != 2) {  // pseudo header: src, dst, 0x00 proto, length (LE domain)
            c32 += swap16(f.src_ip >> 16) + swap16(f.src_ip & 0xFFFFu) + swap16(f.dst_ip >> 16) +
                   swap16(f.dst_ip & 0xFFFFu) + swap16(f.proto == 0 ? kIpUdp : kIpTcp) + swap16(l4len);
        }
        c32 = (c32 & 0xFFFFu) + (c32 >> 16);
        c32 = (c32 & 0xFFFFu) + (c32 >> 16);
        f.l4_csum = swap16(~c32 & 0xFFFFu);

        const uint32_t mut_bit = f.mutated
            ? (uint32_t)(synth_draw(f.key, kSlotMutPos) % (8ull * (len - 14))) + 8u * 14u : 0xFFFFFFFFu;
        for (uint32_t d = lane; d < ndw; d += 64) {
            uint32_t w = frame_dword(f, d);
            if ((mut_bit >> 5) == d) w ^= 1u << ((((mut_bit >> 3) & 3u) * 8) + (mut_bit & 7u));
            if (4 * d + 4 <= len) {
                reinterpret_cast<uint32_t*>(frame)[d] = w;
            } else {  // tail: leave the gap after the frame untouched
                for (uint32_t b = 4 * d; b < len; ++b) frame[b] = (uint8_t)(w >> (8 * (b & 3)));
            }
        }
    }
}

}  // namespace
}  // namespace halo

extern "C" HALO_API int halo_synth_layout(uint64_t seed, uint64_t first_index, uint32_t n, uint32_t size_mode,
                                          uint32_t len, uint32_t proto_mode, uint32_t mutate_shift,
                                          uint16_t* lens, uint32_t* offsets_dw, uint8_t* kinds,
                                          uint64_t* total_bytes) {
    if (size_mode > 1 || proto_mode > 3 || mutate_shift > 63) return HALO_E_INVAL;
    if (size_mode == 0 && (len < 60 || len > halo::kEthMaxJumbo)) return HALO_E_INVAL;
    if (n && (!lens || !kinds)) return HALO_E_INVAL;
    uint64_t off = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const uint64_t key = halo::synth_key(seed, first_index + k);
        uint32_t L = len;
        if (size_mode == 1) {  // IMIX 64/570/1500 at 7:4:1
            const uint32_t r = (uint32_t)(halo::synth_draw(key, halo::kSlotSize) % 12u);
            L = r < 7 ? 64 : (r < 11 ? 570 : 1500);
        }
        uint32_t proto = proto_mode;
        if (proto_mode == 3) {  // UDP 50 / TCP 40 / ICMP 10
            const uint32_t r = (uint32_t)(halo::synth_draw(key, halo::kSlotProto) % 10u);
            proto = r < 5 ? 0 : (r < 9 ? 1 : 2);
        }
        uint32_t mut = 0;
        if (mutate_shift)
            mut = (halo::synth_draw(key, halo::kSlotMutate) & ((1ull << mutate_shift) - 1)) == 0;
        lens[k] = (uint16_t)L;
        kinds[k] = (uint8_t)(proto | (mut << 7));
        if (offsets_dw) {
            if ((off >> 2) > 0xFFFFFFFFull) return HALO_E_RANGE;
            offsets_dw[k] = (uint32_t)(off >> 2);
        }
        off += (L + 3u) & ~3u;
    }
    if (total_bytes) *total_bytes = off;
    return HALO_OK;
}

extern "C" HALO_API int halo_synth_frames_device(uint64_t seed, uint64_t first_index, uint32_t n,
                                                 const uint16_t* d_lens, const uint32_t* d_offsets_dw,
                                                 uint64_t stride, const uint8_t* d_kinds,
                                                 const halo_rx_netif_t* netif, uint8_t* d_bytes,
                                                 halo_stream_t stream) {
    if (n == 0) return HALO_OK;
    if (!d_lens || !d_kinds || !netif || !d_bytes) return HALO_E_INVAL;
    if (!d_offsets_dw && (stride & 3u)) return HALO_E_INVAL;
    int rc = halo::check_device();
    if (rc) return rc;
    const uint32_t mac_lo = (uint32_t)netif->mac[0] | ((uint32_t)netif->mac[1] << 8) |
                            ((uint32_t)netif->mac[2] << 16) | ((uint32_t)netif->mac[3] << 24);
    const uint32_t mac_hi = (uint32_t)netif->mac[4] | ((uint32_t)netif->mac[5] << 8);
    uint64_t blocks = ((uint64_t)n + 3) / 4;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(halo::synth_kernel, dim3((uint32_t)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                       seed, first_index, n, d_lens, d_offsets_dw, stride, d_kinds, mac_lo, mac_hi, netif->ip,
                       d_bytes);
    return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
}
