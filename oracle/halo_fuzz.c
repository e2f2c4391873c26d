/*
 * halo_fuzz.c — TEST INFRASTRUCTURE ONLY: a structured fuzzer for the receive path's parity tests.
 *
 * Builds frames the way ora_synth_frame does (valid UDP / TCP / ICMP addressed to the NetIf), then
 * applies header-targeted mutations drawn so that every check of the reference chain fails or
 * passes in combination: frame length (0..41, 42..1514, 1515..9100), EtherType (the four
 * whitelisted values of protocol/ethernet.go:39-50 and random), IP version/IHL byte
 * (ipv4.go:52), flags/fragment offset (:59), protocol (:63-72), header checksum (:74-78),
 * totalLen under/overrun/padding (:84), UDP length field (udp.go:30), TCP data offset
 * (tcp.go:49), ICMP type/code (icmp.go:38-49), L4 checksum corrupt or zero, destination MAC
 * (own / broadcast / other: ethernet_engine.go:22), destination IP (x.x.x.255 / 10.x / one bit off:
 * ipv4_engine.go:24,31), random bit flips. Checksums are re-filled after some mutations so that
 * later checks are reached. Frames are packed at 4-byte boundaries (ring-record style).
 * Only tests/ load this code.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/halo_rx.h"

#define ORA_API __attribute__((visibility("default")))

void ora_synth_frame(uint64_t seed, uint64_t index, uint32_t len, uint8_t kind, const halo_rx_netif_t* netif,
                     uint8_t* f);
uint16_t ora_get_checksum(const uint8_t* data, size_t len);

static uint64_t sm(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void put16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

/* Refill the IPv4 header checksum (frame bytes 14..33) and, for UDP/TCP/ICMP, the L4 checksum
 * over [34, 14 + totalLen) the way the reference verifies it — only when the region lies inside
 * the frame. */
static void refill(uint8_t* f, uint32_t L) {
    if (L < 34) return;
    f[24] = f[25] = 0;
    put16(f + 24, ora_get_checksum(f + 14, 20));
    const uint32_t total = ((uint32_t)f[16] << 8) | f[17];
    if (total < 28 || 14 + total > L) return;
    const uint32_t seg = total - 20, proto = f[23];
    uint8_t* s = f + 34;
    if (proto == 1) {
        s[2] = s[3] = 0;
        put16(s + 2, ora_get_checksum(s, seg));
    } else if (proto == 17 || (proto == 6 && seg >= 20)) {
        const uint32_t at = proto == 17 ? 6 : 16;
        s[at] = s[at + 1] = 0;
        uint8_t* buf = (uint8_t*)malloc(12 + seg);
        memcpy(buf, f + 26, 8);
        buf[8] = 0;
        buf[9] = (uint8_t)proto;
        put16(buf + 10, proto == 17 ? (((uint32_t)s[4] << 8) | s[5]) : seg);
        memcpy(buf + 12, s, seg);
        put16(s + at, ora_get_checksum(buf, 12 + seg));
        free(buf);
    }
}

/* Lengths and 4-byte-aligned dword offsets of n fuzzed frames (first pass) — the caller then
 * allocates 4 * total_dw bytes and calls ora_fuzz_fill with the same seed. */
ORA_API uint64_t ora_fuzz_layout(uint64_t seed, uint32_t n, uint16_t* lens, uint32_t* offsets_dw) {
    uint64_t off = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t s = seed ^ (0xD1B54A32D192ED03ull * (i + 1));
        const uint64_t r = sm(&s);
        uint32_t L;
        switch (r % 16) {
            case 0: L = (uint32_t)(sm(&s) % 42); break;                  /* ETH_LEN (short)        */
            case 1: L = 1515 + (uint32_t)(sm(&s) % 7600); break;         /* > 1514: jumbo or reject */
            case 2: L = 42 + (uint32_t)(sm(&s) % 30); break;             /* tiny IPv4               */
            case 3: L = 8990 + (uint32_t)(sm(&s) % 30); break;           /* around the jumbo caps   */
            default: L = 42 + (uint32_t)(sm(&s) % 1473); break;          /* 42..1514                */
        }
        lens[i] = (uint16_t)L;
        offsets_dw[i] = (uint32_t)(off >> 2);
        off += (L + 3u) & ~3u;
    }
    return off >> 2;
}

ORA_API void ora_fuzz_fill(uint64_t seed, uint32_t n, const uint16_t* lens, const uint32_t* offsets_dw,
                           const halo_rx_netif_t* netif, uint8_t* bytes) {
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t s = seed ^ (0xD1B54A32D192ED03ull * (i + 1)) ^ 0xA5A5A5A5ull;
        const uint32_t L = lens[i];
        uint8_t* f = bytes + ((uint64_t)offsets_dw[i] << 2);
        if (L == 0) continue;
        const uint32_t base_len = L < 60 ? 60 : L;
        uint8_t* tmp = (uint8_t*)malloc(base_len);
        ora_synth_frame(seed, i, base_len, (uint8_t)(sm(&s) % 3), netif, tmp);
        memcpy(f, tmp, L);
        free(tmp);
        if (L >= 60) {  /* totalLen follows the frame (synth wrote base_len - 14) */
        } else if (L >= 34) {
            put16(f + 16, L - 14);
            refill(f, L);
        }
        const uint32_t muts = (uint32_t)(sm(&s) % 4);
        for (uint32_t m = 0; m < muts; ++m) {
            const uint64_t r = sm(&s);
            const uint32_t what = (uint32_t)(r % 20), v = (uint32_t)(r >> 8);
            int fix = (r >> 40) & 1; /* re-fill checksums so later checks are reached */
            switch (what) {
                case 0: if (L >= 14) { static const uint16_t et[] = {0x0800, 0x0806, 0x86DD, 0x05DC}; put16(f + 12, (v & 4) ? v : et[v & 3]); } break;
                case 1: if (L >= 15) f[14] = (v & 1) ? 0x45 : (uint8_t)v; break;
                case 2: if (L >= 22) { f[20] = (v & 3) == 0 ? 0x40 : (v & 3) == 1 ? 0x00 : (uint8_t)v; f[21] = (v & 4) ? (uint8_t)(v >> 8) : 0; } break;
                case 3: if (L >= 24) { static const uint8_t pr[] = {1, 6, 17, 2}; f[23] = (v & 4) ? (uint8_t)v : pr[v & 3]; } break;
                case 4: if (L >= 26) f[24 + (v & 1)] ^= (uint8_t)(1u << ((v >> 1) & 7)); fix = 0; break;
                case 5: if (L >= 18) { const uint32_t t = (v % 4) == 0 ? (v >> 4) % 20 : (v % 4) == 1 ? L - 14 + 1 + (v >> 4) % 64 : (v % 4) == 2 ? 20 + (v >> 4) % (L > 34 ? L - 33 : 1) : L - 14; put16(f + 16, t & 0xFFFF); } break;
                case 6: if (L >= 40) put16(f + 38, (v & 1) ? v & 0xFFFF : (((uint32_t)f[16] << 8 | f[17]) - 20)); break;
                case 7: if (L >= 47) f[46] = (uint8_t)v; break;                                 /* TCP offset */
                case 8: if (L >= 36) { f[34] = (v & 3) == 0 ? 8 : (v & 3) == 1 ? 0 : (v & 3) == 2 ? 11 : (uint8_t)v; f[35] = (v & 4) ? (uint8_t)(v >> 8) : 0; } break;
                case 9: if (L >= 52) f[40 + (v % 12)] ^= (uint8_t)(1u << ((v >> 4) & 7)); fix = 0; break;  /* L4 cksum region */
                case 10: if (L >= 42) { f[40] = f[41] = 0; } fix = 0; break;                    /* UDP cksum 0 */
                case 11: if (L >= 6) { if (v & 1) memset(f, 0xFF, 6); else if (v & 2) memcpy(f, netif->mac, 6); else f[v % 6] ^= 0x10; } break;
                case 12: if (L >= 34) { if (v & 1) f[33] = 255; else if (v & 2) { f[30] = 10; f[31] = (uint8_t)v; } else f[30 + ((v >> 2) & 3)] ^= 0x01; } break;
                case 13: if (L > 14) f[14 + v % (L - 14)] ^= (uint8_t)(1u << ((v >> 16) & 7)); fix = 0; break;
                case 14: if (L >= 60 && L - 14 > 40) { put16(f + 16, L - 14 - 1 - (v % 16)); } break; /* Ethernet padding */
                default: break;
            }
            if (fix && L >= 34) refill(f, L);
        }
    }
}
