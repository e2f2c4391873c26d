/*
 * halo_xxh3_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline for SURVEY.md
 * §8f row f3, flow-key hashing). Linked into oracle/liboracle.so; never into the product.
 *
 * Restates /root/reference/hashcode/xxh3.go (a trimmed port of github.com/zeebo/xxh3 v1.1.0:
 * XXH3-64, default secret, seed 0 — xxh3.go:1-2) function by function:
 *   xxh3HashCode   xxh3.go:43-56     hashSmall   :59-91     hashMedium  :94-113
 *   hashLarge      :116-129          hashLong    :132-146   accumulateLong :149-178
 *   accumulateStripe :181-209        scramble    :212-218   mix16 :221-225
 *   avalancheSmall :228-235          avalanche   :238-243   rrmxmx :246-253
 *   multiplyFold64 :256-259
 * and the key packing of the reference's flow tables:
 *   NatFlowHash.GetHashCode     engine/ipv4_engine.go:451-459  (13 B little-endian key)
 *   NatWanFlowHash.GetHashCode  engine/ipv4_engine.go:471-479
 *   key normalisation (NatType, ICMP)  NatGetFlowByHash :524-551, NatGetFlowByWan :554-581
 *
 * Pinning: the Go code cannot run here; this restatement is checked against the published
 * XXH3-64 sanity vectors (xxHash's sanity buffer, seed 0) in tests/test_flow_hash_oracle.py and
 * against the independent Python restatement oracle/ref_xxh3_py.py.
 */
#include <stdint.h>
#include <string.h>

#include "../include/halo_rx.h"

#define ORA_API __attribute__((visibility("default")))

static const uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

#define P32_1 2654435761ull
#define P32_2 2246822519ull
#define P32_3 3266489917ull
#define P64_1 11400714785074694791ull
#define P64_2 14029467366897019727ull
#define P64_3 1609587929392839161ull
#define P64_4 9650029242287828579ull
#define P64_5 2870177450012600261ull

static uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }  /* little-endian host */
static uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint16_t rd16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }
static uint64_t s64(int off) { return rd64(kSecret + off); }
static uint32_t s32(int off) { return rd32(kSecret + off); }

static uint64_t mul_fold64(uint64_t a, uint64_t b) {
    const unsigned __int128 p = (unsigned __int128)a * b;
    return (uint64_t)p ^ (uint64_t)(p >> 64);
}
static uint64_t avalanche_small(uint64_t v) {
    v ^= v >> 33; v *= P64_2; v ^= v >> 29; v *= P64_3; v ^= v >> 32;
    return v;
}
static uint64_t avalanche(uint64_t v) {
    v ^= v >> 37; v *= 0x165667919e3779f9ull; v ^= v >> 32;
    return v;
}
static uint64_t rotl64(uint64_t v, int r) { return (v << r) | (v >> (64 - r)); }
static uint64_t rrmxmx(uint64_t v, uint64_t len) {
    v ^= rotl64(v, 49) ^ rotl64(v, 24);
    v *= 0x9fb21c651e98df25ull;
    v ^= (v >> 35) + len;
    v *= 0x9fb21c651e98df25ull;
    v ^= v >> 28;
    return v;
}
static uint64_t mix16(const uint8_t* d, int doff, int soff) {
    return mul_fold64(rd64(d + doff) ^ s64(soff), rd64(d + doff + 8) ^ s64(soff + 8));
}

static uint64_t hash_small(const uint8_t* d, size_t len) {
    uint64_t acc;
    if (len > 8) {
        const uint64_t lo = rd64(d) ^ (s64(24) ^ s64(32));
        const uint64_t hi = rd64(d + len - 8) ^ (s64(40) ^ s64(48));
        return avalanche((uint64_t)len + __builtin_bswap64(lo) + hi + mul_fold64(lo, hi));
    } else if (len > 3) {
        const uint64_t in = (uint64_t)rd32(d + len - 4) + ((uint64_t)rd32(d) << 32);
        return rrmxmx(in ^ (s64(8) ^ s64(16)), (uint64_t)len);
    } else if (len == 3) {
        acc = ((uint64_t)rd16(d) << 16) + (uint64_t)d[2] + (3u << 8);
    } else if (len == 2) {
        acc = (uint64_t)rd16(d) * ((1u << 24) + 1) >> 8;
        acc += 2u << 8;
    } else if (len == 1) {
        acc = (uint64_t)d[0] * ((1u << 24) + (1u << 16) + 1) + (1u << 8);
    } else {
        return 0x2d06800538d394c2ull;
    }
    acc ^= (uint64_t)(s32(0) ^ s32(4));
    return avalanche_small(acc);
}

static uint64_t hash_medium(const uint8_t* d, size_t len) {
    const int L = (int)len;
    uint64_t acc = (uint64_t)len * P64_1;
    if (L > 32) {
        if (L > 64) {
            if (L > 96) {
                acc += mix16(d, 48, 96);
                acc += mix16(d, L - 64, 112);
            }
            acc += mix16(d, 32, 64);
            acc += mix16(d, L - 48, 80);
        }
        acc += mix16(d, 16, 32);
        acc += mix16(d, L - 32, 48);
    }
    acc += mix16(d, 0, 0);
    acc += mix16(d, L - 16, 16);
    return avalanche(acc);
}

static uint64_t hash_large(const uint8_t* d, size_t len) {
    const int L = (int)len;
    uint64_t acc = (uint64_t)len * P64_1;
    for (int off = 0; off < 128; off += 16) acc += mix16(d, off, off);
    acc = avalanche(acc);
    for (int off = 128, top = L & ~15; off < top; off += 16) acc += mix16(d, off, off - 125);
    acc += mix16(d, L - 16, 119);
    return avalanche(acc);
}

static void accumulate_stripe(uint64_t acc[8], const uint8_t* d, const uint8_t* s) {
    for (int j = 0; j < 8; j += 2) {
        const uint64_t in0 = rd64(d + 8 * j), in1 = rd64(d + 8 * j + 8);
        const uint64_t k0 = in0 ^ rd64(s + 8 * j), k1 = in1 ^ rd64(s + 8 * j + 8);
        acc[j] += (uint64_t)(uint32_t)k0 * (k0 >> 32) + in1;
        acc[j + 1] += in0 + (uint64_t)(uint32_t)k1 * (k1 >> 32);
    }
}

static void scramble(uint64_t acc[8]) {
    for (int j = 0; j < 8; ++j) {
        acc[j] ^= acc[j] >> 47;
        acc[j] ^= s64(128 + j * 8);
        acc[j] *= P32_1;
    }
}

static uint64_t hash_long(const uint8_t* d, size_t len) {
    uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    const uint8_t* p = d;
    size_t remaining = len;
    while (remaining > 1024) {
        for (int st = 0; st < 16; ++st) {
            accumulate_stripe(acc, p, kSecret + 8 * st);
            p += 64;
            remaining -= 64;
        }
        scramble(acc);
    }
    if (remaining) {
        const size_t stripes = (remaining - 1) / 64;
        for (size_t st = 0; st < stripes; ++st) {
            accumulate_stripe(acc, p, kSecret + 8 * st);
            p += 64;
            remaining -= 64;
        }
        if (remaining) accumulate_stripe(acc, d + len - 64, kSecret + 121);
    }
    uint64_t r = (uint64_t)len * P64_1;
    r += mul_fold64(acc[0] ^ s64(11), acc[1] ^ s64(19));
    r += mul_fold64(acc[2] ^ s64(27), acc[3] ^ s64(35));
    r += mul_fold64(acc[4] ^ s64(43), acc[5] ^ s64(51));
    r += mul_fold64(acc[6] ^ s64(59), acc[7] ^ s64(67));
    return avalanche(r);
}

/* hashcode.GetHashCodeXXH3 (hashcode/hashcode.go:15-17 -> xxh3.go:43-56) */
ORA_API uint64_t ora_xxh3_64(const uint8_t* d, size_t len) {
    if (len <= 16) return hash_small(d, len);
    if (len <= 128) return hash_medium(d, len);
    if (len <= 240) return hash_large(d, len);
    return hash_long(d, len);
}

ORA_API void ora_xxh3_batch(const uint8_t* bytes, const uint64_t* offsets, const uint32_t* lens, uint32_t n,
                            uint64_t* out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = ora_xxh3_64(bytes + offsets[i], lens[i]);
}

/* The 13-byte key of NatFlowHash / NatWanFlowHash (engine/ipv4_engine.go:451-459, :471-479)
 * built from a parsed record the way the forward path builds it (see include/halo_rx.h,
 * HALO_FLOW_*), then hashed. */
ORA_API uint64_t ora_flow_key_hash(const halo_rx_result_t* r, uint32_t kind, uint32_t nat_type) {
    uint32_t remote_ip, local_ip;
    uint16_t remote_port, local_port;
    if (kind == HALO_FLOW_NAT_WAN) {  /* NatGetFlowByWan(src, sport, dst, dport, proto) */
        remote_ip = r->src_ip; remote_port = r->sport; local_ip = r->dst_ip; local_port = r->dport;
    } else {                          /* NatGetFlowByHash(dst, dport, src, sport, proto) */
        remote_ip = r->dst_ip; remote_port = r->dport; local_ip = r->src_ip; local_port = r->sport;
    }
    uint32_t rip = 0;
    uint16_t rport = 0;
    if (nat_type == HALO_NAT_SYMMETRIC) { rip = remote_ip; rport = remote_port; }
    if (r->ip_proto == 1) rport = 0;
    uint8_t key[13];
    memcpy(key + 0, &rip, 4);        /* binary.LittleEndian.PutUint32 on a little-endian host */
    memcpy(key + 4, &rport, 2);
    memcpy(key + 6, &local_ip, 4);
    memcpy(key + 10, &local_port, 2);
    key[12] = r->ip_proto;
    return ora_xxh3_64(key, 13);
}

/* + the bucket of hashmap.HashMap.Get / Set (hashmap/hashmap.go:64, :84): hash % bucket count */
ORA_API void ora_flow_hash_batch(const halo_rx_result_t* recs, uint32_t n, uint32_t kind, uint32_t nat_type,
                                 uint64_t* out, uint32_t bucket_count, uint32_t* bucket) {
    for (uint32_t i = 0; i < n; ++i) {
        out[i] = ora_flow_key_hash(&recs[i], kind, nat_type);
        if (bucket && bucket_count) bucket[i] = (uint32_t)(out[i] % bucket_count);
    }
}
