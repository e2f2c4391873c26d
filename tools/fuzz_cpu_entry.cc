// fuzz_cpu_entry.cc — drives halo_rx_parse_batch_cpu (halo_amd/csrc/rx_cpu.cc, the shipped CPU entry
// point) under -fsanitize=address,undefined (tests/test_sanitize_host.py): the oracle's structured
// fuzz corpus (oracle/halo_fuzz.c: every size class 0..9100 B, header-targeted mutations) with every
// frame copied into a heap block of EXACTLY its length, so any read past a frame's last byte is an
// ASan report, parsed one frame per call and in batches at odd offsets, as Ethernet frames and as
// LoChan packets (the frame minus its first 14 bytes), under flags 0..3, full and compact records;
// every record is compared with the oracle's for the same bytes.
// usage: fuzz_cpu_entry <frames> <seed>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "halo_rx.h"
#include "halo_rx_cpu.h"

extern "C" {
uint64_t ora_fuzz_layout(uint64_t seed, uint32_t n, uint16_t* lens, uint32_t* offsets_dw);
void ora_fuzz_fill(uint64_t seed, uint32_t n, const uint16_t* lens, const uint32_t* offsets_dw,
                   const halo_rx_netif_t* netif, uint8_t* bytes);
int ora_rx_batch(const uint8_t* bytes, const uint32_t* offsets_dw, const uint16_t* lens, uint64_t stride, uint32_t len,
                 uint32_t n, uint32_t flags, const halo_rx_netif_t* netif, halo_rx_result_t* out, uint32_t* hist,
                 int threads);
}

static int fail(const char* what, uint32_t i, uint32_t flags) {
    fprintf(stderr, "MISMATCH %s frame %u flags %u\n", what, i, flags);
    return 1;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 0) : 20000;
    const uint64_t seed = argc > 2 ? strtoull(argv[2], nullptr, 0) : 0x5EED;
    halo_rx_netif_t ni;
    memset(&ni, 0, sizeof ni);
    memset(ni.mac, 0xAA, 6);
    ni.ip = 0xC0A86464u;
    std::vector<uint16_t> lens(n);
    std::vector<uint32_t> off(n);
    const uint64_t dw = ora_fuzz_layout(seed, n, lens.data(), off.data());
    std::vector<uint8_t> corpus(4 * dw + 64);
    ora_fuzz_fill(seed, n, lens.data(), off.data(), &ni, corpus.data());
    // LoChan packets: frame bytes [14, L) repacked 4-byte aligned (empty below 14 B)
    std::vector<uint16_t> plens(n);
    std::vector<uint32_t> poff(n);
    std::vector<uint8_t> packets(corpus.size());
    uint64_t at = 0;
    for (uint32_t i = 0; i < n; ++i) {
        plens[i] = lens[i] > 14 ? (uint16_t)(lens[i] - 14) : 0;
        poff[i] = (uint32_t)(at >> 2);
        memcpy(packets.data() + at, corpus.data() + 4ull * off[i] + 14, plens[i]);
        at += (plens[i] + 3u) & ~3u;
    }
    uint64_t checked = 0, counts[HALO_RX_STATUS_COUNT] = {};
    for (int l3 = 0; l3 < 2; ++l3) {
        const uint8_t* src = l3 ? packets.data() : corpus.data();
        const uint16_t* ln = l3 ? plens.data() : lens.data();
        const uint32_t* of = l3 ? poff.data() : off.data();
        // every frame in its own exact-size block (a 0-byte frame gets a 1-byte block no one may read)
        std::vector<uint8_t*> blocks(n);
        for (uint32_t i = 0; i < n; ++i) {
            blocks[i] = (uint8_t*)malloc(ln[i] ? ln[i] : 1);
            memcpy(blocks[i], src + 4ull * of[i], ln[i]);
        }
        for (uint32_t flags = 0; flags < 4; ++flags) {
            const uint32_t f = flags | (l3 ? HALO_RX_L3_START : 0u);
            std::vector<halo_rx_result_t> want(n), got(n);
            std::vector<uint32_t> hw(HALO_RX_STATUS_COUNT), hg(HALO_RX_STATUS_COUNT);
            if (ora_rx_batch(src, of, ln, 0, 0, n, f, &ni, want.data(), hw.data(), 4) != 0) return 2;
            // one frame per call, each from its own exact-size block
            for (uint32_t i = 0; i < n; ++i) {
                const uint64_t zero = 0;
                if (halo_rx_parse_batch_cpu(blocks[i], &zero, &ln[i], 1, f, &ni, &got[i], hg.data()) != HALO_OK)
                    return 3;
                if (memcmp(&got[i], &want[i], sizeof got[i]) != 0) return fail(l3 ? "single L3" : "single", i, flags);
                ++counts[got[i].status];
            }
            if (hg != hw) return fail("histogram", 0, flags);
            // compact records from the same exact-size blocks: the packing of the full ones
            for (uint32_t i = 0; i < n; ++i) {
                const uint64_t zero = 0;
                halo_rx_record16_t c;
                if (halo_rx_parse_batch_cpu(blocks[i], &zero, &ln[i], 1, f | HALO_RX_RECORD_COMPACT, &ni,
                                            reinterpret_cast<halo_rx_result_t*>(&c), nullptr) != HALO_OK)
                    return 5;
                const halo_rx_result_t& w = want[i];
                const uint8_t et = w.ethertype == 0x0806 ? HALO_RX_F_ET_ARP : w.ethertype == 0x86DD ? HALO_RX_F_ET_IPV6
                                 : w.ethertype == 0x05DC ? HALO_RX_F_ET_8023 : HALO_RX_F_ET_IPV4;
                if (c.status != w.status || c.flags != (uint8_t)(w.flags | et) || c.ip_proto != w.ip_proto ||
                    c.l4_aux != w.l4_aux || c.src_ip != w.src_ip || c.dst_ip != w.dst_ip || c.sport != w.sport ||
                    c.dport != w.dport)
                    return fail(l3 ? "compact L3" : "compact", i, flags);
            }
            // batches of 1..97 frames repacked back to back at an odd base (no alignment at all)
            uint32_t i = 0;
            while (i < n) {
                const uint32_t k = 1 + (uint32_t)((i * 2654435761u + flags) % 97u);
                const uint32_t m = k < n - i ? k : n - i;
                uint64_t bytes = 0;
                for (uint32_t j = 0; j < m; ++j) bytes += ln[i + j];
                uint8_t* blk = (uint8_t*)malloc(bytes + 1);
                std::vector<uint64_t> bo(m);
                uint64_t p = 1;  // odd base; the block ends exactly at the last frame's last byte
                for (uint32_t j = 0; j < m; ++j) {
                    bo[j] = p;
                    memcpy(blk + p, blocks[i + j], ln[i + j]);
                    p += ln[i + j];
                }
                std::vector<halo_rx_result_t> r(m);
                if (halo_rx_parse_batch_cpu(blk, bo.data(), ln + i, m, f, &ni, r.data(), nullptr) != HALO_OK) return 4;
                for (uint32_t j = 0; j < m; ++j)
                    if (memcmp(&r[j], &want[i + j], sizeof r[j]) != 0) return fail(l3 ? "batch L3" : "batch", i + j, flags);
                free(blk);
                i += m;
                checked += m;
            }
        }
        for (uint32_t i = 0; i < n; ++i) free(blocks[i]);
    }
    printf("cpu entry: %llu records checked against the oracle; statuses", (unsigned long long)(checked * 2));
    for (int s = 0; s < HALO_RX_STATUS_COUNT; ++s) printf(" %d:%llu", s, (unsigned long long)counts[s]);
    printf("\n");
    return 0;
}
