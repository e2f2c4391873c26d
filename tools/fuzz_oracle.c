/* fuzz_oracle.c — TEST TOOL: runs the C oracle (oracle/halo_rx_oracle.c, linked in) over
 * random, mutated and truncated frames under AddressSanitizer / UBSan. Every frame lives in
 * its own exact-size heap block, so any read past a frame's last byte is reported.
 * Build: gcc -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer \
 *        tools/fuzz_oracle.c oracle/halo_rx_oracle.c -o fuzz_oracle -pthread               */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/halo_rx.h"

void ora_rx_frame(const uint8_t* frame, uint32_t len, uint32_t flags, const halo_rx_netif_t* netif,
                  halo_rx_result_t* r);
int ora_engine_rx(const uint8_t* frame, uint32_t len, uint32_t flags, const halo_rx_netif_t* netif);
void ora_synth_frame(uint64_t seed, uint64_t index, uint32_t len, uint8_t kind, const halo_rx_netif_t* netif,
                     uint8_t* f);

static uint64_t rng = 0x48414C4Full;
static uint64_t next(void) {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return rng;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200000;
    halo_rx_netif_t nif;
    memset(&nif, 0, sizeof nif);
    memset(nif.mac, 0xAA, 6);
    nif.ip = 0xC0A86464u;
    unsigned long long ok = 0, st[HALO_RX_STATUS_COUNT] = {0};
    for (int it = 0; it < iters; ++it) {
        const uint32_t kind = next() % 4;
        uint32_t L = 60 + (uint32_t)(next() % 1455);
        if (next() % 8 == 0) L = 9000 + (uint32_t)(next() % 20);
        uint8_t* tmp = (uint8_t*)malloc(L);
        ora_synth_frame(0x1234, (uint64_t)it, L < 60 ? 60 : L, (uint8_t)(kind == 3 ? 0 : kind), &nif, tmp);
        /* mutate: bit flips, header field overwrites, truncation */
        const int flips = (int)(next() % 4);
        for (int k = 0; k < flips; ++k) {
            const uint64_t bit = next() % (8ull * L);
            tmp[bit >> 3] ^= (uint8_t)(1u << (bit & 7));
        }
        if (next() % 4 == 0) { const uint32_t at = 14 + (uint32_t)(next() % 40); if (at < L) tmp[at] = (uint8_t)next(); }
        uint32_t T = L;
        if (next() % 5 == 0) T = (uint32_t)(next() % (L + 1));
        uint8_t* f = (uint8_t*)malloc(T ? T : 1);  /* exact-size block: ASan catches any over-read */
        memcpy(f, tmp, T);
        free(tmp);
        for (uint32_t flags = 0; flags < 4; ++flags) {
            halo_rx_result_t r;
            ora_rx_frame(f, T, flags, &nif, &r);
            (void)ora_engine_rx(f, T, flags, &nif);
            if (r.status >= HALO_RX_STATUS_COUNT) { fprintf(stderr, "bad status\n"); return 2; }
            if (r.payload_off + r.payload_len > T && r.status != HALO_RX_ETH_LEN) {
                fprintf(stderr, "payload slice past frame end\n");
                return 3;
            }
            ++st[r.status];
            ok += r.status == 0;
        }
        free(f);
    }
    printf("fuzzed %d frames x 4 flag settings, statuses:", iters);
    for (int k = 0; k < HALO_RX_STATUS_COUNT; ++k) printf(" %llu", st[k]);
    printf("\n");
    return 0;
}
