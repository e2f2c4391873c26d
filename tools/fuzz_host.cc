// fuzz_host.cc — TEST TOOLING: drives the library's host-only logic (halo_amd/csrc/host_logic.cc)
// under AddressSanitizer + UndefinedBehaviorSanitizer with hostile inputs, and checks it against
// the ring restatement pinned to the reference's own C ring (oracle/halo_ring_oracle.c) and against
// naive models. Built and run by tests/test_sanitize_host.py:
//   g++ -fsanitize=address,undefined host_logic.cc fuzz_host.cc + gcc oracle objects
// Usage: fuzz_host <iterations> [seed]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <vector>

#include "host_logic.h"

extern "C" {
int ora_ring_create(void* memory, uint64_t size);
int ora_ring_write(void* memory, uint64_t* head_io, uint64_t* cached_tail_io, const uint8_t* data, uint32_t len);
int ora_ring_read(void* memory, uint64_t* tail_io, uint64_t* cached_head_io, uint8_t* data, uint32_t capacity,
                  uint32_t* len);
}

namespace {
uint64_t g_state = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {  // xorshift64*
    g_state ^= g_state >> 12;
    g_state ^= g_state << 25;
    g_state ^= g_state >> 27;
    return g_state * 0x2545F4914F6CDD1Dull;
}
uint64_t below(uint64_t n) { return n ? rnd() % n : 0; }

int g_fail = 0;
uint64_t g_frames = 0, g_wraps = 0, g_stops[6] = {0, 0, 0, 0, 0, 0}, g_hostile_ok = 0, g_direct = 0, g_packed = 0;
#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);  \
            if (++g_fail > 20) exit(1);                                           \
        }                                                                         \
    } while (0)

uint8_t* aligned_block(uint64_t bytes) {  // 64-byte aligned, exact size for ASan
    void* p = nullptr;
    if (posix_memalign(&p, 64, bytes)) abort();
    memset(p, 0, bytes);
    return static_cast<uint8_t*>(p);
}

uint64_t rd64(const uint8_t* m, int at) {
    uint64_t v;
    memcpy(&v, m + at, 8);
    return v;
}
void wr64(uint8_t* m, int at, uint64_t v) { memcpy(m + at, &v, 8); }

// ---- 1. producer + ReadPacket walk vs the pinned restatement, with hostile headers and records ----
void fuzz_ring(int iters) {
    for (int it = 0; it < iters; ++it) {
        const uint64_t size = 8ull << below(14);  // 8 B .. 64 KiB data areas
        const uint64_t bytes = halo::kRbHeader + size;
        uint8_t* ours = aligned_block(bytes);
        uint8_t* ref = aligned_block(bytes);
        CHECK(halo_ring_create(ours, bytes) == HALO_OK);
        CHECK(ora_ring_create(ref, bytes) == 0);
        uint64_t rhead = 0, rtail_cache = 0, ctail = 0, chead_cache = 0;
        const uint32_t ops = 1 + (uint32_t)below(60);
        for (uint32_t op = 0; op < ops; ++op) {
            const uint64_t kind = below(10);
            if (kind < 5) {  // produce a batch: some empty, some > size/2, some huge
                // a third of the batches repeat one length (the walk's same-length runs)
                const bool same = below(3) == 0;
                const uint32_t n = (uint32_t)below(same ? 40 : 12);
                std::vector<uint16_t> lens(n);
                std::vector<uint64_t> offs(n);
                uint64_t total = 0;
                for (uint32_t k = 0; k < n; ++k) {
                    const uint64_t pick = below(8);
                    lens[k] = (uint16_t)(same && k ? lens[0] : pick == 0 ? 0 : pick == 1 ? below(65536)
                                                     : pick == 2 ? size / 2 + below(8) : below(size / 2 + 1));
                    offs[k] = total;
                    total += lens[k];
                }
                uint8_t* src = static_cast<uint8_t*>(malloc(total ? total : 1));
                for (uint64_t b = 0; b < total; ++b) src[b] = (uint8_t)rnd();
                std::vector<uint8_t> acc(n ? n : 1);
                uint32_t written = 0;
                CHECK(halo_ring_write_batch(ours, src, offs.data(), lens.data(), n, acc.data(), &written) == HALO_OK);
                uint32_t want = 0;
                for (uint32_t k = 0; k < n; ++k) {
                    const int ok = ora_ring_write(ref, &rhead, &rtail_cache, src + offs[k], lens[k]);
                    CHECK(ok == acc[k]);
                    want += ok;
                }
                CHECK(written == want);
                // byte-identical ring memory (but the stored buffer pointer @88: each ring's own address)
                CHECK(memcmp(ours, ref, 88) == 0 && memcmp(ours + 96, ref + 96, bytes - 96) == 0);
                free(src);
            } else if (kind < 9) {  // consume: walk vs repeated ReadPacket
                const uint64_t head = rd64(ours, 0);
                const uint64_t used = std::min<uint64_t>(head - ctail, size) & ~3ull;
                const uint32_t cap = (uint32_t)(below(4) == 0 ? below(64) : 1514 + below(size + 1));
                const uint32_t maxf = (uint32_t)(below(4) == 0 ? below(8) : 0xFFFFFFFFu);
                std::vector<uint32_t> off(size / 8 + 1);
                std::vector<uint16_t> ln(size / 8 + 1);
                std::vector<uint64_t> pos(size / 8 + 1);
                uint64_t t0 = 0;
                CHECK(halo::validate_ring(ours, 0, &t0, &t0) == HALO_OK);
                const halo::RingWalk w = halo::ring_walk(ours + halo::kRbHeader, size, ctail, used, cap,
                                                         std::min<uint32_t>(maxf, (uint32_t)(size / 8 + 1)), off.data(),
                                                         ln.data(), pos.data());
                // the restatement, one ReadPacket at a time, on a copy of the ring memory
                uint8_t* cp = aligned_block(bytes);
                memcpy(cp, ours, bytes);
                wr64(cp, 88, (uint64_t)(uintptr_t)(cp + halo::kRbHeader));
                uint64_t t = ctail, hc = ctail;
                std::vector<uint8_t> buf(cap + 1);
                uint32_t k = 0;
                for (; k < w.n; ++k) {
                    uint32_t len = 0;
                    const uint64_t before = t;
                    const int ok = ora_ring_read(cp, &t, &hc, buf.data(), cap, &len);
                    CHECK(ok == 1 && len == ln[k] && pos[k] == before);
                    if (ok != 1) break;
                    const uint64_t f = ((before & (size - 1)) + 4) & (size - 1);
                    CHECK(memcmp(buf.data(), ours + halo::kRbHeader + f, len) == 0);
                }
                CHECK(w.end_bytes == t - ctail);
                g_frames += w.n;
                g_wraps += w.wraps;
                if (!w.wraps && w.stop < 6) ++g_stops[w.stop];
                if (!w.wraps && w.stop != HALO_RING_STOP_MAX && t - ctail == used) {
                    uint32_t len = 0;  // the walk stopped where ReadPacket stops, or the span ended
                    const int more = ora_ring_read(cp, &t, &hc, buf.data(), cap, &len);
                    if (w.stop == HALO_RING_STOP_CAPACITY) CHECK(!more && len > cap);
                    if (w.stop == HALO_RING_STOP_BAD_LEN) CHECK(!more);
                    if (w.stop == HALO_RING_STOP_EMPTY && head - ctail == used) CHECK(!more);
                }
                free(cp);
                if (below(2)) {  // commit, as halo_rx_ring_commit does
                    ctail += w.end_bytes;
                    wr64(ours, 64, ctail);
                    wr64(ref, 64, ctail);
                    (void)chead_cache;
                }
            } else {  // hostile: a random length field, or a random header byte
                if (below(2)) {
                    const uint64_t p = (ctail + 4 * below(size / 4)) & (size - 1) & ~3ull;
                    const uint32_t v = below(2) ? (uint32_t)rnd() : (uint32_t)(1 + below(size / 2));
                    memcpy(ours + halo::kRbHeader + p, &v, 4);
                    memcpy(ref + halo::kRbHeader + p, &v, 4);
                } else {
                    uint8_t* m = aligned_block(bytes);
                    memcpy(m, ours, bytes);
                    const uint64_t what = below(7);
                    if (what == 0) m[below(128)] ^= (uint8_t)(1u << below(8));
                    if (what == 1) wr64(m, 72, rnd());
                    if (what == 2) wr64(m, 80, rnd());
                    if (what == 3) wr64(m, 88, below(2) ? 0 : rnd());
                    if (what == 4) wr64(m, 0, rd64(m, 64) + below(2 * size) + below(4));
                    if (what == 5) wr64(m, 64, rd64(m, 0) - below(2 * size) - below(4));
                    if (what == 6) m[8] = (uint8_t)rnd();
                    uint64_t sz = 0, tl = 0;
                    const int rc = halo::validate_ring(m, (int64_t)((uintptr_t)(m + halo::kRbHeader) - rd64(m, 88)), &sz, &tl);
                    if (rc == HALO_OK) {
                        ++g_hostile_ok;
                        CHECK(sz == size && (tl & 3u) == 0 && rd64(m, 0) - tl <= sz);
                        std::vector<uint32_t> o2(sz / 8 + 1);
                        std::vector<uint16_t> l2(sz / 8 + 1);
                        halo::ring_walk(m + halo::kRbHeader, sz, tl, (rd64(m, 0) - tl) & ~3ull, 1514, (uint32_t)(sz / 8 + 1),
                                        o2.data(), l2.data(), nullptr);
                    }
                    uint8_t one = 0x45;
                    const uint64_t zero = 0;
                    const uint16_t l1 = 1;
                    uint32_t wn = 0;
                    (void)halo_ring_write_batch(m, &one, &zero, &l1, 1, nullptr, &wn);  // must not crash
                    free(m);
                }
            }
        }
        free(ours);
        free(ref);
    }
}

// ---- 2. dispatch over arbitrary record bytes -------------------------------------------------
void fuzz_dispatch(int iters) {
    for (int it = 0; it < iters; ++it) {
        const uint32_t n = (uint32_t)below(300);
        halo_rx_result_t* r = static_cast<halo_rx_result_t*>(malloc(sizeof(halo_rx_result_t) * (n ? n : 1)));
        halo_rx_record16_t* r16 = static_cast<halo_rx_record16_t*>(malloc(sizeof(halo_rx_record16_t) * (n ? n : 1)));
        uint8_t* rb = reinterpret_cast<uint8_t*>(r);
        for (uint64_t b = 0; b < sizeof(halo_rx_result_t) * n; ++b) rb[b] = (uint8_t)rnd();
        for (uint32_t i = 0; i < n; ++i) {
            r[i].status = (uint8_t)below(below(4) ? HALO_RX_STATUS_COUNT : 256);
            memcpy(&r16[i], rb + 32 * i, 16);
        }
        halo_rx_netif_t nif;
        memset(&nif, 0, sizeof nif);
        nif.nat_enable = (uint32_t)below(2);
        uint8_t* act = static_cast<uint8_t*>(malloc(n ? n : 1));
        uint32_t hist[HALO_RX_ACT_COUNT] = {0};
        CHECK(halo_rx_dispatch(r, n, &nif, act, hist) == HALO_OK);
        uint64_t sum = 0;
        for (uint32_t i = 0; i < n; ++i) CHECK(act[i] < HALO_RX_ACT_COUNT);
        for (int a = 0; a < HALO_RX_ACT_COUNT; ++a) sum += hist[a];
        CHECK(sum == n);
        CHECK(halo_rx_dispatch_compact(r16, n, &nif, act, nullptr) == HALO_OK);
        for (uint32_t i = 0; i < n; ++i) CHECK(act[i] < HALO_RX_ACT_COUNT);
        CHECK(halo_rx_dispatch_loopback(r, n, &nif, act, nullptr) == HALO_OK);
        for (uint32_t i = 0; i < n; ++i) CHECK(act[i] < HALO_RX_ACT_COUNT);
        CHECK(halo_rx_dispatch(nullptr, n ? n : 1, &nif, act, nullptr) == HALO_E_INVAL);
        free(r);
        free(r16);
        free(act);
        CHECK(strlen(halo_rx_status_name((int)rnd())) > 0 && strlen(halo_rx_strerror((int)rnd())) > 0);
    }
}

// ---- 3. the registration registry vs a naive interval model ------------------------------------
void fuzz_registry(int iters) {
    const uint64_t page = 4096;
    for (int it = 0; it < iters; ++it) {
        halo::RegMap map;
        struct M { uint64_t bytes; int kind; int state; uintptr_t dev; };  // state 0 reserved, 1 live, 2 removing
        std::map<uintptr_t, M> model;
        for (int op = 0; op < 200; ++op) {
            const uintptr_t b = (uintptr_t)(1 + below(64)) * page + (below(8) == 0 ? below(page) : 0);
            const uint64_t bytes = (1 + below(6)) * page + (below(8) == 0 ? below(page) : 0);
            const int kind = 1 + (int)below(2);
            const uint64_t what = below(8);
            if (what <= 1) {
                bool free_ = b % page == 0 && bytes % page == 0;
                for (auto& kv : model)
                    if (kv.first < b + bytes && b < kv.first + kv.second.bytes) free_ = false;
                const int rc = map.reserve(b, bytes, page, (halo::HostRegKind)kind);
                CHECK((rc == HALO_OK) == free_);
                if (rc == HALO_OK) model[b] = M{bytes, kind, 0, 0};
            } else if (what == 2 && !model.empty()) {
                auto it2 = model.begin();
                std::advance(it2, below(model.size()));
                if (it2->second.state == 0) {
                    if (below(4)) {
                        const uintptr_t dev = (uintptr_t)(0x100000000ull + it2->first);
                        map.commit(it2->first, reinterpret_cast<uint8_t*>(dev));
                        it2->second.state = 1;
                        it2->second.dev = dev;
                    } else {
                        map.cancel(it2->first);
                        model.erase(it2);
                    }
                }
            } else if (what == 3 && !model.empty()) {
                auto it2 = model.begin();
                std::advance(it2, below(model.size()));
                const bool ok = map.begin_remove(it2->first, (halo::HostRegKind)kind);
                CHECK(ok == (it2->second.state == 1 && it2->second.kind == kind));
                if (ok) {
                    const bool removed = below(3) != 0;
                    map.end_remove(it2->first, removed);
                    if (removed) model.erase(it2);
                }
            } else {
                const uintptr_t a = (uintptr_t)below(70 * page);
                const uint64_t len = below(3 * page);
                uintptr_t fb = 0;
                uint64_t fbytes = 0;
                uint8_t* fdev = nullptr;
                const bool found = map.find(a, &fb, &fbytes, &fdev);
                const uint8_t* v = map.view(a, len);
                bool mf = false;
                const uint8_t* mv = nullptr;
                for (auto& kv : model)
                    if (kv.second.state == 1 && a >= kv.first && a - kv.first < kv.second.bytes) {
                        mf = true;
                        CHECK(found && fb == kv.first && fbytes == kv.second.bytes);
                        if (a && len <= kv.second.bytes - (a - kv.first))
                            mv = reinterpret_cast<const uint8_t*>(kv.second.dev) + (a - kv.first);
                    }
                CHECK(found == mf);
                CHECK(v == mv);
            }
            CHECK(map.list(nullptr, nullptr, 0) == model.size());
        }
    }
}

// ---- 4. the multi-device split and the host path's chunk planning -------------------------------
void fuzz_planning(int iters) {
    for (int it = 0; it < iters; ++it) {
        const uint32_t n = (uint32_t)below(400);
        std::vector<uint16_t> lens(n ? n : 1);
        uint64_t total = 0;
        for (uint32_t i = 0; i < n; ++i) {
            lens[i] = (uint16_t)(below(10) == 0 ? below(65536) : below(1600));
            total += lens[i];
        }
        const uint32_t n_ctx = 1 + (uint32_t)below(9);
        std::vector<uint32_t> first(n_ctx + 1);
        halo::shard_bounds(lens.data(), n, n_ctx, first.data());
        CHECK(first[0] == 0 && first[n_ctx] == n);
        for (uint32_t j = 0; j < n_ctx; ++j) CHECK(first[j] <= first[j + 1]);
        // frames placed in one exact-size buffer: packed, shuffled or gapped
        const uint64_t mode = below(3);
        std::vector<uint64_t> offs(n ? n : 1);
        uint64_t span = 0;
        for (uint32_t i = 0; i < n; ++i) {
            span += mode == 2 ? below(64) : 0;
            if (mode != 0) span = (span + 3) & ~3ull;
            offs[i] = span;
            span += lens[i];
        }
        if (mode == 1)
            for (uint32_t i = 1; i < n; ++i) std::swap(offs[i], offs[below(i + 1)]);
        uint8_t* bytes = static_cast<uint8_t*>(malloc(span ? span : 1));
        for (uint64_t b = 0; b < span; ++b) bytes[b] = (uint8_t)(b * 131u);
        // the length each offset belongs to moves with it when shuffled: rebuild lens by position
        std::vector<uint16_t> plen(n ? n : 1);
        {
            std::vector<std::pair<uint64_t, uint32_t>> order;
            for (uint32_t i = 0; i < n; ++i) order.emplace_back(offs[i], i);
            std::sort(order.begin(), order.end());
            std::vector<uint16_t> sorted_lens(lens.begin(), lens.begin() + n);
            uint64_t cursor = 0;
            for (auto& pr : order) {
                const uint64_t room = (pr.first >= cursor ? span : 0) - pr.first;
                plen[pr.second] = (uint16_t)std::min<uint64_t>(lens[pr.second], room);
                cursor = pr.first;
            }
        }
        const uint32_t chunk_frames = 1 + (uint32_t)below(300);
        const uint64_t chunk_bytes = 64 + below(200000);
        const uint32_t cap = below(2) ? 1514 : 9014;
        std::vector<uint32_t> h_off(chunk_frames);
        std::vector<uint16_t> h_len(chunk_frames);
        uint8_t* staging = static_cast<uint8_t*>(malloc(chunk_bytes));
        uint64_t next = 0;
        while (next < n) {
            uint64_t lo = 0, hi = 0;
            uint32_t cnt = halo::plan_direct(offs.data(), plen.data(), n, next, chunk_frames, chunk_bytes, h_off.data(),
                                             h_len.data(), &lo, &hi);
            if (cnt) {
                ++g_direct;
                CHECK(hi - lo <= chunk_bytes && hi <= span);
                for (uint32_t j = 0; j < cnt; ++j)
                    CHECK(lo + 4ull * h_off[j] == offs[next + j] && h_len[j] == plen[next + j] &&
                          offs[next + j] + plen[next + j] <= hi);
            } else {
                uint64_t used = 0;
                cnt = halo::pack_chunk(bytes, offs.data(), plen.data(), n, next, chunk_frames, chunk_bytes, cap, staging,
                                       h_off.data(), h_len.data(), &used);
                if (!cnt) break;  // a single frame larger than the staging chunk
                ++g_packed;
                CHECK(used <= chunk_bytes);
                CHECK(used == halo::pack_need(plen.data() + next, cnt, cap));  // the pre-check's sum is the packer's
                for (uint32_t j = 0; j < cnt; ++j)
                    if (plen[next + j] <= cap)
                        CHECK(memcmp(staging + 4ull * h_off[j], bytes + offs[next + j], plen[next + j]) == 0);
            }
            uint64_t slo = 0, shi = 0;
            const bool al = halo::span_aligned(offs.data() + next, plen.data() + next, cnt, &slo, &shi);
            CHECK(slo <= shi || cnt == 0);
            (void)al;
            next += cnt;
        }
        free(staging);
        free(bytes);
    }
}
}  // namespace

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    if (argc > 2) g_state = strtoull(argv[2], nullptr, 0) | 1;
    fuzz_ring(iters);
    fuzz_dispatch(iters);
    fuzz_registry(iters / 10 + 1);
    fuzz_planning(iters);
    if (g_fail) {
        fprintf(stderr, "%d checks failed\n", g_fail);
        return 1;
    }
    printf("host logic fuzzed: %d iterations, 0 failures; ring walk: %llu frames vs ReadPacket, %llu wraps, "
           "stops EMPTY %llu BAD_LEN %llu PARTIAL %llu CAPACITY %llu MAX %llu; %llu hostile headers accepted; "
           "chunks: %llu direct, %llu packed\n",
           iters, (unsigned long long)g_frames, (unsigned long long)g_wraps, (unsigned long long)g_stops[0],
           (unsigned long long)g_stops[1], (unsigned long long)g_stops[2], (unsigned long long)g_stops[3],
           (unsigned long long)g_stops[4], (unsigned long long)g_hostile_ok, (unsigned long long)g_direct,
           (unsigned long long)g_packed);
    return 0;
}
