// host_logic.cc — host-only logic of libhalo_rx.so over memory a caller or a ring producer
// controls (see host_logic.h). No HIP in this file: it is compiled into the library by hipcc and
// into an AddressSanitizer + UndefinedBehaviorSanitizer fuzzer by tests/test_sanitize_host.py.
#include "host_logic.h"

#include <string.h>

#include <algorithm>
#include <iterator>

namespace halo {

bool pow2(uint64_t x) { return x >= 8 && (x & (x - 1)) == 0; }

int validate_ring(const uint8_t* mem, int64_t offset, uint64_t* size, uint64_t* tail) {
    if (!mem || (reinterpret_cast<uintptr_t>(mem) & 7u) || !size || !tail) return HALO_E_INVAL;
    if (mem[8] != 1) return HALO_E_INVAL;  // layout version
    for (int i = 9; i <= 63; ++i)
        if (mem[i] != 0xAA) return HALO_E_INVAL;
    for (int i = 96; i <= 127; ++i)
        if (mem[i] != 0xFF) return HALO_E_INVAL;
    uint64_t sz, mask, stored;
    memcpy(&sz, mem + 72, 8);
    memcpy(&mask, mem + 80, 8);
    memcpy(&stored, mem + 88, 8);
    if (!stored || !pow2(sz) || sz > (1ull << 62) || mask != sz - 1) return HALO_E_INVAL;
    const uint64_t t = __atomic_load_n(reinterpret_cast<const uint64_t*>(mem + 64), __ATOMIC_ACQUIRE);
    const uint64_t h = __atomic_load_n(reinterpret_cast<const uint64_t*>(mem), __ATOMIC_ACQUIRE);
    if (h - t > sz) return HALO_E_INVAL;
    // WritePacket / ReadPacket only ever move head and tail by whole 4-byte records; an unaligned
    // cursor would make the reference read or write a length field across the data area's end
    // (mem/ring_buffer.go:276,318). Refused here instead.
    if ((h | t) & 3u) return HALO_E_INVAL;
    // ring_buffer_local_data: the caller's offset must match this mapping
    const uint64_t local = reinterpret_cast<uintptr_t>(mem + kRbHeader);
    if ((int64_t)(local - stored) != offset) return HALO_E_INVAL;
    *size = sz;
    *tail = t;
    return HALO_OK;
}

RingWalk ring_walk(const uint8_t* data, uint64_t size, uint64_t cursor, uint64_t used, uint32_t capacity,
                   uint32_t max_frames, uint32_t* off_dw, uint16_t* lens, uint64_t* positions) {
    RingWalk w;
    const uint64_t mask = size - 1, half = size >> 1;
    uint64_t a = 0;
    for (;;) {
        if (used - a < 4) { w.stop = HALO_RING_STOP_EMPTY; break; }
        const uint64_t p = (cursor + a) & mask;
        uint32_t len = 0;  // the length field; never read past the data area (a 4-aligned field fits)
        if (!(p & 3u)) {
            memcpy(&len, data + p, 4);
        } else {
            for (int k = 3; k >= 0; --k) len = (len << 8) | data[(p + (uint64_t)k) & mask];
        }
        if (len == 0 || len > half) { w.stop = HALO_RING_STOP_BAD_LEN; break; }
        const uint64_t bytes = (4ull + len + 3ull) & ~3ull;
        if (used - a < bytes) { w.stop = HALO_RING_STOP_PARTIAL; break; }
        if (len > capacity) { w.stop = HALO_RING_STOP_CAPACITY; break; }
        if (w.n == max_frames) { w.stop = HALO_RING_STOP_MAX; break; }
        const uint64_t f = (p + 4) & mask;
        if (f + len > size) { w.wraps = true; break; }
        off_dw[w.n] = (uint32_t)(f >> 2);
        lens[w.n] = (uint16_t)len;
        if (positions) positions[w.n] = cursor + a;
        w.max_len = std::max(w.max_len, len);
        w.min_len = std::min(w.min_len, len);
        ++w.n;
        a += bytes;
        // A run of records of this same length (config 1: every frame 64 B). Above, the next
        // record's position waits for this record's length field to load (~2 ns a record, 1k
        // records ~2 us on the small poll's critical path); here it is a + bytes whatever the field
        // holds, and the field is only compared with `len`, so successive fields load in parallel.
        // A same-length record passes the length and capacity checks this one passed; any record
        // that is not a whole same-length record inside the span, or that would wrap, or the
        // max_frames bound, leaves the run and is re-examined above with every ReadPacket check.
        while (w.n < max_frames && used - a >= bytes) {
            const uint64_t q0 = (cursor + a) & mask;
            if (q0 & 3u) break;
            // candidates: whole records inside the span, under max_frames, and ending before the
            // data area's end (so no frame of the run wraps)
            const uint64_t k = std::min<uint64_t>(std::min<uint64_t>(max_frames - w.n, (used - a) / bytes),
                                                  (size - q0) / bytes);
            uint64_t i = 0;
            for (; i < k; ++i) {
                const uint64_t q = q0 + i * bytes;
                uint32_t l2;
                memcpy(&l2, data + q, 4);
                if (l2 != len) break;
                off_dw[w.n + i] = (uint32_t)((q + 4) >> 2);
                lens[w.n + i] = (uint16_t)len;
                if (positions) positions[w.n + i] = cursor + a + i * bytes;
            }
            w.n += (uint32_t)i;
            a += i * bytes;
            if (i < k || k == 0) break;  // a different record, or the data area's end: see above
        }
    }
    w.end_bytes = a;
    return w;
}

// ---- registry ---------------------------------------------------------------------------------
int RegMap::reserve(uintptr_t b, uint64_t bytes, uint64_t page, HostRegKind kind) {
    if (!b || !bytes || !page || (b % page) || (bytes % page) || b + bytes < b) return HALO_E_INVAL;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.lower_bound(b);  // the first registration starting at or after b
    if (it != m_.end() && it->first < b + bytes) return HALO_E_INVAL;
    if (it != m_.begin()) {
        auto pv = std::prev(it);
        if (pv->first + pv->second.bytes > b) return HALO_E_INVAL;
    }
    m_.emplace(b, Entry{bytes, kind, nullptr, kReserved});
    return HALO_OK;
}

void RegMap::commit(uintptr_t b, uint8_t* dev) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.find(b);
    if (it != m_.end()) {
        it->second.dev = dev;
        it->second.state = kLive;
    }
}

void RegMap::cancel(uintptr_t b) {
    std::lock_guard<std::mutex> lk(mu_);
    m_.erase(b);
}

bool RegMap::begin_remove(uintptr_t b, HostRegKind kind) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.find(b);
    if (it == m_.end() || it->second.kind != kind || it->second.state != kLive) return false;
    it->second.state = kRemoving;
    return true;
}

void RegMap::end_remove(uintptr_t b, bool removed) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.find(b);
    if (it == m_.end()) return;
    if (removed)
        m_.erase(it);
    else
        it->second.state = kLive;
}

bool RegMap::find(uintptr_t a, uintptr_t* base, uint64_t* bytes, uint8_t** dev) const {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.upper_bound(a);
    if (it == m_.begin()) return false;
    --it;
    if (it->second.state != kLive || a - it->first >= it->second.bytes) return false;
    *base = it->first;
    *bytes = it->second.bytes;
    *dev = it->second.dev;
    return true;
}

uint8_t* RegMap::view(uintptr_t a, uint64_t bytes) const {
    if (!a || a + bytes < a) return nullptr;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.upper_bound(a);  // the first registration starting after a
    if (it == m_.begin()) return nullptr;
    --it;
    const Entry& e = it->second;
    if (e.state != kLive || !e.dev || a - it->first > e.bytes || bytes > e.bytes - (a - it->first)) return nullptr;
    return e.dev + (a - it->first);
}

uint32_t RegMap::list(void** bases, uint64_t* sizes, uint32_t cap) const {
    std::lock_guard<std::mutex> lk(mu_);
    uint32_t i = 0;
    for (const auto& kv : m_) {
        if (i >= cap) break;
        if (bases) bases[i] = reinterpret_cast<void*>(kv.first);
        if (sizes) sizes[i] = kv.second.bytes;
        ++i;
    }
    return (uint32_t)m_.size();
}

RegMap& registry() {
    static RegMap r;
    return r;
}

// ---- multi-device split and host-path planning ----------------------------------------------------
void shard_bounds(const uint16_t* lens, uint32_t n, uint32_t n_ctx, uint32_t* first) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += lens[i];
    for (uint32_t j = 0; j <= n_ctx; ++j) first[j] = n;
    first[0] = 0;
    uint64_t acc = 0;
    uint32_t k = 1;
    for (uint32_t i = 0; i < n && k < n_ctx; ++i) {
        while (k < n_ctx && acc >= total * k / n_ctx) first[k++] = i;
        acc += lens[i];
    }
    while (k < n_ctx) first[k++] = n;
}

uint32_t plan_direct(const uint64_t* offsets, const uint16_t* lens, uint64_t n, uint64_t next, uint32_t chunk_frames,
                     uint64_t chunk_bytes, uint32_t* h_off, uint16_t* h_len, uint64_t* lo_out, uint64_t* hi_out) {
    const uint64_t lo = offsets[next];
    uint64_t hi = lo;
    uint32_t cnt = 0;
    while (next + cnt < n && cnt < chunk_frames) {
        const uint64_t o = offsets[next + cnt];
        const uint64_t e = o + lens[next + cnt];
        if (o < lo || e < o || ((o - lo) & 3u) || std::max(e, hi) - lo > chunk_bytes) break;
        h_off[cnt] = (uint32_t)((o - lo) >> 2);
        h_len[cnt] = lens[next + cnt];
        hi = std::max(hi, e);
        ++cnt;
    }
    *lo_out = lo;
    *hi_out = hi;
    // worth one DMA only when it covers a whole chunk's worth of frames
    return cnt > 0 && (next + cnt == n || cnt == chunk_frames || hi - lo > chunk_bytes / 2) ? cnt : 0;
}

uint32_t pack_chunk(const uint8_t* bytes, const uint64_t* offsets, const uint16_t* lens, uint64_t n, uint64_t next,
                    uint32_t chunk_frames, uint64_t chunk_bytes, uint32_t cap, uint8_t* staging, uint32_t* h_off,
                    uint16_t* h_len, uint64_t* used_out) {
    uint64_t used = 0;
    uint32_t cnt = 0;
    while (next + cnt < n && cnt < chunk_frames) {
        const uint32_t L = lens[next + cnt];
        const uint64_t need = L <= cap ? ((L + 3u) & ~3u) : 0;  // over-long frames are never read
        if (used + need > chunk_bytes) break;
        if (need) {
            memcpy(staging + used, bytes + offsets[next + cnt], L);
            memset(staging + used + L, 0, need - L);  // the dword tail a kernel load may cover
        }
        h_off[cnt] = (uint32_t)(used >> 2);
        h_len[cnt] = (uint16_t)L;
        used += need;
        ++cnt;
    }
    *used_out = used;
    return cnt;
}

uint64_t pack_need(const uint16_t* lens, uint64_t n, uint32_t cap) {
    uint64_t need = 0;
    for (uint64_t i = 0; i < n; ++i) {  // vectorisable
        const uint32_t L = lens[i];
        need += L <= cap ? ((L + 3u) & ~3u) : 0u;
    }
    return need;
}

bool span_aligned(const uint64_t* offsets, const uint16_t* lens, uint32_t cnt, uint64_t* lo_out, uint64_t* hi_out) {
    uint64_t lo = ~0ull, hi = 0, mis = 0;
    for (uint32_t j = 0; j < cnt; ++j) {  // vectorisable
        const uint64_t e = offsets[j] + lens[j];
        lo = std::min(lo, offsets[j]);
        hi = std::max(hi, e);
        mis |= offsets[j] - offsets[0];
    }
    *lo_out = lo;
    *hi_out = hi;
    return (mis & 3u) == 0;
}

}  // namespace halo

// ---- library identity, errors ------------------------------------------------------------------
extern "C" HALO_API const char* halo_rx_version(void) { return "halo_rx 0.3 (gfx950)"; }

extern "C" HALO_API const char* halo_rx_strerror(int code) {
    switch (code) {
        case HALO_OK: return "ok";
        case HALO_E_INVAL: return "invalid argument";
        case HALO_E_NODEV: return "no HIP device";
        case HALO_E_ARCH: return "device is not gfx950";
        case HALO_E_HIP: return "HIP runtime error";
        case HALO_E_NOMEM: return "out of memory";
        case HALO_E_RANGE: return "batch exceeds addressing range";
        default: return "unknown error";
    }
}

extern "C" HALO_API const char* halo_rx_status_name(int status) {
    static const char* const names[HALO_RX_STATUS_COUNT] = {
        "OK", "ETH_LEN", "ETH_TYPE", "IP_LEN", "IP_VER", "IP_FRAG", "IP_PROTO", "IP_HDR_CKSUM",
        "IP_TOTLEN_UNDERFLOW", "IP_TOTLEN_OVERRUN", "L4_LEN", "ICMP_TYPE", "ICMP_CODE", "L4_CKSUM"};
    return (status >= 0 && status < HALO_RX_STATUS_COUNT) ? names[status] : "UNKNOWN";
}

// ---- engine decision (engine/ethernet_engine.go:13-31, engine/ipv4_engine.go:18-47) -----------
namespace {
uint16_t ethertype_of(const halo_rx_result_t& r) { return r.ethertype; }
uint16_t ethertype_of(const halo_rx_record16_t& r) {
    if (r.status == HALO_RX_ETH_LEN || r.status == HALO_RX_ETH_TYPE) return halo::kEthUnknown;
    switch (r.flags & 0x30u) {
        case HALO_RX_F_ET_ARP: return halo::kEthArp;
        case HALO_RX_F_ET_IPV6: return halo::kEthIpv6;
        case HALO_RX_F_ET_8023: return halo::kEthIeee8023;
        default: return halo::kEthIpv4;
    }
}

uint8_t local_action(uint8_t ip_proto) {
    return ip_proto == halo::kIpIcmp ? HALO_RX_ACT_LOCAL_ICMP
         : ip_proto == halo::kIpUdp  ? HALO_RX_ACT_LOCAL_UDP
                                     : HALO_RX_ACT_LOCAL_TCP;
}

template <typename Rec>
int dispatch(const Rec* results, uint32_t n, const halo_rx_netif_t* netif, uint8_t* actions, uint32_t* action_hist) {
    if (n && (!results || !netif || !actions)) return HALO_E_INVAL;
    for (uint32_t i = 0; i < n; ++i) {
        const Rec& r = results[i];
        const uint16_t ethertype = ethertype_of(r);
        uint8_t a;
        if (r.status == HALO_RX_ETH_LEN || r.status == HALO_RX_ETH_TYPE) {
            a = HALO_RX_ACT_DROP_ETH;                        // ethernet_engine.go:18-21
        } else if (!(r.flags & HALO_RX_F_MAC_MATCH)) {
            a = HALO_RX_ACT_IGNORE_MAC;                      // ethernet_engine.go:22
        } else if (ethertype == halo::kEthArp) {
            a = HALO_RX_ACT_ARP;                             // ethernet_engine.go:24-25
        } else if (ethertype != halo::kEthIpv4) {
            a = HALO_RX_ACT_IGNORE_TYPE;                     // ethernet_engine.go:28
        } else if (r.status >= HALO_RX_IP_LEN && r.status <= HALO_RX_IP_TOTLEN_OVERRUN) {
            a = HALO_RX_ACT_DROP_IP;                         // ipv4_engine.go:19-23
        } else if (r.flags & HALO_RX_F_IP_BCAST) {           // ipv4_engine.go:24-30
            if (r.ip_proto == halo::kIpUdp)
                a = r.status == HALO_RX_OK ? HALO_RX_ACT_BCAST_UDP : HALO_RX_ACT_DROP_BCAST_UDP;
            else
                a = HALO_RX_ACT_IGNORE_BCAST;
        } else if (!(r.flags & HALO_RX_F_DST_IS_OWN) || netif->nat_enable) {
            a = HALO_RX_ACT_FORWARD;                         // ipv4_engine.go:31-37
        } else if (r.status != HALO_RX_OK) {
            a = HALO_RX_ACT_DROP_L4;                         // {udp,tcp,icmp}_engine.go Rx*
        } else {
            a = local_action(r.ip_proto);                    // ipv4_engine.go:38-46
        }
        actions[i] = a;
        if (action_hist) ++action_hist[a];
    }
    return HALO_OK;
}
}  // namespace

extern "C" HALO_API int halo_rx_dispatch(const halo_rx_result_t* results, uint32_t n, const halo_rx_netif_t* netif,
                                         uint8_t* actions, uint32_t* action_hist) {
    return dispatch(results, n, netif, actions, action_hist);
}

extern "C" HALO_API int halo_rx_dispatch_compact(const halo_rx_record16_t* records, uint32_t n,
                                                 const halo_rx_netif_t* netif, uint8_t* actions,
                                                 uint32_t* action_hist) {
    return dispatch(records, n, netif, actions, action_hist);
}

extern "C" HALO_API int halo_rx_dispatch_loopback(const halo_rx_result_t* results, uint32_t n,
                                                  const halo_rx_netif_t* netif, uint8_t* actions,
                                                  uint32_t* action_hist) {
    if (n && (!results || !netif || !actions)) return HALO_E_INVAL;
    for (uint32_t i = 0; i < n; ++i) {
        const halo_rx_result_t& r = results[i];
        uint8_t a;
        if (r.status >= HALO_RX_ETH_LEN && r.status <= HALO_RX_IP_TOTLEN_OVERRUN) {
            a = HALO_RX_ACT_DROP_IP;                         // engine.go:362-365 (no Ethernet layer)
        } else if (!(r.flags & HALO_RX_F_DST_IS_OWN)) {
            a = HALO_RX_ACT_LO_NOT_OWN;                      // engine.go:366-368
        } else if (r.status != HALO_RX_OK) {
            a = HALO_RX_ACT_DROP_L4;                         // Rx{Icmp,Udp,Tcp} log and drop
        } else {
            a = local_action(r.ip_proto);                    // engine.go:369-376
        }
        actions[i] = a;
        if (action_hist) ++action_hist[a];
    }
    return HALO_OK;
}

// ---- ring producer (engine.NewWire / Wire.Tx: RingBufferCreate, WritePacket) -------------------
extern "C" HALO_API int halo_ring_create(void* memory, uint64_t bytes) {
    uint8_t* m = static_cast<uint8_t*>(memory);
    if (!m || (reinterpret_cast<uintptr_t>(m) & 63u) || bytes < halo::kRbHeader + 8) return HALO_E_INVAL;
    const uint64_t size = bytes - halo::kRbHeader;
    if (!halo::pow2(size) || size > (1ull << 62)) return HALO_E_INVAL;
    memset(m, 0, halo::kRbHeader);
    const uint64_t mask = size - 1;
    const uintptr_t buffer = reinterpret_cast<uintptr_t>(m + halo::kRbHeader);
    memcpy(m + 72, &size, 8);
    memcpy(m + 80, &mask, 8);
    memcpy(m + 88, &buffer, 8);
    m[8] = 1;  // layout version
    memset(m + 9, 0xAA, 55);
    memset(m + 96, 0xFF, 32);
    return HALO_OK;
}

extern "C" HALO_API int halo_ring_write_batch(void* memory, const uint8_t* bytes, const uint64_t* offsets,
                                              const uint16_t* lens, uint32_t n, uint8_t* accepted,
                                              uint32_t* written) {
    uint64_t size = 0, tail_unused = 0;
    uint8_t* m = static_cast<uint8_t*>(memory);
    if (!m || (reinterpret_cast<uintptr_t>(m) & 7u)) return HALO_E_INVAL;
    uint64_t stored;
    memcpy(&stored, m + 88, 8);
    int rc = halo::validate_ring(m, (int64_t)(reinterpret_cast<uintptr_t>(m + halo::kRbHeader) - stored), &size,
                                 &tail_unused);
    if (rc) return rc;
    if (n && (!bytes || !offsets || !lens)) return HALO_E_INVAL;
    uint64_t* head_p = reinterpret_cast<uint64_t*>(m);
    const uint64_t* tail_p = reinterpret_cast<const uint64_t*>(m + 64);
    uint8_t* data = m + halo::kRbHeader;
    const uint64_t mask = size - 1;
    uint64_t head = __atomic_load_n(head_p, __ATOMIC_RELAXED);  // this process is the producer
    uint64_t cached_tail = __atomic_load_n(tail_p, __ATOMIC_ACQUIRE);
    uint32_t count = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t len = lens[i];
        bool ok = len != 0 && (uint64_t)len <= size / 2;
        const uint64_t total = (4ull + len + 3ull) & ~3ull;
        if (ok) {  // WritePacket's space check, re-reading the tail only when short
            uint64_t used = head - cached_tail;
            if (used > size || size - used < total) {
                cached_tail = __atomic_load_n(tail_p, __ATOMIC_ACQUIRE);
                used = head - cached_tail;
                ok = used <= size && size - used >= total && !(cached_tail & 3u);
            }
        }
        if (ok) {
            const uint64_t pos = head & mask;  // 4-byte aligned (validate_ring): the field fits before the end
            memcpy(data + pos, &len, 4);
            const uint64_t dpos = (pos + 4) & mask, after = size - dpos;
            const uint8_t* src = bytes + offsets[i];
            if (after >= len) {
                memcpy(data + dpos, src, len);
            } else {
                memcpy(data + dpos, src, after);
                memcpy(data, src + after, len - after);
            }
            head += total;
            __atomic_store_n(head_p, head, __ATOMIC_RELEASE);
            ++count;
        }
        if (accepted) accepted[i] = ok ? 1 : 0;
    }
    if (written) *written = count;
    return HALO_OK;
}
