// host_logic.h — the host-only logic of libhalo_rx.so that reads memory a caller or a ring
// producer controls: ring header validation and the producer (WritePacket), the ReadPacket walk
// of a small ring poll, the engine's per-record decision, the registry of host registrations,
// the multi-device split and the host path's chunk planning. No HIP: host_logic.cc is compiled
// into the library by hipcc and, by tests/test_sanitize_host.py, with g++
// -fsanitize=address,undefined into the fuzzer tools/fuzz_host.cc.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <map>
#include <mutex>

#include "halo_limits.h"
#include "halo_rx.h"

namespace halo {

bool pow2(uint64_t x);  // a power of two >= 8 (RingBuffer.size)

// ring_buffer_mapping + ring_buffer_consumer_init (cgo/ring_buffer.h:158-204, :228-246): layout
// version, fill bytes, size / mask, head - tail <= size, the mapping offset. mem: the 128-byte
// header (8-byte aligned). HALO_OK with *size and *tail, else HALO_E_INVAL.
int validate_ring(const uint8_t* mem, int64_t offset, uint64_t* size, uint64_t* tail);

// ReadPacket repeated over [cursor, cursor + used) of a ring's data area (mem/ring_buffer.go:298-352):
// frame k's data offset in dwords and length go to off_dw[k] / lens[k] (and its record position to
// positions[k] when non-null), at most max_frames of them. Stops as ReadPacket stops
// (HALO_RING_STOP_*); `wraps` is set, and the walk stops, at the first frame whose bytes wrap around
// the data area's end (the caller then linearises the span instead).
struct RingWalk {
    uint32_t n = 0, stop = HALO_RING_STOP_EMPTY, max_len = 0, min_len = 0xFFFFFFFFu;
    uint64_t end_bytes = 0;  // record bytes taken: the tail advance
    bool wraps = false;
};
RingWalk ring_walk(const uint8_t* data, uint64_t size, uint64_t cursor, uint64_t used, uint32_t capacity,
                   uint32_t max_frames, uint32_t* off_dw, uint16_t* lens, uint64_t* positions);

// Live host registrations (hipHostRegister) made through the library. A registration pins whole
// pages, so each must start on a page boundary, cover whole pages, and share no page with another.
// Adding is reserve -> (register with the runtime, no lock held) -> commit / cancel; removing is
// begin_remove -> (synchronise, unregister, no lock held) -> end_remove. Lookups see committed
// entries only; a reserved or removing range still blocks overlapping reservations.
enum HostRegKind : int { kRegUser = 1, kRegRing = 2 };
class RegMap {
public:
    int reserve(uintptr_t base, uint64_t bytes, uint64_t page, HostRegKind kind);  // HALO_OK / HALO_E_INVAL
    void commit(uintptr_t base, uint8_t* dev);
    void cancel(uintptr_t base);
    bool begin_remove(uintptr_t base, HostRegKind kind);  // false: no live registration of that kind at base
    void end_remove(uintptr_t base, bool removed);         // removed: forget it; else live again
    // The committed registration holding address a.
    bool find(uintptr_t a, uintptr_t* base, uint64_t* bytes, uint8_t** dev) const;
    // The device address of [a, a + bytes) if it lies inside one committed registration with a
    // device view, else nullptr.
    uint8_t* view(uintptr_t a, uint64_t bytes) const;
    // Every registration (reserved, live or removing), in address order: returns the count and
    // copies up to cap (base, bytes) pairs.
    uint32_t list(void** bases, uint64_t* sizes, uint32_t cap) const;

private:
    enum State : int { kReserved = 0, kLive = 1, kRemoving = 2 };
    struct Entry {
        uint64_t bytes;
        HostRegKind kind;
        uint8_t* dev;
        State state;
    };
    mutable std::mutex mu_;
    std::map<uintptr_t, Entry> m_;
};
RegMap& registry();

// halo_rx_shard_multi's split: contiguous frame ranges balanced by bytes; first[0..n_ctx].
void shard_bounds(const uint16_t* lens, uint32_t n, uint32_t n_ctx, uint32_t* first);

// Host-path chunk planning over the caller's offsets and lengths, from frame `next` of n:
// Direct mode: frames ascending from the first, 4-byte aligned relative to it, spanning at most
// chunk_bytes — one DMA of [lo, hi). Returns the frame count it covers (0: not worth it), with
// staging dword offsets / lengths in h_off / h_len.
uint32_t plan_direct(const uint64_t* offsets, const uint16_t* lens, uint64_t n, uint64_t next, uint32_t chunk_frames,
                     uint64_t chunk_bytes, uint32_t* h_off, uint16_t* h_len, uint64_t* lo, uint64_t* hi);
// Pack mode: frames copied into `staging` at 4-byte aligned offsets; frames longer than `cap` are
// not copied (their verdict needs no byte). Returns the count, *used = staging bytes.
uint32_t pack_chunk(const uint8_t* bytes, const uint64_t* offsets, const uint16_t* lens, uint64_t n, uint64_t next,
                    uint32_t chunk_frames, uint64_t chunk_bytes, uint32_t cap, uint8_t* staging, uint32_t* h_off,
                    uint16_t* h_len, uint64_t* used);
// The staging bytes pack_chunk would use for frames [0, n) (no copy): a batch is checked against
// a staging area before any byte is packed.
uint64_t pack_need(const uint16_t* lens, uint64_t n, uint32_t cap);
// The byte span [*lo, *hi) of cnt frames and whether their offsets agree modulo 4.
bool span_aligned(const uint64_t* offsets, const uint16_t* lens, uint32_t cnt, uint64_t* lo, uint64_t* hi);

}  // namespace halo
