/*
 * halo_ring_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker and the CPU baseline for
 * SURVEY.md §8f row f1 and BASELINE config 1).
 *
 * A plain-C restatement of halo's SPSC packet ring as its Go side uses it, and of the receive
 * loop that drains it:
 *   RingBuffer layout         mem/ring_buffer.go:18-26      (= cgo/ring_buffer.h:20-55)
 *   ringBufferRecordSize      mem/ring_buffer.go:47-50      u32 length + bytes, 4-byte aligned
 *   RingBufferCreate          mem/ring_buffer.go:93-126     version byte + 0xAA / 0xFF fill
 *   WritePacket               mem/ring_buffer.go:249-295
 *   ReadPacket                mem/ring_buffer.go:298-352
 *   Wire.Rx / EthQueueRxPkt   engine/engine.go:535-545, dpdk/dpdk.go:183-199 (1514 B buffer)
 *   PacketHandle              engine/engine.go:339-351 -> RxEthernet (ora_rx_frame / ora_engine_rx)
 * The reference's own C twin of the ring (cgo/ring_buffer.h) is compiled from where it lies into
 * oracle/_ref/ (oracle/Makefile, target `ref`), and the CPU tests check this restatement against
 * it; this file never includes it.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this code.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/halo_rx.h"

#define ORA_API __attribute__((visibility("default")))

#define RB_HDR 128u /* sizeof(RingBuffer) */
#define RB_REC_HDR 4u
#define RB_ALIGN 4u

void ora_rx_frame(const uint8_t* frame, uint32_t len, uint32_t flags, const halo_rx_netif_t* netif,
                  halo_rx_result_t* r);
int ora_engine_rx(const uint8_t* frame, uint32_t len, uint32_t flags, const halo_rx_netif_t* netif);

typedef struct {
    uint64_t head; /* @0  */
    uint8_t pad0[56];
    uint64_t tail; /* @64 */
    uint64_t size; /* @72 */
    uint64_t mask; /* @80 */
    uint8_t* buffer; /* @88 */
    uint8_t pad1[32];
} ora_ring_t;
_Static_assert(sizeof(ora_ring_t) == RB_HDR, "RingBuffer is 128 bytes");

/* mem/ring_buffer.go:47-50 */
static uint64_t record_size(uint32_t len) {
    return (RB_REC_HDR + (uint64_t)len + RB_ALIGN - 1) & ~(uint64_t)(RB_ALIGN - 1);
}

/* mem/ring_buffer.go:93-126: `size` is the whole block; the data area behind the 128-byte
 * header must be a power of two >= 8. Returns 0 or -1. */
ORA_API int ora_ring_create(void* memory, uint64_t size) {
    if (!memory || size < RB_HDR + 8) return -1;
    size -= RB_HDR;
    if (size < 8 || (size & (size - 1))) return -1;
    ora_ring_t* rb = (ora_ring_t*)memory;
    rb->head = 0;
    rb->tail = 0;
    rb->size = size;
    rb->mask = size - 1;
    rb->buffer = (uint8_t*)memory + RB_HDR;
    uint8_t* b = (uint8_t*)memory;
    b[8] = 1; /* ringBufferLayoutVersion */
    for (int i = 9; i <= 63; ++i) b[i] = 0xAA;
    for (int i = 96; i <= 127; ++i) b[i] = 0xFF;
    return 0;
}

/* A fresh producer (consumer != 0: consumer) cursor, as NewRingBufferProducer / Consumer take
 * it (mem/ring_buffer.go:203-246), mapping offset 0 (same process, as Wire and the DPDK driver). */
ORA_API void ora_ring_cursor(void* memory, int consumer, uint64_t* pos, uint64_t* cached) {
    ora_ring_t* rb = (ora_ring_t*)memory;
    const uint64_t tail = __atomic_load_n(&rb->tail, __ATOMIC_ACQUIRE);
    const uint64_t head = __atomic_load_n(&rb->head, __ATOMIC_ACQUIRE);
    *pos = consumer ? tail : head;
    *cached = consumer ? head : tail;
}

/* WritePacket, mem/ring_buffer.go:249-295. Returns 1 when the record was written. */
ORA_API int ora_ring_write(void* memory, uint64_t* head_io, uint64_t* cached_tail_io, const uint8_t* data,
                           uint32_t len) {
    ora_ring_t* rb = (ora_ring_t*)memory;
    if (!data || len == 0) return 0;
    if ((uint64_t)len > rb->size / 2) return 0;
    const uint64_t head = *head_io;
    uint64_t used = head - *cached_tail_io;
    if (used > rb->size) {
        *cached_tail_io = __atomic_load_n(&rb->tail, __ATOMIC_ACQUIRE);
        used = head - *cached_tail_io;
        if (used > rb->size) return 0;
    }
    const uint64_t total = record_size(len);
    if (rb->size - used < total) {
        *cached_tail_io = __atomic_load_n(&rb->tail, __ATOMIC_ACQUIRE);
        used = head - *cached_tail_io;
        if (used > rb->size || rb->size - used < total) return 0;
    }
    const uint64_t pos = head & rb->mask;
    memcpy(rb->buffer + pos, &len, 4);
    const uint64_t dpos = (pos + RB_REC_HDR) & rb->mask;
    const uint64_t after = rb->size - dpos;
    if (after >= len) {
        memcpy(rb->buffer + dpos, data, len);
    } else {
        memcpy(rb->buffer + dpos, data, after);
        memcpy(rb->buffer, data + after, len - after);
    }
    *head_io = head + total;
    __atomic_store_n(&rb->head, head + total, __ATOMIC_RELEASE);
    return 1;
}

/* ReadPacket, mem/ring_buffer.go:298-352. Returns 1 and the frame in data[0:*len] when a record
 * was consumed; 0 otherwise (*len = the record length when only the capacity was short). */
ORA_API int ora_ring_read(void* memory, uint64_t* tail_io, uint64_t* cached_head_io, uint8_t* data,
                          uint32_t capacity, uint32_t* len) {
    ora_ring_t* rb = (ora_ring_t*)memory;
    *len = 0;
    const uint64_t tail = *tail_io;
    uint64_t used = *cached_head_io - tail;
    if (used > rb->size || used < RB_REC_HDR) {
        *cached_head_io = __atomic_load_n(&rb->head, __ATOMIC_ACQUIRE);
        used = *cached_head_io - tail;
        if (used > rb->size || used < RB_REC_HDR) return 0;
    }
    const uint64_t pos = tail & rb->mask;
    uint32_t plen;
    memcpy(&plen, rb->buffer + pos, 4);
    if (plen == 0 || (uint64_t)plen > rb->size / 2) return 0;
    const uint64_t total = record_size(plen);
    if (used < total) {
        *cached_head_io = __atomic_load_n(&rb->head, __ATOMIC_ACQUIRE);
        used = *cached_head_io - tail;
        if (used > rb->size || used < total) return 0;
    }
    if (capacity < plen) {
        *len = plen;
        return 0;
    }
    const uint64_t dpos = (pos + RB_REC_HDR) & rb->mask;
    const uint64_t after = rb->size - dpos;
    if (after >= plen) {
        memcpy(data, rb->buffer + dpos, plen);
    } else {
        memcpy(data, rb->buffer + dpos, after);
        memcpy(data + after, rb->buffer, plen - after);
    }
    *len = plen;
    *tail_io = tail + total;
    __atomic_store_n(&rb->tail, tail + total, __ATOMIC_RELEASE);
    return 1;
}

/* BASELINE config 1's loop over a ring (engine/engine.go:339-351 with EthRxFunc = Wire.Rx,
 * engine/engine.go:535-545, or dpdk.EthQueueRxPkt): ReadPacket into a `capacity`-byte receive
 * buffer, then RxEthernet on the frame, until ReadPacket returns false or max_frames frames were
 * handled. Per frame i (all outputs optional): the parse record (ora_rx_frame), the engine action
 * (ora_engine_rx), the record's stream position (the tail before the read), and a copy of the
 * frame at frames_out + 4 * frames_out_offsets_dw[i] (frames packed at 4-byte boundaries).
 * Returns the number of frames handled. */
ORA_API uint32_t ora_ring_packet_handle(void* memory, uint64_t* tail_io, uint64_t* cached_head_io,
                                        uint32_t capacity, uint32_t max_frames, uint32_t flags,
                                        const halo_rx_netif_t* netif, halo_rx_result_t* out, uint8_t* actions,
                                        uint64_t* positions, uint8_t* frames_out, uint32_t* frames_out_offsets_dw) {
    uint8_t* buf = (uint8_t*)malloc(capacity ? capacity : 1);
    if (!buf) return 0;
    uint32_t n = 0;
    uint64_t fo = 0;
    while (n < max_frames) {
        const uint64_t before = *tail_io;
        uint32_t len = 0;
        if (!ora_ring_read(memory, tail_io, cached_head_io, buf, capacity, &len)) break;
        if (positions) positions[n] = before;
        if (out) ora_rx_frame(buf, len, flags, netif, &out[n]);
        if (actions) actions[n] = (uint8_t)ora_engine_rx(buf, len, flags, netif);
        if (frames_out) {
            memcpy(frames_out + fo, buf, len);
            frames_out_offsets_dw[n] = (uint32_t)(fo >> 2);
            fo += (len + 3u) & ~3u;
        }
        ++n;
    }
    free(buf);
    return n;
}

/* The walk repeated ReadPacket calls make over `used` bytes of a ring laid out in stream order
 * (the bytes between a consumer's tail and the producer's head, unwrapped), without copying:
 * frame i's bytes start at span + 4 * off_dw[i] and are lens[i] long. Stops where ReadPacket
 * returns false (its checks in its order, mem/ring_buffer.go:309-335) or after max_frames frames
 * when another frame was available. Returns the frame count; *stop is HALO_RING_STOP_*,
 * *end_bytes the bytes consumed (the tail advance), *max_len the longest frame taken. */
ORA_API uint32_t ora_ring_scan(const uint8_t* span, uint64_t used, uint64_t ring_size, uint32_t capacity,
                               uint32_t max_frames, uint32_t* off_dw, uint16_t* lens, uint32_t* stop,
                               uint64_t* end_bytes, uint32_t* max_len) {
    uint64_t pos = 0;
    uint32_t n = 0, ml = 0, why;
    for (;;) {
        const uint64_t rem = used - pos;
        uint32_t plen = 0;
        if (rem < RB_REC_HDR) { why = HALO_RING_STOP_EMPTY; break; }
        memcpy(&plen, span + pos, 4);
        if (plen == 0 || (uint64_t)plen > ring_size / 2) { why = HALO_RING_STOP_BAD_LEN; break; }
        if (rem < record_size(plen)) { why = HALO_RING_STOP_PARTIAL; break; }
        if (plen > capacity) { why = HALO_RING_STOP_CAPACITY; break; }
        if (n == max_frames) { why = HALO_RING_STOP_MAX; break; }
        off_dw[n] = (uint32_t)((pos + RB_REC_HDR) >> 2);
        lens[n] = (uint16_t)plen;
        if (plen > ml) ml = plen;
        ++n;
        pos += record_size(plen);
    }
    *stop = why;
    *end_bytes = pos;
    *max_len = ml;
    return n;
}
