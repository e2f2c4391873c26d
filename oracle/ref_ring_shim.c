/*
 * ref_ring_shim.c — TEST INFRASTRUCTURE ONLY.
 *
 * Compiles the REFERENCE's own SPSC packet ring, cgo/ring_buffer.h, from where it lies
 * (oracle/Makefile target `ref` passes -I/root/reference/cgo) into oracle/_ref/libref_ring.so,
 * so the CPU tests can check oracle/halo_ring_oracle.c and the product's ring producer / consumer
 * against the reference's code itself. Exported wrappers only, no logic of their own; nothing
 * of the reference is copied into this repository. Built only where /root/reference exists.
 */
#include <stdlib.h>

#include "ring_buffer.h"

#define REF_API __attribute__((visibility("default")))

REF_API void* ref_ring_create(void* memory, uint64_t size) { return ring_buffer_create(memory, size); }

REF_API void* ref_ring_mapping(void* memory, int64_t* offset) { return ring_buffer_mapping(memory, offset); }

REF_API void* ref_producer_new(void* rb, int64_t offset) {
    ring_buffer_producer_t* p = aligned_alloc(CACHE_LINE_SIZE, sizeof *p);
    if (p && !ring_buffer_producer_init(p, (ring_buffer_t*)rb, offset)) {
        free(p);
        p = NULL;
    }
    return p;
}

REF_API void* ref_consumer_new(void* rb, int64_t offset) {
    ring_buffer_consumer_t* c = aligned_alloc(CACHE_LINE_SIZE, sizeof *c);
    if (c && !ring_buffer_consumer_init(c, (ring_buffer_t*)rb, offset)) {
        free(c);
        c = NULL;
    }
    return c;
}

REF_API void ref_free(void* p) { free(p); }

REF_API int ref_write(void* producer, const uint8_t* data, uint32_t len) {
    return ring_buffer_producer_write_packet((ring_buffer_producer_t*)producer, data, len);
}

REF_API int ref_read(void* consumer, uint8_t* data, uint32_t capacity, uint32_t* len) {
    return ring_buffer_consumer_read_packet((ring_buffer_consumer_t*)consumer, data, capacity, len);
}
