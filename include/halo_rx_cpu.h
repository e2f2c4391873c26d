/*
 * halo_rx_cpu.h — the CPU entry point SURVEY.md §8b lists beside the device ones:
 * halo_rx_parse_batch_cpu, the same per-frame chain as halo_rx_parse_batch_device
 * (protocol/{ethernet,ipv4,udp,tcp,icmp}.go, protocol/utils.go:11-31; see halo_rx.h) run on
 * the calling core over frames in host memory, writing the same halo_rx_result_t records.
 *
 * It lives in its own library, libhalo_rx_cpu.so (halo_amd/csrc/rx_cpu.cc, no HIP), and is
 * NOT a fallback: libhalo_rx.so never calls it, and every halo_rx_parse_* entry point of
 * libhalo_rx.so still fails with HALO_E_NODEV / HALO_E_ARCH without a gfx950 device. A caller
 * chooses it explicitly, for what a GPU round trip cannot serve well: a poll of a few hundred
 * frames or fewer (engine/engine.go:339-353 drains the LoChan every 99 polls; the resident
 * consumer takes ~7 us per call whatever the size, INTEGRATION.md §1a gives the crossover) and
 * the single-frame Parse* calls of an Ipv4PktFwdHook (engine/engine.go:132).
 *
 * Records are bit-identical to the device entry points' for every frame and flags word
 * (tests/test_cpu_entry.py against the C oracle and the golden fixtures, and
 * tests/test_gpu_cpu_entry.py against the GPU kernels).
 */
#ifndef HALO_RX_CPU_H
#define HALO_RX_CPU_H

#include "halo_rx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Frames in host memory: frame i is lens[i] bytes at bytes + offsets[i] (any alignment).
 * `out` receives n halo_rx_result_t records, or n halo_rx_record16_t with HALO_RX_RECORD_COMPACT
 * (the device entry points' compact records, byte for byte); `status_hist`, if not NULL, receives
 * HALO_RX_STATUS_COUNT u32 counters that are INCREMENTED. Flags: HALO_RX_CSUM_ENABLE,
 * HALO_RX_JUMBO_EXT, HALO_RX_L3_START, HALO_RX_RECORD_COMPACT; HALO_RX_UNIFORM_LEN and the variant
 * bits are accepted and ignored (they only pick kernels). Synchronous, on the calling thread;
 * thread-safe (no state). No byte outside [offsets[i], offsets[i] + lens[i]) is read, and no byte
 * of a frame that fails ParseEthFrm's length check (ParseIpv4Pkt's, with HALO_RX_L3_START).
 * n = 0: HALO_OK with null arrays; otherwise a null pointer or unknown flag bit is HALO_E_INVAL.  */
HALO_API int halo_rx_parse_batch_cpu(const uint8_t* bytes, const uint64_t* offsets, const uint16_t* lens,
                                     uint32_t n, uint32_t flags, const halo_rx_netif_t* netif,
                                     halo_rx_result_t* out, uint32_t* status_hist);
HALO_API const char* halo_rx_cpu_version(void);

#ifdef __cplusplus
}
#endif

#endif /* HALO_RX_CPU_H */
