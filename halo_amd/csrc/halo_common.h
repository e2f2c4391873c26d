// halo_common.h — constants and helpers shared by the HIP kernels and the host side of
// libhalo_rx.so. Device code is written for gfx950 (CDNA4) only.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <vector>

#include "halo_limits.h"
#include "halo_rx.h"
#include "host_logic.h"

namespace halo {

// Kernel parameter block (passed by value; one per launch).
struct RxParams {
    const uint8_t* bytes;
    const uint32_t* offsets_dw;  // ragged layout (LAYOUT 0)
    const uint16_t* lens;        // per-frame lengths (LAYOUT 0, 1)
    uint64_t stride;             // strided layouts (LAYOUT 1, 2)
    uint32_t len;                // uniform length (LAYOUT 2)
    uint32_t n;
    uint32_t flags;
    uint32_t mac_lo;  // own MAC bytes 0..3, little-endian packed
    uint32_t mac_hi;  // own MAC bytes 4..5
    uint32_t own_ip;  // IpAddrToU(NetIf.IpAddr)
    halo_rx_result_t* out;
    uint32_t* hist;      // the device's histogram tree set (hist_trees), or null
    uint32_t* hist_out;  // the caller's counters the last block of the launch adds into
    // fused NAT flow-key hash of every record (halo_rx_parse_flow_batch_device), or null
    uint64_t* flow_hash;
    uint32_t* flow_bucket;
    uint32_t flow_buckets, flow_kind, flow_nat;
    // fused FindRoute of every record's dst (halo_rx_parse_route_batch_device), or null
    const uint32_t* rt_tbl24;
    const uint32_t* rt_tbl8;
    const uint2* rt_lists;
    const uint32_t* rt_ids;
    uint32_t* route_out;
};

// splitmix64 finaliser — the synthetic-traffic generator's only randomness source.
__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t synth_key(uint64_t seed, uint64_t index) {
    return mix64(seed ^ mix64(index));
}
__host__ __device__ inline uint64_t synth_draw(uint64_t key, uint64_t slot) {
    return mix64(key + slot * 0xD6E8FEB86659FD93ull);
}
enum SynthSlot : uint32_t {
    kSlotSize = 1, kSlotProto = 2, kSlotMutate = 3, kSlotMutPos = 4, kSlotMac = 5,
    kSlotIp = 6, kSlotPorts = 7, kSlotSeq = 8, kSlotWin = 9, kSlotPayload = 64
};

int check_device();  // 0 if the current device is gfx950, else HALO_E_*

// Partial status histograms of an rx launch (flush_hist, rx_parse.hip). A tree is kHistSlots
// level-1 slots (one per block modulo kHistSlots) then kHistSlots / kHistFan level-2 slots,
// kHistStride 64-bit words each (arrivals << 40 | count, one per status), zero between launches.
// Trees belong to HSA queues, not to streams: a device's tree set holds kHistTrees trees and a key
// word per tree, and a launch's blocks take the tree whose key is their queue (queue_ptr), claiming
// a free key on the queue's first launch; keys are released only by halo_rx_release, with the
// device drained, so every block of every launch on a queue agrees on its tree. Sharing a tree between launches of one queue is safe because
// every HIP dispatch carries the AQL barrier bit (profiles/r05/queue_probe.log: null, created and
// per-thread streams, graph replays): a packet starts only after every earlier packet of its queue
// has completed, so no two launches are ever inside one tree. hist_trees checks the bit once per
// device with a probe dispatch; without it the keys are poisoned and launches add straight into the
// caller's counters (so do launches beyond kHistTrees queues). Streams that share a queue are
// serialised by those barriers; hipStreamPerThread, graph replays on several streams at once and
// streams of other devices need no host-side key at all.
constexpr uint32_t kHistSlots = 1024, kHistFan = 32, kHistStride = 16;
constexpr uint32_t kHistWords = (kHistSlots + kHistSlots / kHistFan) * kHistStride;  // 64-bit words
// 64 trees (round 6; 16 before): more queues than a process normally has (GPU_MAX_HW_QUEUES = 4
// per device, plus one per CU-masked stream). A launch whose queue finds no free key takes the
// fallback, 9x slower at 1M frames.
constexpr uint32_t kHistTrees = 64, kHistKeyWords = 64;  // keys first (four 128 B lines), then trees
constexpr uint64_t kHistSetBytes = 8ull * (kHistKeyWords + (uint64_t)kHistTrees * kHistWords);
// The tree set of `device`, allocated and zeroed at first use (halo_rx_init does it ahead of any
// capture); nullptr when that fails, or when it is first needed inside a stream capture. Once made,
// a set lives as long as the process: graphs captured with its address stay valid.
uint32_t* hist_trees(int device, hipStream_t capture_probe);
int stream_device(hipStream_t s);  // the device a launch on `s` runs on (-1: unknown)
// Frees every key of the device's set (poisoned keys stay poisoned): queues that no longer exist
// give their trees back. The caller has drained the device, and no launch may run alongside.
int hist_trees_reset_keys(int device);
// Test hook behind halo_rx_debug_hist_keys: op 0 counts the claimed keys; 1 poisons every key; 2
// occupies all keys but `arg` with ids no queue has; 3 = hist_trees_reset_keys.
int hist_keys_debug(int device, int op, uint32_t arg);

// The resident small-poll consumer of a ring attached with HALO_RING_PERSISTENT (ring_rx.hip
// drives it, rx_parse.hip runs it): kSvcGroups workgroups that wait on this control block, in
// pinned host memory, for a request, parse its n frames as the lane kernel would (frames at
// data + 4 * off_dw[i], the host's ReadPacket walk wrote off_dw / lens into pinned memory; 64-frame
// windows dealt round-robin over the groups) and write their records to `out`; each group then
// publishes its done_seq slot. The host never launches per poll.
#ifndef HALO_SVC_GROUPS
#define HALO_SVC_GROUPS 8   // workgroups of the resident consumer (each on its own CU)
#endif
#ifndef HALO_SVC_WAVES
#define HALO_SVC_WAVES 8    // waves per workgroup (64 frames each per pass)
#endif
constexpr uint32_t kSvcGroups = HALO_SVC_GROUPS;
constexpr uint32_t kSvcWaves = HALO_SVC_WAVES;
struct alignas(64) RingServiceCtl {
    // The request: one 64-byte line. The host writes the fields, then `check` (svc_check of the
    // fields), then req_seq with release. Each workgroup reads the whole line with one 16-lane load
    // and takes a request whose req_seq is new and whose check matches (a torn read is re-read).
    uint32_t req_seq;        // host: the request number
    uint32_t n, flags, mac_lo, mac_hi, own_ip;
    uint32_t out_lo, out_hi; // device address of the request's records
    uint32_t stop;           // host: 1 = exit now
    uint32_t check;
    // A poll whose frames all have one length and follow each other in the ring (config 1) is
    // described here instead of by the offset / length arrays: frame i at data + 4 * (uni_off +
    // i * uni_stride), uni_len bytes (0: use the arrays). It arrives with the request, so the
    // consumer skips the arrays' PCIe round trip.
    uint32_t uni_off, uni_stride, uni_len;
    uint32_t pad0[3];
    // Completion: one slot per workgroup, each written by its group after its records are visible
    // (system-scope release)
    uint32_t done_seq[kSvcGroups];
    uint32_t alive[kSvcGroups];   // 1 while the group runs (diagnostics)
    uint64_t t_seen[kSvcGroups];  // real-time counter (100 MHz) when the group took the request
    uint64_t t_done[kSvcGroups];  // ... when it published its records
};
static_assert(offsetof(RingServiceCtl, done_seq) == 64, "request line");
__host__ __device__ inline uint32_t svc_check(uint32_t seq, uint32_t n, uint32_t flags, uint32_t mac_lo, uint32_t mac_hi,
                                              uint32_t own_ip, uint32_t out_lo, uint32_t out_hi, uint32_t uni_off,
                                              uint32_t uni_stride, uint32_t uni_len) {
    const uint32_t w[11] = {seq, n, flags, mac_lo, mac_hi, own_ip, out_lo, out_hi, uni_off, uni_stride, uni_len};
    uint32_t h = 0x811C9DC5u;
    for (int i = 0; i < 11; ++i) h = (h ^ w[i]) * 0x01000193u;
    return h;
}
// Launches the consumer on `s`: it serves requests after `last`, and exits when `stop` is set, when
// another of its workgroups has left (*d_quit, device memory, zeroed before the launch), or after
// idle_us microseconds without a request (the first group to time out sets *d_quit, so the whole
// grid leaves together instead of one group at a time).
int launch_ring_service(RingServiceCtl* d_ctl, const uint8_t* d_data, const uint32_t* d_off,
                        const uint16_t* d_len, uint32_t* d_quit, uint32_t last, uint32_t idle_us, hipStream_t s);

// ---- resident consumers (resident.hip): one RingServiceCtl + its kernel, driven from the host ----
// Used by rings attached with HALO_RING_PERSISTENT and by host contexts with a resident consumer
// (halo_rx_host_ctx_set_resident). The frames of a request live at d_data (+ the u32 dword offsets /
// u16 lengths at d_off / d_len, or the uniform layout carried in the request line).
constexpr uint32_t kSvcMaxFrames = 16384;  // larger requests take a full-grid launch
constexpr uint32_t kSvcIdleUs = 20000;      // the consumer exits after 20 ms without a request
constexpr int kResidentParked = 1;          // resident_request: not served, launch instead
struct Resident;
struct ResidentStats {
    uint64_t requests;  // requests served
    uint64_t launches;  // kernel launches (first use, after idle exits, after parks)
    uint64_t gpu_ns;    // the consumer's own time per request (first group in, last group out), summed
    uint64_t parked;    // requests refused while a device drain had the consumers parked
};
int resident_create(int device, const uint8_t* d_data, const uint32_t* d_off, const uint16_t* d_len,
                    Resident** out);
void resident_destroy(Resident* s);
// Serves n <= kSvcMaxFrames frames into dout (device address). HALO_OK when every group published;
// kResidentParked when a drain is in progress (nothing was requested: the caller launches); HALO_E_HIP
// when the wait passed the timeout — the request is retired first (the consumer is stopped and its
// kernel has ended), so nothing is written to dout after the call returns.
int resident_request(Resident* s, uint32_t n, uint32_t flags, const halo_rx_netif_t* netif, halo_rx_result_t* dout,
                     uint32_t uni_off, uint32_t uni_stride, uint32_t uni_len);
void resident_set_timeout(Resident* s, uint64_t us);  // 0: the default (2 s)
// New frame / offset / length arrays for the next launch of the consumer (the owner reallocated
// them). The caller holds a ParkResidents on the device, so the consumer's kernel has ended.
void resident_set_arrays(Resident* s, const uint8_t* d_data, const uint32_t* d_off, const uint16_t* d_len);
ResidentStats resident_stats(const Resident* s);
// While one lives, the resident consumers of `device` are stopped (their kernels have ended) and new
// requests take the launch path. Every library call that frees device or pinned memory or
// synchronises the whole device runs under one: hipFree / hipHostFree / hipDeviceSynchronize wait
// for every kernel on the device, and a resident kernel ends only 20 ms after its last request —
// never, while another thread keeps polling it.
class ParkResidents {
  public:
    explicit ParkResidents(int device);
    ~ParkResidents();
    ParkResidents(const ParkResidents&) = delete;
    ParkResidents& operator=(const ParkResidents&) = delete;

  private:
    int device_;
};
// The resident consumers of every device this library has launched on, and of `also`, parked for a
// scope: a host free (hipHostFree) waits for kernels on every device, not only the owner's.
struct ParkUsed {
    explicit ParkUsed(int also = -1);
    std::vector<std::unique_ptr<ParkResidents>> parks;
};
// hipDeviceSynchronize on `device` under a ParkResidents.
int drain_device(int device);
// The calling thread's current device (0 if none).
int current_device();

// Live host registrations made through this library (halo_rx_host_register and
// halo_rx_ring_attach(HALO_RING_REGISTER)), over RegMap (host_logic.h): page-aligned whole pages,
// no shared page, checked before any HIP call. Removal waits for every device this library has
// launched on, unregisters, and checks that the runtime no longer maps the range.
uint64_t host_page_size();
int host_reg_add(void* base, uint64_t bytes, HostRegKind kind);  // bytes: a page multiple
int host_reg_remove(void* base, HostRegKind kind);
// The device's address for host range [p, p + bytes) if it lies inside one live registration,
// else nullptr.
void* host_reg_device_view(const void* p, uint64_t bytes);
// The live registration holding host address p: base, size and device address.
bool host_reg_find(const void* p, uintptr_t* base, uint64_t* bytes, uint8_t** dev);

}  // namespace halo
