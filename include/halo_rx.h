/*
 * halo_rx.h — C ABI of the MI355X-native receive parse-and-checksum engine.
 *
 * This is the drop-in boundary for halo's software receive path.
 * The reference has no FFI on this path: the parsers are plain Go functions that
 * engine.(*NetIf).PacketHandle calls once per frame. This ABI replaces that per-frame
 * chain with one call per BATCH of frames:
 *
 *   reference (one frame at a time)                       replaced by
 *   -----------------------------------------------------  -------------------------------
 *   protocol.ParseEthFrm        protocol/ethernet.go:29-55 \
 *   protocol.ParseIpv4Pkt       protocol/ipv4.go:48-86      |
 *   protocol.ParseUdpPkt        protocol/udp.go:21-49       |  halo_rx_parse_batch_device()
 *   protocol.ParseTcpPkt        protocol/tcp.go:36-70       |  halo_rx_parse_strided_device()
 *   protocol.ParseIcmpPkt       protocol/icmp.go:33-63      |  (one halo_rx_result_t per frame)
 *   protocol.GetCheckSum        protocol/utils.go:11-31     |
 *   protocol.NatGetSrcDstPort   protocol/ipv4.go:229-246    |
 *   protocol.IpAddrToU          protocol/utils.go:34-44    /
 *   protocol.CheckSumEnable     protocol/utils.go:8         -> HALO_RX_CSUM_ENABLE bit of `flags`
 *   NetIf.RxEthernet filter     engine/ethernet_engine.go:22 -> HALO_RX_F_MAC_MATCH
 *   NetIf.RxIpv4 branch inputs  engine/ipv4_engine.go:24,31  -> HALO_RX_F_IP_BCAST / _DST_IS_OWN
 *   NetIf.PacketHandle loop     engine/engine.go:339-385    -> halo_rx_parse_batch_host() (pinned H2D,
 *                                                              kernel, D2H) + halo_rx_dispatch()
 *
 * Conventions (SURVEY.md §8b "Error convention"):
 *   - Every entry point returns int: 0 (HALO_OK) or a negative HALO_E_* code. A malformed
 *     frame is DATA (its status code in halo_rx_result_t), never a call failure.
 *   - The caller owns every buffer. No globals: `flags` replaces protocol.CheckSumEnable.
 *   - Calls are thread-safe per (device, stream).
 *   - There is no CPU fallback: without a gfx950 device every compute entry point
 *     returns HALO_E_NODEV / HALO_E_ARCH. The CPU entry point SURVEY.md §8b also lists,
 *     halo_rx_parse_batch_cpu, is a separate library a caller picks by name
 *     (include/halo_rx_cpu.h, libhalo_rx_cpu.so); nothing here calls it.
 *
 * Frame layout in device memory (DESIGN.md "Data layout in HBM"):
 *   - ragged:  frame i starts at bytes + 4*offsets_dw[i] (4-byte aligned starts, as the
 *              reference's ring records are: mem/ring_buffer.go:47-50) and is lens[i] bytes
 *              long. u32 dword offsets address 16 GiB per call.
 *   - strided: frame i starts at bytes + i*stride (stride a multiple of 4), length
 *              lens[i] or, when lens == NULL, the uniform length `len`.
 *   Read contract: no kernel reads a 4 KB page that holds no byte of a frame of the call, so the
 *   frames may sit in several allocations (or around unmapped holes) addressed from one base.
 *   The per-frame kernels never read past the 4-byte word holding a frame's last byte; the
 *   byte-stream kernel (HALO_RX_VARIANT_STREAM) reads whole 16-byte-aligned blocks between a
 *   window's (64 consecutive frames') lowest and highest frame bytes only when every page of
 *   that range holds a frame byte, and otherwise sums that window frame by frame. Bytes between
 *   frames that it does read never enter a record.
 */
#ifndef HALO_RX_H
#define HALO_RX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define HALO_API __attribute__((visibility("default")))
#else
#define HALO_API
#endif

/* ---- return codes ------------------------------------------------------------------ */
#define HALO_OK 0
#define HALO_E_INVAL (-1)   /* bad argument (null pointer, bad stride/flags)              */
#define HALO_E_NODEV (-2)   /* no HIP device / device index out of range                  */
#define HALO_E_ARCH (-3)    /* device is not gfx950 (MI355X)                              */
#define HALO_E_HIP (-4)     /* a HIP runtime call or kernel launch failed                 */
#define HALO_E_NOMEM (-5)   /* device or pinned host allocation failed                    */
#define HALO_E_RANGE (-6)   /* batch too large for the addressing mode                    */

/* ---- flags (replaces the protocol.CheckSumEnable package global, protocol/utils.go:8) - */
#define HALO_RX_CSUM_ENABLE 0x1u /* verify IPv4 header + UDP/TCP checksums (ICMP: always)  */
#define HALO_RX_JUMBO_EXT 0x2u   /* build-defined extension: lift the 1514/1500/1480 caps   */
                                 /* to 9014/9000/8980 (MTU 9000); arithmetic unchanged      */
#define HALO_RX_RECORD_COMPACT 0x4u /* write halo_rx_record16_t (16 B) instead of            */
                                    /* halo_rx_result_t (32 B); device entry points and      */
                                    /* halo_rx_parse_batch_cpu (include/halo_rx_cpu.h) only  */
#define HALO_RX_UNIFORM_LEN 0x8u    /* ragged batch whose frames all have length max_len_hint */
                                    /* (a speed hint: picks the uniform-length kernel table)  */
/* Every buffer starts at its IPv4 header: the packets of a NetIf's LoChan, which
 * PacketHandle drains every 99 polls through ParseIpv4Pkt -> own-address filter -> local
 * Rx{Icmp,Udp,Tcp} (engine/engine.go:353-381; fed by TxIpv4's loopback copy,
 * engine/ipv4_engine.go:72-79). The record is the one of the Ethernet chain minus its
 * Ethernet layer: ParseIpv4Pkt's own length check (len<20 || len>1500, ipv4.go:49) is the
 * first check and can fail (HALO_RX_IP_LEN); ethertype is 0x0800 (the channel carries IPv4
 * only); MAC_MATCH is never set; payload_off is in packet coordinates (IPv4 payload at 20,
 * UDP/ICMP payload at 28, TCP at 20 + headerLen) and 0/0 when ParseIpv4Pkt fails;
 * NatGetSrcDstPort's ports are 0 for packets shorter than 26 B (ipv4.go:230). Map the records
 * to the drain's decisions with halo_rx_dispatch_loopback. Ragged device and host entry
 * points only (halo_rx_parse_batch_device / _host); not with the fused passes or strided
 * layouts (HALO_E_INVAL).                                                                   */
#define HALO_RX_L3_START 0x10u
/* Per-call kernel variant (tuning and tests; results are identical for every value, only speed
 * changes): flags |= HALO_RX_VARIANT_x << HALO_RX_VARIANT_SHIFT. AUTO picks from max_len_hint /
 * the uniform length; LANE = one lane per frame; G4/G8/G16 = that many lanes per frame; MIX =
 * the size-class kernel (each wave sorts 256 frames by size and runs lane-per-frame, 4-, 8- and
 * 16-lane passes); STREAM = the byte-stream kernel (one frame header per lane, every L4
 * segment summed from one coalesced pass over the window's bytes). Device parse entry points
 * only.                                                                                     */
#define HALO_RX_VARIANT_SHIFT 8
#define HALO_RX_VARIANT_MASK 0x700u
#define HALO_RX_VARIANT_AUTO 0u
#define HALO_RX_VARIANT_LANE 1u
#define HALO_RX_VARIANT_G4 2u
#define HALO_RX_VARIANT_G8 3u
#define HALO_RX_VARIANT_G16 4u
#define HALO_RX_VARIANT_MIX 5u
#define HALO_RX_VARIANT_STREAM 6u

/* ---- per-frame status: the FIRST failing check in reference order, 0 = OK ---------- */
typedef enum halo_rx_status {
    HALO_RX_OK = 0,
    HALO_RX_ETH_LEN = 1,              /* len<42 || len>1514        protocol/ethernet.go:31    */
    HALO_RX_ETH_TYPE = 2,             /* EtherType not whitelisted protocol/ethernet.go:39-50 */
    HALO_RX_IP_LEN = 3,               /* len<20 || len>1500        protocol/ipv4.go:49        */
    HALO_RX_IP_VER = 4,               /* pkt[0] != 0x45            protocol/ipv4.go:52        */
    HALO_RX_IP_FRAG = 5,              /* flags/offset not DF|0     protocol/ipv4.go:59        */
    HALO_RX_IP_PROTO = 6,             /* proto not ICMP/TCP/UDP    protocol/ipv4.go:63-72     */
    HALO_RX_IP_HDR_CKSUM = 7,         /* GetCheckSum(hdr) != 0     protocol/ipv4.go:74-78     */
    HALO_RX_IP_TOTLEN_UNDERFLOW = 8,  /* totalLen < 20: Go panics  protocol/ipv4.go:84 (build-defined) */
    HALO_RX_IP_TOTLEN_OVERRUN = 9,    /* totalLen > len(pkt): Go reads stale bytes or panics (build-defined) */
    HALO_RX_L4_LEN = 10,              /* udp.go:22 / tcp.go:37 / icmp.go:34                   */
    HALO_RX_ICMP_TYPE = 11,           /* type not 8/0/11           protocol/icmp.go:38-47     */
    HALO_RX_ICMP_CODE = 12,           /* code != 0                 protocol/icmp.go:49        */
    HALO_RX_L4_CKSUM = 13,            /* udp.go:42 / tcp.go:54 / icmp.go:53                   */
    HALO_RX_STATUS_COUNT = 14
} halo_rx_status_t;

/* ---- per-frame flags: what engine/{ethernet,ipv4}_engine.go branch on ---------------- */
#define HALO_RX_F_MAC_MATCH 0x01u  /* dst MAC == own || broadcast   engine/ethernet_engine.go:22 */
#define HALO_RX_F_IP_BCAST 0x02u   /* dst IP byte 3 == 255           engine/ipv4_engine.go:24     */
#define HALO_RX_F_DST_IS_OWN 0x04u /* dst IP == own IP               engine/ipv4_engine.go:31     */

/* ---- per-frame result record (32 B, written once per frame) ---------------------------
 * Each field is the output of the reference layer that produced it, filled only when that
 * layer returned without error (Go returns zero values / nil slices on error):
 *   ethertype     ParseEthFrm ethProto (0xFFFF on error: ETH_PROTO_UNKNOWN)
 *   ip_proto      ParseIpv4Pkt ipHeadProto (0xFF when not IPv4 or on error: IPH_PROTO_UNKNOWN)
 *   src_ip/dst_ip IpAddrToU(srcAddr/dstAddr)   (0 when ParseIpv4Pkt did not succeed)
 *   ip_total_len  IPv4 totalLen field           (0 when ParseIpv4Pkt did not succeed)
 *   sport/dport   NatGetSrcDstPort(ethPayload)  (ICMP: echo id twice; 0 when IP failed)
 *   l4_aux        TCP flags (tcp.go:50) or ICMP type (icmp.go:38)   (0 unless L4 succeeded)
 *   l4_seq        TCP seqNum, or ICMP id<<16 | seq                   (0 unless L4 succeeded)
 *   l4_ack        TCP ackNum                                         (0 unless L4 succeeded)
 *   payload_off/payload_len  the innermost successfully returned payload slice, in frame
 *                 coordinates: Ethernet frm[14:], IPv4 pkt[20:totalLen], UDP pkt[8:],
 *                 TCP pkt[headerLen:] (headerLen = data-offset nibble used as BYTES,
 *                 protocol/tcp.go:49,68), ICMP pkt[8:]. 0/0 on an Ethernet error.
 * The kernel evaluates the L4 parser selected by ip_proto for EVERY IPv4 frame; which of
 * those verdicts the reference engine would actually have evaluated follows from `flags`
 * (see halo_rx_dispatch).                                                               */
typedef struct halo_rx_result {
    uint8_t status;        /* halo_rx_status_t */
    uint8_t flags;         /* HALO_RX_F_*      */
    uint16_t ethertype;
    uint8_t ip_proto;
    uint8_t l4_aux;
    uint16_t ip_total_len;
    uint32_t src_ip;
    uint32_t dst_ip;
    uint16_t sport;
    uint16_t dport;
    uint16_t payload_off;
    uint16_t payload_len;
    uint32_t l4_seq;
    uint32_t l4_ack;
} halo_rx_result_t;

/* ---- compact per-frame record (16 B; flags |= HALO_RX_RECORD_COMPACT) ------------------
 * The verdict and the extracted 5-tuple only: the fields of halo_rx_result_t named the same,
 * with the EtherType folded into flags bits 4-5 (HALO_RX_F_ET_*; the EtherType is 0xFFFF when
 * status is HALO_RX_ETH_LEN or HALO_RX_ETH_TYPE, whatever those bits hold).                */
#define HALO_RX_F_ET_SHIFT 4
#define HALO_RX_F_ET_IPV4 0x00u    /* 0x0800 */
#define HALO_RX_F_ET_ARP 0x10u     /* 0x0806 */
#define HALO_RX_F_ET_IPV6 0x20u    /* 0x86DD */
#define HALO_RX_F_ET_8023 0x30u    /* 0x05DC */
typedef struct halo_rx_record16 {
    uint8_t status;
    uint8_t flags;     /* HALO_RX_F_* | HALO_RX_F_ET_* */
    uint8_t ip_proto;
    uint8_t l4_aux;
    uint32_t src_ip;
    uint32_t dst_ip;
    uint16_t sport;
    uint16_t dport;
} halo_rx_record16_t;

/* ---- the interface a frame is received on (engine.NetIfConfig, engine/engine.go:65-81) - */
typedef struct halo_rx_netif {
    uint8_t mac[6];  /* NetIf.MacAddr                              */
    uint8_t pad[2];
    uint32_t ip;     /* IpAddrToU(NetIf.IpAddr), host integer      */
    uint32_t nat_enable; /* NetIfConfig.NatEnable (only halo_rx_dispatch reads it) */
} halo_rx_netif_t;

typedef void* halo_stream_t; /* a hipStream_t (NULL = the device's null stream) */

/* ---- device / library -------------------------------------------------------------- */
HALO_API const char* halo_rx_version(void);
/* Selects `device` for the calling thread, checks that it is a gfx950 part and makes the device's
 * status-histogram trees (8.7 MB, zeroed, kept for the life of the process): call it before
 * capturing histogram-on parses in a hipGraph, since a capture cannot allocate (such a call
 * returns HALO_E_NOMEM when the trees were never made). A failure to make the trees does not fail
 * this call: the next histogram-on call outside a capture tries again. Idempotent. */
HALO_API int halo_rx_init(int device);
/* Waits for all work on `device` the way hipDeviceSynchronize does, after stopping this library's
 * resident consumers on it (rings attached with HALO_RING_PERSISTENT, host contexts with
 * halo_rx_host_ctx_set_resident). A caller's own hipDeviceSynchronize / torch.cuda.synchronize()
 * waits for those kernels too, and they end only 20 ms after their last request (never, while
 * another thread keeps them busy); this call does not. The consumers restart on their next request.
 * Like hipDeviceSynchronize on ROCm 7, it does NOT wait for the per-thread stream
 * (hipStreamPerThread) of a host thread that has already exited: synchronise that stream on its
 * own thread before the thread ends. */
HALO_API int halo_rx_device_synchronize(int device);
/* Drains `device` (as halo_rx_device_synchronize) and hands back every status-histogram tree key,
 * so that the HSA queues of streams destroyed since no longer hold trees (64 keys per device; a
 * queue that finds none left counts straight into the caller's counters, exact but ~9x slower at
 * 1M frames). The trees themselves stay: graphs captured with histogram-on parses remain valid and
 * count exactly when replayed after this call. Rings, contexts and route tables stay valid. Must
 * not run while another thread launches parses on `device`. */
HALO_API int halo_rx_release(int device);
/* TESTING ONLY — the histogram tree keys of `device`. op 0: returns how many keys HSA queues have
 * claimed (>= 0); op 1: poisons every key (every histogram-on launch takes the fallback); op 2:
 * occupies all keys but `arg` (<= 64) with ids no queue has; op 3: frees every key as
 * halo_rx_release does. Ops 1-3 drain the device first and must not run alongside parses. */
HALO_API int halo_rx_debug_hist_keys(int device, int op, uint32_t arg);
HALO_API const char* halo_rx_strerror(int code);
HALO_API const char* halo_rx_status_name(int status);

/* ---- device-resident batch parse (the hot path) --------------------------------------
 * All pointers are device pointers. `d_out` receives n records (halo_rx_result_t, or
 * halo_rx_record16_t with HALO_RX_RECORD_COMPACT; 16-byte aligned). `d_status_hist`, if not
 * NULL, receives HALO_RX_STATUS_COUNT u32 counters that are INCREMENTED (the caller
 * zeroes them). `max_len_hint` (a bound on every frame's length; 0 = unknown) selects the
 * lanes-per-frame variant; with HALO_RX_UNIFORM_LEN every frame has exactly that length.
 * Asynchronous on `stream`.                                                              */
HALO_API int halo_rx_parse_batch_device(const uint8_t* d_bytes, const uint32_t* d_offsets_dw,
                                        const uint16_t* d_lens, uint32_t n, uint32_t flags,
                                        const halo_rx_netif_t* netif, uint32_t max_len_hint,
                                        halo_rx_result_t* d_out, uint32_t* d_status_hist,
                                        halo_stream_t stream);

HALO_API int halo_rx_parse_strided_device(const uint8_t* d_bytes, uint64_t stride,
                                          const uint16_t* d_lens, uint32_t len, uint32_t n,
                                          uint32_t flags, const halo_rx_netif_t* netif,
                                          halo_rx_result_t* d_out, uint32_t* d_status_hist,
                                          halo_stream_t stream);

/* ---- several device-resident batches in one launch ------------------------------------
 * The reference's receive loop is an unbounded stream of polls (engine/engine.go:344-351); a
 * caller holding K ragged batches at once (consecutive batches of one queue, or the batches of
 * several NetIf queues) hands them over together. Each batch keeps its own arrays and records,
 * exactly as K halo_rx_parse_batch_device calls on `stream` would produce them; the status
 * histogram (optional) counts all of them. With frames of at most 64 B (max_len_hint 1..64, or
 * HALO_RX_VARIANT_LANE) the K batches run as ONE grid of lane-per-frame waves, so the launch ramp
 * and tail are paid once per K batches instead of once per batch; larger frames take one launch
 * per batch. k <= 32; `batches` is a host array read during the call; batches with n = 0 are
 * skipped. Flags as halo_rx_parse_batch_device (HALO_RX_L3_START included). Asynchronous.   */
typedef struct halo_rx_batch_desc {
    const uint8_t* d_bytes;
    const uint32_t* d_offsets_dw;
    const uint16_t* d_lens;
    halo_rx_result_t* d_out; /* n records (or halo_rx_record16_t), 16-byte aligned */
    uint32_t n;
    uint32_t pad;
} halo_rx_batch_desc_t;    /* 40 B */
HALO_API int halo_rx_parse_batches_device(const halo_rx_batch_desc_t* batches, uint32_t k, uint32_t flags,
                                          const halo_rx_netif_t* netif, uint32_t max_len_hint,
                                          uint32_t* d_status_hist, halo_stream_t stream);

/* ---- host-memory batch parse -----------------------------------
 * Frames in HOST memory (any alignment, ragged byte offsets). Stages them into pinned
 * buffers, copies H2D, runs the kernel and copies results D2H, double-buffered in chunks
 * of `chunk_frames` (0 = default). Synchronous: returns when `out` is filled.           */
typedef struct halo_rx_host_ctx halo_rx_host_ctx_t;
HALO_API int halo_rx_host_ctx_create(int device, uint32_t chunk_frames, uint64_t chunk_bytes,
                                     halo_rx_host_ctx_t** ctx);
HALO_API int halo_rx_host_ctx_destroy(halo_rx_host_ctx_t* ctx);
HALO_API int halo_rx_parse_batch_host(halo_rx_host_ctx_t* ctx, const uint8_t* bytes,
                                      const uint64_t* offsets, const uint16_t* lens, uint32_t n,
                                      uint32_t flags, const halo_rx_netif_t* netif,
                                      halo_rx_result_t* out, uint32_t* status_hist);
/* Frames whose offsets are 4-byte aligned relative to each other and that lie inside one live
 * registration (halo_rx_host_register, or a ring attached with HALO_RING_REGISTER) are parsed
 * in place: the kernel reads them over PCIe, no staging copy (zero-copy mode, the default), and
 * writes the records straight into `out` when `out` is registered as well. Otherwise frames
 * whose offsets are ascending and relatively aligned (a drained ring segment, a packed batch)
 * are sent with one DMA per chunk straight from `bytes`, and other batches are repacked into
 * pinned staging by the CPU. halo_rx_host_ctx_set_zero_copy(ctx, 0) keeps registered batches
 * on the DMA path. Registered memory must stay registered until the call returns.         */
HALO_API int halo_rx_host_ctx_set_zero_copy(halo_rx_host_ctx_t* ctx, int enable);
/* Resident consumer for small batches (the latency path of a batched PacketHandle: EthRxFunc polls
 * gathered into batches of a few frames to a few thousand, engine/engine.go:339-385, and of the
 * single-frame Parse* wrappers an Ipv4PktFwdHook calls, engine/engine.go:132). Batches of at most
 * `max_frames` frames (<= 16384; 0 turns the path off) whose frames fit `max_bytes` of staging
 * (0: min(1516 * max_frames, 64 MiB); at most 64 MiB) are copied into pinned staging this context
 * owns, and a kernel resident on 8 CUs — waiting on a control block in pinned memory — parses them
 * there and writes the records into `out` (directly when `out` lies in a live registration): no
 * launch and no stream synchronisation per call. The kernel leaves 20 ms after its last request and
 * the next call relaunches it; a device drain (halo_rx_host_unregister, a ring detach, a route sync)
 * stops it first and serves calls by launches until the drain is over. Same records as the chunked
 * path. Larger batches take the chunked path. */
HALO_API int halo_rx_host_ctx_set_resident(halo_rx_host_ctx_t* ctx, uint32_t max_frames, uint64_t max_bytes);
/* Bounds the wait for one resident request (default 2 s; 0 restores it). A request that times out
 * is retired before the call returns HALO_E_HIP: the consumer is stopped and its kernel has ended,
 * so nothing is written into the caller's arrays afterwards. (Diagnostics and fault injection.) */
HALO_API int halo_rx_host_ctx_set_service_timeout(halo_rx_host_ctx_t* ctx, uint64_t us);
typedef struct halo_rx_host_stats {
    uint64_t calls;            /* halo_rx_parse_batch_host calls with frames                     */
    uint64_t frames;           /* frames parsed                                                   */
    uint64_t resident_calls;   /* calls served on the resident path                              */
    uint64_t resident_parked;  /* resident calls served by a launch while a device drain ran     */
    uint64_t service_launches; /* resident consumer launches (first use, after idle exits)       */
    uint64_t pack_ns;          /* resident path: host time packing frames into pinned staging    */
    uint64_t wait_ns;          /* resident path: request to completion                            */
    uint64_t service_gpu_ns;   /* resident consumer: GPU time per request (first group in to last
                                  group out), summed                                              */
} halo_rx_host_stats_t;
HALO_API int halo_rx_host_ctx_get_stats(const halo_rx_host_ctx_t* ctx, halo_rx_host_stats_t* out);
/*
 * Registration pins whole pages, so the library enforces: `ptr` page-aligned and `bytes` a
 * multiple of the page size (hugepages, mmap regions; halo_amd._lib.host_array in Python), and
 * no page shared with a live registration (this call's or a ring's) — otherwise HALO_E_INVAL,
 * before any HIP call. Unregister before the memory is freed: `ptr` must be the base of a live
 * registration made here (else HALO_E_INVAL); the call first waits for all work this library
 * queued on every device it used, then unregisters and checks that the runtime no longer maps
 * the range (HALO_E_HIP if it still does: keep the memory allocated then).                 */
HALO_API int halo_rx_host_register(const void* ptr, uint64_t bytes);
HALO_API int halo_rx_host_unregister(const void* ptr);
/* Live registrations (halo_rx_host_register + rings attached with HALO_RING_REGISTER). The
 * second form also copies up to `cap` (base, bytes) pairs, in address order; either array may
 * be NULL. Both return the total count. */
HALO_API uint32_t halo_rx_host_registered_count(void);
HALO_API uint32_t halo_rx_host_registrations(void** bases, uint64_t* bytes, uint32_t cap);

/* Multi-GPU host batch: frames [0, n) are split into n_ctx contiguous index
 * ranges balanced by bytes; ctxs[k] (one host context per device, or several on one device)
 * parses range k on its own host thread with halo_rx_parse_batch_host. Records land in out[i]
 * in frame order; `status_hist` gets the sum. No data crosses devices, no collective.
 * `shard_first` (optional, n_ctx + 1 entries) receives the range boundaries.              */
HALO_API int halo_rx_shard_multi(halo_rx_host_ctx_t* const* ctxs, uint32_t n_ctx, const uint8_t* bytes,
                                 const uint64_t* offsets, const uint16_t* lens, uint32_t n, uint32_t flags,
                                 const halo_rx_netif_t* netif, halo_rx_result_t* out, uint32_t* status_hist,
                                 uint32_t* shard_first);

/* ---- halo's SPSC packet ring as the batch source --------------------
 * The ring is the reference's own shared-memory layout (mem/ring_buffer.go:18-26 =
 * cgo/ring_buffer.h:20-55): a 128-byte header (head @0, layout version 1 @8, tail @64,
 * size @72, mask @80, buffer @88) followed by a power-of-two data area of records
 * `u32 len` + bytes, each padded to 4 bytes (mem/ring_buffer.go:47-50). The DPDK lcore
 * (cgo/dpdk.c:280-307) or engine.Wire.Tx (engine/engine.go:548-553) is the producer.
 *
 * A consumer replaces the per-record ReadPacket (mem/ring_buffer.go:298-352) + EthRxFunc +
 * RxEthernet loop: each poll takes every record between its cursor and the producer's head
 * (at most max_bytes / max_frames) and returns one record per frame, exactly the frames and
 * the order repeated ReadPacket(buf[capacity]) calls would return. The span goes to HBM raw,
 * record boundaries are found on the GPU, the frames are parsed where they lie; the host only
 * reads `head` and, on commit, writes `tail` (release), as ReadPacket does.              */
#define HALO_RING_STOP_EMPTY 0u      /* every record in the span was taken (usedSpace < 4)        */
#define HALO_RING_STOP_BAD_LEN 1u    /* record length 0 or > size/2: ReadPacket returns false     */
#define HALO_RING_STOP_PARTIAL 2u    /* next record not wholly in the span (usedSpace < totalSize;
                                        also when max_bytes cut it)                              */
#define HALO_RING_STOP_CAPACITY 3u   /* record longer than the receive buffer (len(data)):
                                        ReadPacket leaves it, and the tail, in place              */
#define HALO_RING_STOP_MAX 4u        /* max_frames taken, more records available                  */
#define HALO_RING_STOP_BAD_CURSOR 5u /* head - tail > size: ReadPacket returns false              */
#define HALO_RING_REGISTER 0x1u      /* attach: hipHostRegister the ring for full-rate DMA. The ring
                                        must start on a page boundary; the whole pages through the end
                                        of its data area are registered and must not be shared with
                                        another live registration (HALO_E_INVAL; see
                                        halo_rx_host_register)                                      */
#define HALO_RING_PERSISTENT 0x2u    /* attach (with HALO_RING_REGISTER): small polls of up to 16384
                                        frames are served by a resident consumer kernel (8
                                        workgroups, one per CU) that waits on a control block in
                                        pinned memory: a poll writes a request and spins on its
                                        completion, with no kernel launch and no stream
                                        synchronisation. The kernel exits after 20 ms without a
                                        request (the next poll relaunches it) and at detach. Same
                                        records, stops and cursor as the other paths.                */

typedef struct halo_rx_ring_scan {
    uint32_t n_frames;  /* frames taken                                                      */
    uint32_t stop;      /* HALO_RING_STOP_*: why the walk ended                              */
    uint64_t end_bytes; /* ring bytes the frames occupy: the tail advance                    */
    uint32_t max_len;   /* longest frame taken                                               */
    uint32_t pad;
} halo_rx_ring_scan_t;

typedef struct halo_rx_ring halo_rx_ring_t;

/* Attach as the ring's consumer: ring_buffer_mapping + ring_buffer_consumer_init
 * (cgo/ring_buffer.h:158-204, :228-246; mem/ring_buffer.go:150-200, :226-246): layout version,
 * fill bytes, size/mask, head - tail <= size, and `offset` == this mapping's data address minus
 * the stored buffer pointer (0 in the creating process). capacity = the receive buffer's
 * len(data) (0: 1514, dpdk/dpdk.go:139; at most 16376); max_bytes (0: min(size, 256 MiB)) and
 * max_frames (0: max_bytes / 8) bound one poll. The header is validated before any device call. */
HALO_API int halo_rx_ring_attach(int device, void* ring_mem, int64_t offset, uint32_t capacity,
                                 uint64_t max_bytes, uint32_t max_frames, uint32_t attach_flags,
                                 halo_rx_ring_t** out);
/* Synchronises the ring's streams and frees its resources. HALO_E_HIP: the ring memory could not be
 * unregistered (the caller must then keep it allocated). */
HALO_API int halo_rx_ring_detach(halo_rx_ring_t* ring);
/* Parse the next frames (flags: HALO_RX_CSUM_ENABLE | HALO_RX_JUMBO_EXT; full records). They
 * stay in the ring until commit: positions[i] (optional) is frame i's record position in the
 * stream (the tail value before its ReadPacket; the frame's bytes start 4 bytes later, modulo
 * the size). Polls without a commit continue after the previous poll's frames. Synchronous. */
HALO_API int halo_rx_ring_poll(halo_rx_ring_t* ring, uint32_t flags, const halo_rx_netif_t* netif,
                               halo_rx_result_t* out, uint32_t* status_hist, uint64_t* positions,
                               halo_rx_ring_scan_t* info);
/* Small polls (rings attached with HALO_RING_REGISTER; default: spans up to 4 MiB): the host
 * reads the records' length fields as ReadPacket does and ONE rx launch parses the frames in
 * place in the registered ring, writing the records straight into `out` when it is pinned or
 * registered. Same results, stop and cursor as the pipelined path (a poll whose span has a frame
 * wrapping around the data area's end takes the pipelined path). `bytes` = 0 turns the small
 * path off; at most 16 MiB; HALO_E_INVAL for an unregistered ring.                         */
HALO_API int halo_rx_ring_set_small_poll(halo_rx_ring_t* ring, uint64_t bytes);
/* Release everything polled so far to the producer: tail = cursor (store-release). */
HALO_API int halo_rx_ring_commit(halo_rx_ring_t* ring);
/* Counters of a consumer since attach (observability; cheap enough to keep on): where a poll's
 * time goes. Times are host steady-clock ns, except service_gpu_ns (the resident consumer's own
 * real-time counter, from seeing a request to publishing its records). */
typedef struct halo_rx_ring_stats {
    uint64_t polls;            /* halo_rx_ring_poll calls that found records                      */
    uint64_t frames;           /* frames returned                                                  */
    uint64_t small_polls;      /* polls on the small path (one launch, or a service request)      */
    uint64_t service_requests; /* small polls served by the resident consumer (HALO_RING_PERSISTENT) */
    uint64_t service_launches; /* resident consumer launches (first use, after idle exits)       */
    uint64_t walk_ns;          /* small polls: the host's ReadPacket walk of the length fields    */
    uint64_t wait_ns;          /* small polls: launch + synchronisation, or request to completion */
    uint64_t service_gpu_ns;   /* resident consumer: GPU time per request, summed                 */
} halo_rx_ring_stats_t;
HALO_API int halo_rx_ring_get_stats(const halo_rx_ring_t* ring, halo_rx_ring_stats_t* out);
/* HALO_RING_PERSISTENT rings: bounds the wait for one resident request (default 2 s; 0 restores
 * it). A poll whose request times out retires it before returning HALO_E_HIP (the consumer is
 * stopped and its kernel has ended: nothing is written into `out` afterwards) and leaves the cursor
 * where it was, so the next poll parses the same frames. (Diagnostics and fault injection.)    */
HALO_API int halo_rx_ring_set_service_timeout(halo_rx_ring_t* ring, uint64_t us);

/* The record walk alone, device-resident: `used` bytes of ring data in stream order at d_span
 * (4-byte aligned; used a multiple of 4, <= ring_size), ring_size = RingBuffer.size. Writes
 * n = info.n_frames (offset in dwords, length) pairs and *d_info. Workspace: at least
 * halo_rx_ring_scan_workspace(used, capacity) bytes of device memory. Asynchronous.       */
HALO_API uint64_t halo_rx_ring_scan_workspace(uint64_t used, uint32_t capacity);
HALO_API int halo_rx_ring_scan_device(const uint8_t* d_span, uint64_t used, uint64_t ring_size,
                                      uint32_t capacity, uint32_t max_frames, uint32_t* d_offsets_dw,
                                      uint16_t* d_lens, halo_rx_ring_scan_t* d_info, void* d_workspace,
                                      uint64_t workspace_bytes, halo_stream_t stream);

/* The producer side, for rings this process creates (engine.NewWire / Wire.Tx,
 * engine/engine.go:520-553): RingBufferCreate (mem/ring_buffer.go:93-126) over `bytes` of
 * 64-byte-aligned memory (128-byte header + a power-of-two data area), and WritePacket
 * (mem/ring_buffer.go:249-295) for every frame in order — a frame the ring refuses (full,
 * empty, longer than size/2) is dropped, as the DPDK rx lcore drops it (cgo/dpdk.c:288-305).
 * accepted[i] (optional) = 1 if frame i was written; *written = the count. Host only.      */
HALO_API int halo_ring_create(void* memory, uint64_t bytes);
HALO_API int halo_ring_write_batch(void* memory, const uint8_t* bytes, const uint64_t* offsets,
                                   const uint16_t* lens, uint32_t n, uint8_t* accepted, uint32_t* written);

/* ---- forward / transmit direction: in-place header rewrite + checksum fill --------------
 * (SURVEY.md §8f row f2). Frame i's IPv4 packet is pkt = frame[14 : len] — exactly the slice
 * engine.RxIpv4 hands to Ipv4RouteForward (engine/ipv4_engine.go:31-37) — and each frame gets
 * the steps set in ops[i].steps, applied in this order (the order Ipv4RouteForward applies
 * them, engine/ipv4_engine.go:108-269):
 *   HALO_TX_NAT_DST   NatChangeDst(pkt, dst_ip, dst_port)      protocol/ipv4.go:277-302
 *   HALO_TX_TTL       HandleIpv4PktTtl(pkt)                    protocol/ipv4.go:134-145
 *   HALO_TX_NAT_SRC   NatChangeSrc(pkt, src_ip, src_port)      protocol/ipv4.go:249-275
 *   HALO_TX_RECALC    ReCalcIpv4CheckSum + the L4 ReCalc* picked by pkt[9]
 *                                                               protocol/ipv4.go:148-226
 *   HALO_TX_DPDK_FILL eth_tx's software checksum fill (cgo/dpdk.c:333-365: rte_ipv4_cksum and
 *                     rte_ipv4_udptcp_cksum of DPDK 20.11, the reference's pinned DPDK)
 * `flags & HALO_RX_CSUM_ENABLE` is protocol.CheckSumEnable for the Go steps (ReCalcIcmp and
 * DPDK_FILL ignore it, as the reference does). Every length guard of the Go functions is kept:
 * a step whose guard fails leaves the packet as Go would. Result byte per frame: HALO_TX_R_*. */
#define HALO_TX_NAT_DST 0x01u
#define HALO_TX_TTL 0x02u
#define HALO_TX_NAT_SRC 0x04u
#define HALO_TX_RECALC 0x08u
#define HALO_TX_DPDK_FILL 0x10u
#define HALO_TX_R_TTL_ALIVE 0x01u /* HandleIpv4PktTtl returned true                        */
#define HALO_TX_R_SKIPPED 0x02u   /* a step's length guard left the packet (partly) as is   */
#define HALO_TX_R_OVERRUN 0x04u   /* DPDK_FILL: IPv4 totalLen runs past the frame (DPDK would
                                     read stale mbuf bytes); L4 checksum left zero          */
typedef struct halo_tx_op {
    uint8_t steps;     /* HALO_TX_* */
    uint8_t pad;
    uint16_t dst_port; /* NatChangeDst port */
    uint32_t dst_ip;   /* NatChangeDst address, IpAddrToU form */
    uint16_t src_port; /* NatChangeSrc port */
    uint16_t pad2;
    uint32_t src_ip;   /* NatChangeSrc address, IpAddrToU form */
} halo_tx_op_t;       /* 16 B */

/* Device pointers; frames rewritten in place; `d_result` (optional) gets one byte per frame.
 * Ragged layout as halo_rx_parse_batch_device. Asynchronous on `stream`.                */
HALO_API int halo_tx_fixup_batch_device(uint8_t* d_bytes, const uint32_t* d_offsets_dw,
                                        const uint16_t* d_lens, uint32_t n,
                                        const halo_tx_op_t* d_ops, uint32_t flags,
                                        uint32_t max_len_hint, uint8_t* d_result,
                                        halo_stream_t stream);

/* ---- IcmpTtlDeepNat (engine/icmp_engine.go:55-86) -------------------------------------------
 * The forward path calls it on every received Ethernet payload of a NATing interface before its
 * own DNAT (engine/ipv4_engine.go:111-130): when the packet is an ICMP time-exceeded message
 * (ParseIpv4Pkt and ParseIcmpPkt pass, type ICMP_TTL) quoting at least 28 bytes of the original
 * packet, it looks the quoted flow up with NatGetFlowByWan(quoted dst, its dst port, quoted src,
 * its src port, quoted proto) and, when a flow exists, rewrites the quote's source to the flow's
 * LAN host (NatChangeSrc on the quote, with its ReCalc* — TCP's needs 38 quoted bytes) and the
 * message's destination to the LAN host with "port" 0 (NatChangeDst on the untrimmed Ethernet
 * payload: its ICMP checksum covers Ethernet padding). The NAT table stays the caller's: call
 * once with d_nat = NULL to get per frame a quote record — status HALO_RX_OK when the message
 * qualifies, else the failing rx status, HALO_RX_IP_PROTO (not ICMP), HALO_RX_ICMP_TYPE (not
 * ICMP_TTL) or HALO_RX_L4_LEN (quote < 28 B); ip_proto = the quoted protocol; src_ip / sport =
 * the quoted destination and its port, dst_ip / dport = the quoted source and its port, so that
 * halo_flow_hash_device(HALO_FLOW_NAT_WAN) of the records is NatGetFlowByWan's key — then again
 * with the lookups' results in d_nat to rewrite the frames in place. d_applied[i] = 1 when frame
 * i was rewritten (IcmpTtlDeepNat returned true). Frames are the ragged layout of the rx parse;
 * `flags & HALO_RX_CSUM_ENABLE` is protocol.CheckSumEnable. A slow path: one wavefront per frame. */
typedef struct halo_tx_deep_nat {
    uint32_t lan_ip;   /* NatFlow.LanHostIpAddr (IpAddrToU form)       */
    uint16_t lan_port; /* NatFlow.LanHostPort                          */
    uint8_t found;     /* NatGetFlowByWan returned a flow               */
    uint8_t pad;
} halo_tx_deep_nat_t;  /* 8 B */
HALO_API int halo_tx_icmp_deep_nat_batch_device(uint8_t* d_bytes, const uint32_t* d_offsets_dw,
                                                const uint16_t* d_lens, uint32_t n,
                                                const halo_tx_deep_nat_t* d_nat, uint32_t flags,
                                                halo_rx_result_t* d_quote, uint8_t* d_applied,
                                                halo_stream_t stream);

/* ---- transmit direction: batch packet construction (the Build* half) --
 * The locally originated send chain, one frame per descriptor:
 *   NetIf.TxUdp / TxTcp / TxIcmp   engine/{udp,tcp,icmp}_engine.go:24-32 / :29-37 / :26-34
 *    -> protocol.BuildUdpPkt        protocol/udp.go:52-91   (payload <= 1472)
 *       protocol.BuildTcpPkt        protocol/tcp.go:73-123  (payload <= 1460; 20 B header, window 256)
 *       protocol.BuildIcmpPkt       protocol/icmp.go:66-89  (payload <= 1472; code 0)
 *    -> NetIf.TxIpv4                engine/ipv4_engine.go:50-99
 *       protocol.BuildIpv4Pkt       protocol/ipv4.go:89-131 (iphId++ per packet, TTL 0x80, no frag)
 *    -> NetIf.TxEthernet            engine/ethernet_engine.go:34-50
 *       protocol.BuildEthFrm        protocol/ethernet.go:58-82 (src MAC = the NetIf's, pad to 60 B)
 * `flags & HALO_RX_CSUM_ENABLE` is protocol.CheckSumEnable: it gates the IPv4 header, UDP and
 * TCP checksums (0 when off); the ICMP checksum is always filled (icmp.go:84-87). TxIpv4's
 * control-plane decisions (FindRoute, the ARP cache, broadcast) are the caller's: each
 * descriptor carries the destination MAC they produced and its mode:
 *   HALO_TX_BUILD_ETH       the Ethernet frame TxEthernet hands to EthTxFunc
 *   HALO_TX_BUILD_LOOPBACK  the IPv4 packet alone: the copy TxIpv4 puts into the NetIf's LoChan
 *                           when the destination is its own address (engine/ipv4_engine.go:72-79),
 *                           which the L3 loopback parse (HALO_RX_L3_START) consumes.
 * iphId (protocol/ipv4.go:33, process-global in Go) is the device u16 *d_ip_id: BuildIpv4Pkt's
 * `iphId++` runs once per packet that reaches it, in descriptor order, so the k-th successfully
 * built packet of the batch (k = 1, 2, ...) carries id *d_ip_id + k, and *d_ip_id is advanced by
 * the number built. A descriptor whose Build* call returns an error is not built (no iphId step,
 * length 0, result code below). */
#define HALO_TX_BUILD_ETH 0u
#define HALO_TX_BUILD_LOOPBACK 1u
#define HALO_TX_B_OK 0u
#define HALO_TX_B_PAYLOAD_LEN 1u /* "payload len must <= 1472" (udp.go:55, icmp.go:71) / "<= 1460" (tcp.go:78) */
#define HALO_TX_B_PROTO 2u       /* build-defined: proto is not UDP (17), TCP (6) or ICMP (1)          */
#define HALO_TX_B_SLOT 3u        /* build-defined: the frame is longer than out_stride                  */
typedef struct halo_tx_build_desc {
    uint64_t payload_off;  /* byte offset of the L4 payload in d_payload (any alignment)         */
    uint16_t payload_len;
    uint8_t proto;         /* IPH_PROTO_UDP / _TCP / _ICMP (protocol/ipv4.go:27-32)               */
    uint8_t aux;           /* TCP flags; ICMP type                                                */
    uint16_t src_port;     /* UDP/TCP source port; ICMP: the 2 icmpId bytes as a big-endian u16  */
    uint16_t dst_port;     /* UDP/TCP destination port; ICMP: icmpSeq                            */
    uint32_t src_ip;       /* IpAddrToU(srcAddr): the NetIf's address for Tx*                    */
    uint32_t dst_ip;       /* IpAddrToU(dstAddr)                                                 */
    uint32_t seq;          /* TCP seqNum                                                         */
    uint32_t ack;          /* TCP ackNum                                                         */
    uint8_t dst_mac[6];    /* ETH mode: TxIpv4's broadcast / ARP-cache result                    */
    uint8_t mode;          /* HALO_TX_BUILD_*                                                    */
    uint8_t pad;
} halo_tx_build_desc_t;    /* 40 B */

/* Device scratch for n descriptors (bytes, 4-byte aligned; no initialisation needed). One
 * launch at a time per workspace. */
HALO_API uint64_t halo_tx_build_workspace(uint32_t n);
/* Build n frames into fixed output slots: frame i at d_frames + i * out_stride (a multiple of
 * 4, at least 60), d_out_lens[i] = its length (0 when not built), d_result[i] (optional) =
 * HALO_TX_B_*. The bytes of a slot past the frame's last 4-byte word are left untouched.
 * `max_payload_hint` (0 = unknown) picks the lanes per frame. Asynchronous on `stream`.     */
HALO_API int halo_tx_build_batch_device(const halo_tx_build_desc_t* d_desc, uint32_t n, const uint8_t* d_payload,
                                        uint32_t flags, const halo_rx_netif_t* netif, uint32_t max_payload_hint,
                                        uint8_t* d_frames, uint32_t out_stride, uint16_t* d_out_lens,
                                        uint8_t* d_result, uint16_t* d_ip_id, void* d_workspace,
                                        uint64_t workspace_bytes, halo_stream_t stream);

/* ---- flow-key hashing --------------------------------------------
 * hashcode.GetHashCodeXXH3 (hashcode/hashcode.go:15-17 -> hashcode/xxh3.go:43-287, XXH3-64 with
 * the default secret and seed 0, ported from github.com/zeebo/xxh3 v1.1.0) over a batch of byte
 * strings, and the NAT flow-table keys the forward path hashes for every NATed packet. */
#define HALO_FLOW_NAT_LAN 0u  /* NatFlowHash{remote=dst, dport, lan host=src, sport, proto} as
                                 NatGetFlowByHash builds it (engine/ipv4_engine.go:524-551)   */
#define HALO_FLOW_NAT_WAN 1u  /* NatWanFlowHash{remote=src, sport, wan=dst, dport, proto} as
                                 NatGetFlowByWan builds it (engine/ipv4_engine.go:554-581)    */
#define HALO_NAT_SYMMETRIC 0u /* NetIfConfig.NatType (engine/ipv4_engine.go:423-426): remote  */
#define HALO_NAT_FULL_CONE 1u /* address/port kept (symmetric) or zeroed (any other value)   */

/* d_hash[i] = XXH3-64(d_bytes[d_offsets[i] : d_offsets[i] + d_lens[i]]). Byte offsets, any
 * alignment. Asynchronous on `stream`. */
HALO_API int halo_xxh3_64_batch_device(const uint8_t* d_bytes, const uint64_t* d_offsets, const uint32_t* d_lens,
                                       uint32_t n, uint64_t* d_hash, halo_stream_t stream);

/* For each parsed record: build the 13-byte little-endian flow key of `kind` (the ICMP remote
 * port is 0, the remote address and port are 0 unless nat_type is HALO_NAT_SYMMETRIC), hash it
 * with XXH3-64 (NatFlowHash.GetHashCode, engine/ipv4_engine.go:451-459; NatWanFlowHash
 * :471-479) into d_hash[i], and, when d_bucket is non-null, write the hashmap bucket
 * hash % bucket_count (hashmap/hashmap.go:64) into d_bucket[i]. Records are used as they are;
 * callers hash the records whose engine action is FORWARD. */
HALO_API int halo_flow_hash_device(const halo_rx_result_t* d_records, uint32_t n, uint32_t kind, uint32_t nat_type,
                                   uint64_t* d_hash, uint32_t bucket_count, uint32_t* d_bucket,
                                   halo_stream_t stream);

/* The same over compact records (HALO_RX_RECORD_COMPACT parse output): the five key fields are the
 * whole 16-byte record, so nothing is fetched that the key does not use (a full record's key fields
 * are 20 of its 32 bytes). Identical hashes and buckets for the same frames.                      */
HALO_API int halo_flow_hash_compact_device(const halo_rx_record16_t* d_records, uint32_t n, uint32_t kind,
                                           uint32_t nat_type, uint64_t* d_hash, uint32_t bucket_count,
                                           uint32_t* d_bucket, halo_stream_t stream);

/* The rx parse (halo_rx_parse_batch_device, same arguments and records) with the NAT flow key
 * of every record hashed in the same pass, exactly as halo_flow_hash_device would hash the
 * records it writes: the engine's receive -> forward -> NAT lookup chain without re-reading the
 * records. Full or compact records (flags); d_hash (8-byte aligned) and d_bucket as above.     */
HALO_API int halo_rx_parse_flow_batch_device(const uint8_t* d_bytes, const uint32_t* d_offsets_dw,
                                             const uint16_t* d_lens, uint32_t n, uint32_t flags,
                                             const halo_rx_netif_t* netif, uint32_t max_len_hint,
                                             halo_rx_result_t* d_out, uint32_t* d_status_hist,
                                             uint32_t flow_kind, uint32_t nat_type, uint64_t* d_hash,
                                             uint32_t bucket_count, uint32_t* d_bucket, halo_stream_t stream);

/* ---- route lookup ---------------------------------------------------
 * RouteTable (engine/ipv4_engine.go:270-390): a binary trie of route lists, longest-prefix
 * FindRoute with an ECMP pick lastMatch[fnv32a(ip) % len] (engine/engine.go:159). The trie is
 * the control plane and is kept on the host exactly as UpdateRoute builds it (including lists
 * emptied by DeleteRoute, which still end a lookup); halo_route_sync_device compiles it into a
 * DIR-24-8 table in HBM (a 2^24-entry first level, 256-entry second-level blocks for prefixes
 * longer than /24) and lookups run on the GPU only. Route ids identify the RouteEntry objects:
 * each insertion gets a fresh id. */
typedef struct halo_route_table halo_route_table_t;
typedef struct halo_route_entry {
    uint32_t dst_ip;       /* IpAddrToU(DstIpAddr)   */
    uint32_t network_mask; /* IpAddrToU(NetworkMask) */
    uint32_t next_hop;     /* IpAddrToU(NextHop); 0 for nil (direct routes) */
    uint32_t netif;        /* the caller's id for the NetIf name */
} halo_route_entry_t;
#define HALO_ROUTE_NONE 0xFFFFFFFFu  /* FindRoute returns nil (no route)                        */
#define HALO_ROUTE_PANIC 0xFFFFFFFEu /* the longest match is a list DeleteRoute emptied: Go's
                                        `% uint32(len(lastMatch))` divides by zero (:382)       */

HALO_API int halo_route_table_create(halo_route_table_t** out);
HALO_API int halo_route_table_destroy(halo_route_table_t* t);
/* UpdateRoute(old, new) (:304-348): walks old's prefix, drops entries equal to old (dst, mask,
 * next hop, netif), appends new (if non-null, with a fresh id written to *new_id). AddRoute is
 * update(r, r), DeleteRoute is update(r, NULL) (:293-301). */
HALO_API int halo_route_update(halo_route_table_t* t, const halo_route_entry_t* old_route,
                               const halo_route_entry_t* new_route, uint32_t* new_id);
HALO_API int halo_route_get(const halo_route_table_t* t, uint32_t id, halo_route_entry_t* out);
/* Compile the trie into the device table on `device` (allocates / grows HBM; synchronous).
 * Double-buffered: the new table is written into the generation not in use, after the device
 * has drained every lookup that could still read that one (a device synchronisation), and is
 * then published. A lookup sees the table last published when it was launched — never one
 * being rewritten, as FindRoute under RouteTable.RLock never does (engine/ipv4_engine.go:351).
 * Lookups and syncs may run on different threads: a lookup holds the table's read lock from
 * taking its view until its kernel is enqueued, and a sync takes the write lock before it
 * drains the device, so no launch can slip in between (RWMutex semantics, :270-275). */
HALO_API int halo_route_sync_device(halo_route_table_t* t, int device);
/* FindRoute for each address (IpAddrToU form) / each record's dst_ip: route id, HALO_ROUTE_NONE
 * or HALO_ROUTE_PANIC. Asynchronous on `stream`; uses the last synced table. */
HALO_API int halo_route_lookup_device(const halo_route_table_t* t, const uint32_t* d_ips, uint32_t n,
                                      uint32_t* d_route_ids, halo_stream_t stream);
HALO_API int halo_route_lookup_records_device(const halo_route_table_t* t, const halo_rx_result_t* d_records,
                                              uint32_t n, uint32_t* d_route_ids, halo_stream_t stream);
/* The rx parse (halo_rx_parse_batch_device, same arguments and records) with FindRoute of every
 * record's dst_ip in the same pass — the RxIpv4 -> Ipv4RouteForward -> FindRoute chain
 * (engine/ipv4_engine.go:18-47, :108-269, :351-390) without re-reading the records: d_route_ids
 * equals halo_route_lookup_records_device over the records written.                         */
HALO_API int halo_rx_parse_route_batch_device(const uint8_t* d_bytes, const uint32_t* d_offsets_dw,
                                              const uint16_t* d_lens, uint32_t n, uint32_t flags,
                                              const halo_rx_netif_t* netif, uint32_t max_len_hint,
                                              halo_rx_result_t* d_out, uint32_t* d_status_hist,
                                              const halo_route_table_t* table, uint32_t* d_route_ids,
                                              halo_stream_t stream);

/* ---- the reference engine's per-frame decision (engine/ethernet_engine.go:13-31,
 *      engine/ipv4_engine.go:18-47, engine/{udp,tcp,icmp}_engine.go) ------------------ */
typedef enum halo_rx_action {
    HALO_RX_ACT_DROP_ETH = 0,      /* ParseEthFrm error: logged and dropped              */
    HALO_RX_ACT_IGNORE_MAC = 1,    /* not for this NetIf (dst MAC filter)                */
    HALO_RX_ACT_ARP = 2,           /* -> HandleArp                                       */
    HALO_RX_ACT_IGNORE_TYPE = 3,   /* 802.3 / IPv6: silently ignored                     */
    HALO_RX_ACT_DROP_IP = 4,       /* ParseIpv4Pkt error (incl. build-defined totalLen)   */
    HALO_RX_ACT_BCAST_UDP = 5,     /* RxUdpBroadcast, UDP parse+verify OK (-> DHCP)      */
    HALO_RX_ACT_DROP_BCAST_UDP = 6,/* RxUdpBroadcast, UDP parse error                    */
    HALO_RX_ACT_IGNORE_BCAST = 7,  /* x.x.x.255 and not UDP                              */
    HALO_RX_ACT_FORWARD = 8,       /* Ipv4RouteForward (no L4 verification)              */
    HALO_RX_ACT_LOCAL_ICMP = 9,    /* RxIcmp OK                                          */
    HALO_RX_ACT_LOCAL_UDP = 10,    /* RxUdp OK -> UdpServiceMap                          */
    HALO_RX_ACT_LOCAL_TCP = 11,    /* RxTcp OK -> TcpServiceMap                          */
    HALO_RX_ACT_DROP_L4 = 12,      /* local L4 parse error: logged and dropped           */
    HALO_RX_ACT_LO_NOT_OWN = 13,   /* loopback drain: dst != NetIf.IpAddr, skipped       */
                                   /* (engine/engine.go:367-369)                         */
    HALO_RX_ACT_COUNT = 14
} halo_rx_action_t;

/* Host-side: maps n results to the action the reference engine takes (u8 per frame).
 * Pure host code over the kernel's records; no GPU needed. `action_hist` (optional)
 * receives HALO_RX_ACT_COUNT counters (incremented).                                    */
HALO_API int halo_rx_dispatch(const halo_rx_result_t* results, uint32_t n,
                              const halo_rx_netif_t* netif, uint8_t* actions,
                              uint32_t* action_hist);
/* The same over compact records. */
HALO_API int halo_rx_dispatch_compact(const halo_rx_record16_t* records, uint32_t n,
                                      const halo_rx_netif_t* netif, uint8_t* actions,
                                      uint32_t* action_hist);
/* PacketHandle's LoChan drain (engine/engine.go:353-381) over records parsed with
 * HALO_RX_L3_START: ParseIpv4Pkt error -> DROP_IP (:362-365); dst != NetIf.IpAddr ->
 * LO_NOT_OWN (:366-368); otherwise the local parse of ip_proto -> LOCAL_ICMP / LOCAL_UDP /
 * LOCAL_TCP, or DROP_L4 when it failed (:369-376). No broadcast or NAT branch: the drain
 * has none. */
HALO_API int halo_rx_dispatch_loopback(const halo_rx_result_t* results, uint32_t n,
                                       const halo_rx_netif_t* netif, uint8_t* actions,
                                       uint32_t* action_hist);

/* ---- synthetic traffic (bench + tests; SURVEY.md §8d generator) ----------------------
 * Every field of frame i is a pure function of (seed, i), so any shard of the global
 * stream [first_index, first_index + n) is generated independently.
 * halo_synth_layout (host): per-frame length, kind byte and ragged 4-byte-aligned dword
 * offsets (frames packed back to back, each rounded up to 4 bytes).
 *   size_mode : 0 = uniform `len`, 1 = IMIX 64/570/1500 at 7:4:1
 *   proto_mode: 0 = UDP, 1 = TCP, 2 = ICMP, 3 = mix UDP 50 / TCP 40 / ICMP 10
 *   mutate_shift: frame mutated with probability 2^-mutate_shift (0 = never)
 *   kinds[i]  : bits 0-1 protocol (0 UDP, 1 TCP, 2 ICMP), bit 7 = mutated
 *   *total_bytes = bytes the ragged layout spans.
 * halo_synth_frames_device: writes the frame bytes for a layout into d_bytes (ragged
 * dword offsets, or i*stride when d_offsets_dw == NULL). A mutated frame has one bit
 * flipped in [14, len) after its checksums were filled.                                 */
HALO_API int halo_synth_layout(uint64_t seed, uint64_t first_index, uint32_t n,
                               uint32_t size_mode, uint32_t len, uint32_t proto_mode,
                               uint32_t mutate_shift, uint16_t* lens, uint32_t* offsets_dw,
                               uint8_t* kinds, uint64_t* total_bytes);
HALO_API int halo_synth_frames_device(uint64_t seed, uint64_t first_index, uint32_t n,
                                      const uint16_t* d_lens, const uint32_t* d_offsets_dw,
                                      uint64_t stride, const uint8_t* d_kinds,
                                      const halo_rx_netif_t* netif, uint8_t* d_bytes,
                                      halo_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* HALO_RX_H */
