/*
 * halo_rx_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker and the CPU baseline).
 *
 * A plain-C, scalar, one-frame-at-a-time restatement of halo's receive parse path, written
 * to follow the Go source line by line (slices become pointer/length pairs, `append` into
 * `sumData` becomes a copy into a stack buffer, errors become status codes). Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it; the product library
 * (halo_amd/lib/libhalo_rx.so) never links or calls it.
 *
 * Followed reference lines (all paths under /root/reference):
 *   GetCheckSum        protocol/utils.go:11-31      IpAddrToU      protocol/utils.go:34-44
 *   ParseEthFrm        protocol/ethernet.go:29-55   ParseIpv4Pkt   protocol/ipv4.go:48-86
 *   ParseUdpPkt        protocol/udp.go:21-49        ParseTcpPkt    protocol/tcp.go:36-70
 *   ParseIcmpPkt       protocol/icmp.go:33-63       NatGetSrcDstPort protocol/ipv4.go:229-246
 *   RxEthernet         engine/ethernet_engine.go:13-31
 *   RxIpv4             engine/ipv4_engine.go:18-47
 *   RxUdp / RxUdpBroadcast engine/udp_engine.go:10-21, :35-44
 *   RxTcp              engine/tcp_engine.go:10-26   RxIcmp         engine/icmp_engine.go:12-23
 *   PacketHandle's LoChan drain (HALO_RX_L3_START)   engine/engine.go:353-381
 *
 * Parity pinning: the reference is Go and no Go toolchain exists here or on the GPU box, so
 * the reference itself cannot run. GetCheckSum is pinned by the RFC 1071 §3 known answer and
 * the IPv4-header and canonical-frame known answers of SURVEY.md §8a; the parse semantics are
 * pinned only by this restatement and the independent pure-Python restatement in
 * oracle/ref_py.py agreeing on the committed fixtures (tests/golden/). DESIGN.md records this
 * as "parse semantics: parity unpinned by reference execution".
 *
 * Two documented deviations, both where the reference has no defined result:
 *   - ParseIpv4Pkt slices pkt[20:totalLen] (ipv4.go:84): Go panics for totalLen < 20 and
 *     reads stale buffer bytes or panics for totalLen > len(pkt). Reported as
 *     HALO_RX_IP_TOTLEN_UNDERFLOW / _OVERRUN.
 *   - HALO_RX_JUMBO_EXT lifts the 1514/1500/1480 limits to 9014/9000/8980.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/halo_rx.h"

#define ORA_API __attribute__((visibility("default")))

typedef struct { const uint8_t* p; size_t len; } slice_t;

typedef struct {
    int csum;     /* protocol.CheckSumEnable */
    size_t eth_max, ip_max, l4_max;
} ora_cfg_t;

static ora_cfg_t cfg_of(uint32_t flags) {
    ora_cfg_t c;
    c.csum = (flags & HALO_RX_CSUM_ENABLE) != 0;
    if (flags & HALO_RX_JUMBO_EXT) { c.eth_max = 9014; c.ip_max = 9000; c.l4_max = 8980; }
    else { c.eth_max = 1514; c.ip_max = 1500; c.l4_max = 1480; }
    return c;
}

/* protocol/utils.go:11-31 */
ORA_API uint16_t ora_get_checksum(const uint8_t* data, size_t len) {
    uint32_t sum = 0;
    size_t length = len, index = 0;
    while (length > 1) {
        sum += ((uint32_t)data[index] << 8) + (uint32_t)data[index + 1];
        index += 2;
        length -= 2;
    }
    if (length > 0) sum += (uint32_t)data[index] << 8;
    while (sum >> 16) sum = (sum & 0xffff) + (sum >> 16);
    return (uint16_t)~sum;
}

/* protocol/utils.go:34-44 */
static uint32_t ip_addr_to_u(const uint8_t* a) {
    if (!a) return 0;
    return ((uint32_t)a[0] << 24) | ((uint32_t)a[1] << 16) | ((uint32_t)a[2] << 8) | (uint32_t)a[3];
}
static uint16_t be16(const uint8_t* p) { return (uint16_t)(((uint16_t)p[0] << 8) | p[1]); }

/* protocol/ethernet.go:29-55. Returns 0 or a status. */
static int parse_eth_frm(slice_t frm, const ora_cfg_t* c, slice_t* payload, const uint8_t** dst,
                         const uint8_t** src, uint16_t* eth_proto) {
    *eth_proto = 0xffff;
    if (frm.len < 42 || frm.len > c->eth_max) return HALO_RX_ETH_LEN;
    const uint16_t t = be16(frm.p + 12);
    if (t != 0x05dc && t != 0x0800 && t != 0x0806 && t != 0x86dd) return HALO_RX_ETH_TYPE;
    *dst = frm.p;
    *src = frm.p + 6;
    *eth_proto = t;
    payload->p = frm.p + 14;
    payload->len = frm.len - 14;
    return 0;
}

/* protocol/ipv4.go:48-86 */
static int parse_ipv4_pkt(slice_t pkt, const ora_cfg_t* c, slice_t* payload, uint8_t* proto,
                          const uint8_t** src, const uint8_t** dst, uint16_t* total_len_out) {
    *proto = 0xff;
    if (pkt.len < 20 || pkt.len > c->ip_max) return HALO_RX_IP_LEN;
    if (pkt.p[0] != 0x45) return HALO_RX_IP_VER;
    const uint16_t total_len = be16(pkt.p + 2);
    if ((pkt.p[6] != 0x40 && pkt.p[6] != 0x00) || pkt.p[7] != 0x00) return HALO_RX_IP_FRAG;
    const uint8_t pr = pkt.p[9];
    if (pr != 0x01 && pr != 0x06 && pr != 0x11) return HALO_RX_IP_PROTO;
    if (c->csum && ora_get_checksum(pkt.p, 20) != 0) return HALO_RX_IP_HDR_CKSUM;
    /* payload = pkt[20:totalLen]: undefined in Go outside [20, len] (see header comment) */
    if (total_len < 20) return HALO_RX_IP_TOTLEN_UNDERFLOW;
    if (total_len > pkt.len) return HALO_RX_IP_TOTLEN_OVERRUN;
    *proto = pr;
    *src = pkt.p + 12;
    *dst = pkt.p + 16;
    *total_len_out = total_len;
    payload->p = pkt.p + 20;
    payload->len = (size_t)total_len - 20;
    return 0;
}

/* protocol/udp.go:21-49 */
static int parse_udp_pkt(slice_t pkt, const uint8_t* src_addr, const uint8_t* dst_addr, const ora_cfg_t* c,
                         slice_t* payload, uint16_t* sport, uint16_t* dport) {
    if (pkt.len < 8 || pkt.len > c->l4_max) return HALO_RX_L4_LEN;
    const uint16_t src_port = be16(pkt.p), dst_port = be16(pkt.p + 2);
    const uint16_t total_len = be16(pkt.p + 4); /* udp.go:30 — NOT validated */
    if (c->csum) {
        uint8_t sum_data[12 + 9000];
        memcpy(sum_data, src_addr, 4);
        memcpy(sum_data + 4, dst_addr, 4);
        sum_data[8] = 0x00;
        sum_data[9] = 0x11;
        sum_data[10] = (uint8_t)(total_len >> 8);
        sum_data[11] = (uint8_t)total_len;
        memcpy(sum_data + 12, pkt.p, pkt.len); /* all len(pkt) bytes (udp.go:41) */
        if (ora_get_checksum(sum_data, 12 + pkt.len) != 0) return HALO_RX_L4_CKSUM;
    }
    *sport = src_port;
    *dport = dst_port;
    payload->p = pkt.p + 8;
    payload->len = pkt.len - 8;
    return 0;
}

/* protocol/tcp.go:36-70 */
static int parse_tcp_pkt(slice_t pkt, const uint8_t* src_addr, const uint8_t* dst_addr, const ora_cfg_t* c,
                         slice_t* payload, uint16_t* sport, uint16_t* dport, uint32_t* seq, uint32_t* ack,
                         uint8_t* flags) {
    if (pkt.len < 20 || pkt.len > c->l4_max) return HALO_RX_L4_LEN;
    const uint16_t src_port = be16(pkt.p), dst_port = be16(pkt.p + 2);
    const uint32_t seq_num = ((uint32_t)be16(pkt.p + 4) << 16) | be16(pkt.p + 6);
    const uint32_t ack_num = ((uint32_t)be16(pkt.p + 8) << 16) | be16(pkt.p + 10);
    const size_t header_len = pkt.p[12] >> 4; /* tcp.go:49: 32-bit words, used as bytes */
    const uint8_t fl = pkt.p[13];
    if (c->csum) {
        const size_t total_len = pkt.len; /* tcp.go:54 */
        uint8_t sum_data[12 + 9000];
        memcpy(sum_data, src_addr, 4);
        memcpy(sum_data + 4, dst_addr, 4);
        sum_data[8] = 0x00;
        sum_data[9] = 0x06;
        sum_data[10] = (uint8_t)(total_len >> 8);
        sum_data[11] = (uint8_t)total_len;
        memcpy(sum_data + 12, pkt.p, pkt.len);
        if (ora_get_checksum(sum_data, 12 + pkt.len) != 0) return HALO_RX_L4_CKSUM;
    }
    *sport = src_port;
    *dport = dst_port;
    *seq = seq_num;
    *ack = ack_num;
    *flags = fl;
    payload->p = pkt.p + header_len; /* tcp.go:68 */
    payload->len = pkt.len - header_len;
    return 0;
}

/* protocol/icmp.go:33-63 (checksum always verified, icmp.go:53) */
static int parse_icmp_pkt(slice_t pkt, const ora_cfg_t* c, slice_t* payload, uint8_t* type,
                          uint16_t* id, uint16_t* seq) {
    *type = 0xff;
    if (pkt.len < 8 || pkt.len > c->l4_max) return HALO_RX_L4_LEN;
    const uint8_t t = pkt.p[0];
    if (t != 0x08 && t != 0x00 && t != 0x0b) return HALO_RX_ICMP_TYPE;
    if (pkt.p[1] != 0x00) return HALO_RX_ICMP_CODE;
    if (ora_get_checksum(pkt.p, pkt.len) != 0) return HALO_RX_L4_CKSUM;
    *type = t;
    *id = be16(pkt.p + 4);
    *seq = be16(pkt.p + 6);
    payload->p = pkt.p + 8;
    payload->len = pkt.len - 8;
    return 0;
}

/* protocol/ipv4.go:229-246 */
static void nat_get_src_dst_port(slice_t pkt, uint16_t* sp, uint16_t* dp) {
    *sp = *dp = 0;
    if (pkt.len < 26) return;
    switch (pkt.p[9]) {
        case 0x01: *sp = *dp = be16(pkt.p + 24); break;
        case 0x06:
        case 0x11: *sp = be16(pkt.p + 20); *dp = be16(pkt.p + 22); break;
        default: break;
    }
}

static void set_payload(halo_rx_result_t* r, const uint8_t* frame, slice_t s) {
    r->payload_off = (uint16_t)(s.p - frame);
    r->payload_len = (uint16_t)s.len;
}

/* The per-frame chain RxEthernet -> RxIpv4 -> Rx{Udp,Tcp,Icmp} as parse calls, every L4
 * verdict evaluated (the record definition of include/halo_rx.h). */
ORA_API void ora_rx_frame(const uint8_t* frame, uint32_t len, uint32_t flags, const halo_rx_netif_t* netif,
                          halo_rx_result_t* r) {
    memset(r, 0, sizeof *r);
    r->ethertype = 0xffff;
    r->ip_proto = 0xff;
    const ora_cfg_t c = cfg_of(flags);
    slice_t frm = {frame, len}, eth_payload;
    int st;
    if (flags & HALO_RX_L3_START) {
        /* a LoChan packet (engine/engine.go:361): ParseIpv4Pkt straight on the buffer */
        r->ethertype = 0x0800;
        eth_payload = frm;
    } else {
        const uint8_t *dst_mac = NULL, *src_mac = NULL;
        uint16_t eth_proto;
        st = parse_eth_frm(frm, &c, &eth_payload, &dst_mac, &src_mac, &eth_proto);
        r->ethertype = eth_proto;
        if (st) { r->status = (uint8_t)st; return; }
        static const uint8_t bcast[6] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
        if (memcmp(dst_mac, netif->mac, 6) == 0 || memcmp(dst_mac, bcast, 6) == 0) r->flags |= HALO_RX_F_MAC_MATCH;
        set_payload(r, frame, eth_payload);
        if (eth_proto != 0x0800) return;
    }

    slice_t ip_payload;
    uint8_t proto;
    const uint8_t *src = NULL, *dst = NULL;
    uint16_t total_len = 0;
    st = parse_ipv4_pkt(eth_payload, &c, &ip_payload, &proto, &src, &dst, &total_len);
    if (st) { r->status = (uint8_t)st; return; }
    r->ip_proto = proto;
    r->ip_total_len = total_len;
    r->src_ip = ip_addr_to_u(src);
    r->dst_ip = ip_addr_to_u(dst);
    if (dst[3] == 255) r->flags |= HALO_RX_F_IP_BCAST;
    if (r->dst_ip == netif->ip) r->flags |= HALO_RX_F_DST_IS_OWN;
    nat_get_src_dst_port(eth_payload, &r->sport, &r->dport);
    set_payload(r, frame, ip_payload);

    slice_t l4_payload;
    if (proto == 0x11) {
        uint16_t sp, dp;
        /* pseudo dst: NetIf IP (unicast, udp_engine.go:11) or packet dst (broadcast, :36);
           both equal the packet's dst bytes on every branch that reaches the parse */
        st = parse_udp_pkt(ip_payload, src, dst, &c, &l4_payload, &sp, &dp);
    } else if (proto == 0x06) {
        uint16_t sp, dp;
        uint32_t seq, ack;
        uint8_t fl;
        st = parse_tcp_pkt(ip_payload, src, dst, &c, &l4_payload, &sp, &dp, &seq, &ack, &fl);
        if (!st) { r->l4_aux = fl; r->l4_seq = seq; r->l4_ack = ack; }
    } else {
        uint8_t type;
        uint16_t id, seq;
        st = parse_icmp_pkt(ip_payload, &c, &l4_payload, &type, &id, &seq);
        if (!st) { r->l4_aux = type; r->l4_seq = ((uint32_t)id << 16) | seq; }
    }
    if (st) { r->status = (uint8_t)st; return; }
    set_payload(r, frame, l4_payload);
}

/* engine/ethernet_engine.go:13-31 -> engine/ipv4_engine.go:18-47 -> Rx{Udp,Tcp,Icmp}:
 * the action the reference engine takes for one frame, re-derived from the parse calls
 * (independent of the record-based halo_rx_dispatch in the product library). */
ORA_API int ora_engine_rx(const uint8_t* frame, uint32_t len, uint32_t flags, const halo_rx_netif_t* netif) {
    const ora_cfg_t c = cfg_of(flags);
    slice_t frm = {frame, len}, eth_payload;
    const uint8_t *dst_mac, *src_mac;
    uint16_t eth_proto;
    if (parse_eth_frm(frm, &c, &eth_payload, &dst_mac, &src_mac, &eth_proto)) return HALO_RX_ACT_DROP_ETH;
    static const uint8_t bcast[6] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
    if (!(memcmp(dst_mac, netif->mac, 6) == 0 || memcmp(dst_mac, bcast, 6) == 0)) return HALO_RX_ACT_IGNORE_MAC;
    if (eth_proto == 0x0806) return HALO_RX_ACT_ARP;
    if (eth_proto != 0x0800) return HALO_RX_ACT_IGNORE_TYPE;
    slice_t ip_payload, l4;
    uint8_t proto;
    const uint8_t *src, *dst;
    uint16_t total_len;
    if (parse_ipv4_pkt(eth_payload, &c, &ip_payload, &proto, &src, &dst, &total_len)) return HALO_RX_ACT_DROP_IP;
    uint16_t sp, dp;
    if (dst[3] == 255) {
        if (proto != 0x11) return HALO_RX_ACT_IGNORE_BCAST;
        return parse_udp_pkt(ip_payload, src, dst, &c, &l4, &sp, &dp) ? HALO_RX_ACT_DROP_BCAST_UDP
                                                                      : HALO_RX_ACT_BCAST_UDP;
    }
    uint8_t own_ip[4] = {(uint8_t)(netif->ip >> 24), (uint8_t)(netif->ip >> 16), (uint8_t)(netif->ip >> 8),
                         (uint8_t)netif->ip};
    if (memcmp(dst, own_ip, 4) != 0 || netif->nat_enable) return HALO_RX_ACT_FORWARD;
    if (proto == 0x01) {
        uint8_t t;
        uint16_t id, sq;
        return parse_icmp_pkt(ip_payload, &c, &l4, &t, &id, &sq) ? HALO_RX_ACT_DROP_L4 : HALO_RX_ACT_LOCAL_ICMP;
    }
    if (proto == 0x11)
        return parse_udp_pkt(ip_payload, src, own_ip, &c, &l4, &sp, &dp) ? HALO_RX_ACT_DROP_L4
                                                                          : HALO_RX_ACT_LOCAL_UDP;
    uint32_t seq, ack;
    uint8_t fl;
    return parse_tcp_pkt(ip_payload, src, own_ip, &c, &l4, &sp, &dp, &seq, &ack, &fl) ? HALO_RX_ACT_DROP_L4
                                                                                       : HALO_RX_ACT_LOCAL_TCP;
}

/* engine/engine.go:353-381: PacketHandle's LoChan drain for one packet (HALO_RX_L3_START). */
ORA_API int ora_engine_lo(const uint8_t* pkt, uint32_t len, uint32_t flags, const halo_rx_netif_t* netif) {
    const ora_cfg_t c = cfg_of(flags);
    slice_t ipv4_pkt = {pkt, len}, ip_payload, l4;
    uint8_t proto;
    const uint8_t *src, *dst;
    uint16_t total_len;
    if (parse_ipv4_pkt(ipv4_pkt, &c, &ip_payload, &proto, &src, &dst, &total_len)) return HALO_RX_ACT_DROP_IP;
    uint8_t own_ip[4] = {(uint8_t)(netif->ip >> 24), (uint8_t)(netif->ip >> 16), (uint8_t)(netif->ip >> 8),
                         (uint8_t)netif->ip};
    if (memcmp(dst, own_ip, 4) != 0) return HALO_RX_ACT_LO_NOT_OWN; /* :366-368 */
    uint16_t sp, dp;
    switch (proto) { /* :369-376 -> RxIcmp / RxUdp / RxTcp with the NetIf address as pseudo dst */
        case 0x01: {
            uint8_t t;
            uint16_t id, sq;
            return parse_icmp_pkt(ip_payload, &c, &l4, &t, &id, &sq) ? HALO_RX_ACT_DROP_L4 : HALO_RX_ACT_LOCAL_ICMP;
        }
        case 0x11:
            return parse_udp_pkt(ip_payload, src, own_ip, &c, &l4, &sp, &dp) ? HALO_RX_ACT_DROP_L4
                                                                              : HALO_RX_ACT_LOCAL_UDP;
        default: {
            uint32_t seq, ack;
            uint8_t fl;
            return parse_tcp_pkt(ip_payload, src, own_ip, &c, &l4, &sp, &dp, &seq, &ack, &fl) ? HALO_RX_ACT_DROP_L4
                                                                                           : HALO_RX_ACT_LOCAL_TCP;
        }
    }
}

/* ---- batches (ragged dword offsets, or strided when offsets_dw == NULL) ---------------- */
typedef struct {
    const uint8_t* bytes;
    const uint32_t* offsets_dw;
    const uint16_t* lens;
    uint64_t stride;
    uint32_t len;
    uint32_t flags;
    const halo_rx_netif_t* netif;
    halo_rx_result_t* out;
    uint64_t first, last;
    uint32_t reps;
    uint32_t hist[HALO_RX_STATUS_COUNT];
} ora_job_t;

static void* ora_job(void* arg) {
    ora_job_t* j = (ora_job_t*)arg;
    memset(j->hist, 0, sizeof j->hist);
    for (uint32_t r = 0; r < j->reps; ++r) {
        for (uint64_t i = j->first; i < j->last; ++i) {
            const uint8_t* f = j->offsets_dw ? j->bytes + ((uint64_t)j->offsets_dw[i] << 2) : j->bytes + i * j->stride;
            const uint32_t L = j->lens ? j->lens[i] : j->len;
            ora_rx_frame(f, L, j->flags, j->netif, &j->out[i]);
            if (r == 0) j->hist[j->out[i].status]++;
        }
    }
    return NULL;
}

/* threads <= 1: run on the calling thread (the reference's one goroutine per NetIf). `reps`: every
 * thread parses its shard that many times (the same records each time) — for timing many passes
 * with one thread start each, so the thread starts do not dominate a many-core measurement. */
ORA_API int ora_rx_batch_reps(const uint8_t* bytes, const uint32_t* offsets_dw, const uint16_t* lens, uint64_t stride,
                              uint32_t len, uint32_t n, uint32_t flags, const halo_rx_netif_t* netif,
                              halo_rx_result_t* out, uint32_t* hist, int threads, uint32_t reps) {
    if (reps < 1) reps = 1;
    if (threads < 1) threads = 1;
    if (threads > 1024) threads = 1024;
    ora_job_t* jobs = (ora_job_t*)calloc((size_t)threads, sizeof(ora_job_t));
    pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !tid) { free(jobs); free(tid); return -1; }
    for (int t = 0; t < threads; ++t) {
        ora_job_t* j = &jobs[t];
        j->bytes = bytes; j->offsets_dw = offsets_dw; j->lens = lens; j->stride = stride; j->len = len;
        j->flags = flags; j->netif = netif; j->out = out;
        j->first = (uint64_t)n * t / threads;
        j->last = (uint64_t)n * (t + 1) / threads;
        j->reps = reps;
    }
    int rc = 0;
    int started = 0;
    for (int t = 1; t < threads; ++t) {
        if (pthread_create(&tid[t], NULL, ora_job, &jobs[t]) != 0) { rc = -1; break; }
        started = t;
    }
    if (rc == 0) ora_job(&jobs[0]);
    for (int t = 1; t <= started; ++t) pthread_join(tid[t], NULL);
    if (rc == 0 && hist)
        for (int t = 0; t < threads; ++t)
            for (int s = 0; s < HALO_RX_STATUS_COUNT; ++s) hist[s] += jobs[t].hist[s];
    free(jobs);
    free(tid);
    return rc;
}

ORA_API int ora_rx_batch(const uint8_t* bytes, const uint32_t* offsets_dw, const uint16_t* lens, uint64_t stride,
                         uint32_t len, uint32_t n, uint32_t flags, const halo_rx_netif_t* netif,
                         halo_rx_result_t* out, uint32_t* hist, int threads) {
    return ora_rx_batch_reps(bytes, offsets_dw, lens, stride, len, n, flags, netif, out, hist, threads, 1);
}

ORA_API void ora_engine_batch(const uint8_t* bytes, const uint32_t* offsets_dw, const uint16_t* lens,
                              uint64_t stride, uint32_t len, uint32_t n, uint32_t flags,
                              const halo_rx_netif_t* netif, uint8_t* actions) {
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* f = offsets_dw ? bytes + ((uint64_t)offsets_dw[i] << 2) : bytes + i * stride;
        const uint32_t L = lens ? lens[i] : len;
        actions[i] = (uint8_t)((flags & HALO_RX_L3_START) ? ora_engine_lo(f, L, flags, netif)
                                                            : ora_engine_rx(f, L, flags, netif));
    }
}

/* ---- synthetic-traffic twin (the spec halo_amd/csrc/synth.hip implements) ---
 * Written independently from the spec: every random field of frame i is drawn from
 * splitmix64 streams keyed by (seed, i); the frame is then built byte by byte the way
 * BuildEthFrm/BuildIpv4Pkt/BuildUdpPkt/BuildTcpPkt/BuildIcmpPkt lay it out, and the
 * checksums are filled with ora_get_checksum over pseudo-header + segment.               */
static uint64_t sm64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint64_t draw(uint64_t key, uint64_t slot) { return sm64(key + slot * 0xD6E8FEB86659FD93ull); }

ORA_API void ora_synth_kind(uint64_t seed, uint64_t index, uint32_t size_mode, uint32_t len, uint32_t proto_mode,
                            uint32_t mutate_shift, uint16_t* out_len, uint8_t* out_kind) {
    const uint64_t key = sm64(seed ^ sm64(index));
    uint32_t L = len;
    if (size_mode == 1) {
        const uint64_t r = draw(key, 1) % 12;
        L = r < 7 ? 64 : (r < 11 ? 570 : 1500);
    }
    uint32_t proto = proto_mode;
    if (proto_mode == 3) {
        const uint64_t r = draw(key, 2) % 10;
        proto = r < 5 ? 0 : (r < 9 ? 1 : 2);
    }
    uint32_t mut = 0;
    if (mutate_shift) mut = (draw(key, 3) & ((1ull << mutate_shift) - 1)) == 0;
    *out_len = (uint16_t)L;
    *out_kind = (uint8_t)(proto | (mut << 7));
}

static void put16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void put32(uint8_t* p, uint32_t v) { put16(p, v >> 16); put16(p + 2, v & 0xffff); }

ORA_API void ora_synth_frame(uint64_t seed, uint64_t index, uint32_t len, uint8_t kind, const halo_rx_netif_t* netif,
                             uint8_t* f) {
    const uint64_t key = sm64(seed ^ sm64(index));
    const uint32_t proto = kind & 3u;
    /* payload stream first: byte b = byte (b%4) of the b/4-th little-endian dword */
    for (uint32_t b = 0; b < len; ++b) {
        const uint32_t d = b >> 2;
        const uint32_t dw = (uint32_t)(draw(key, 64 + (d >> 1)) >> (32 * (d & 1)));
        f[b] = (uint8_t)(dw >> (8 * (b & 3)));
    }
    /* Ethernet */
    memcpy(f, netif->mac, 6);
    const uint64_t rm = draw(key, 5);
    const uint32_t mlo = ((uint32_t)rm & 0xFFFFFFFCu) | 2u, mhi = (uint32_t)(rm >> 32);
    f[6] = (uint8_t)mlo; f[7] = (uint8_t)(mlo >> 8); f[8] = (uint8_t)(mlo >> 16); f[9] = (uint8_t)(mlo >> 24);
    f[10] = (uint8_t)mhi; f[11] = (uint8_t)(mhi >> 8);
    put16(f + 12, 0x0800);
    /* IPv4 */
    const uint64_t ri = draw(key, 6);
    const uint32_t total_len = len - 14;
    const uint32_t src_ip = 0x0A000000u | ((uint32_t)ri & 0x00FFFFFFu);
    f[14] = 0x45; f[15] = 0x00;
    put16(f + 16, total_len);
    put16(f + 18, (uint32_t)(ri >> 24) & 0xffff);
    f[20] = ((ri >> 40) & 1) ? 0x40 : 0x00; f[21] = 0x00;
    f[22] = (uint8_t)((ri >> 48) % 255 + 1);
    f[23] = proto == 0 ? 0x11 : (proto == 1 ? 0x06 : 0x01);
    put16(f + 24, 0);
    put32(f + 26, src_ip);
    put32(f + 30, netif->ip);
    put16(f + 24, ora_get_checksum(f + 14, 20));
    /* L4 */
    const uint64_t rp = draw(key, 7), rs = draw(key, 8);
    uint32_t sport = (uint32_t)rp & 0xffff, dport = (uint32_t)(rp >> 16) & 0xffff;
    uint8_t* s = f + 34;
    const uint32_t seg_len = total_len - 20;
    if (proto == 2) {
        s[0] = 0x08; s[1] = 0x00; put16(s + 2, 0); put16(s + 4, sport); put16(s + 6, dport);
        put16(s + 2, ora_get_checksum(s, seg_len));
    } else {
        if (!sport) sport = 1;
        if (!dport) dport = 1;
        put16(s, sport);
        put16(s + 2, dport);
        uint32_t cks_at;
        if (proto == 0) {
            put16(s + 4, seg_len); put16(s + 6, 0); cks_at = 6;
        } else {
            put32(s + 4, (uint32_t)rs); put32(s + 8, (uint32_t)(rs >> 32));
            s[12] = 0x50; s[13] = 0x18;
            put16(s + 14, (uint32_t)draw(key, 9) & 0xffff);
            put16(s + 16, 0); put16(s + 18, 0); cks_at = 16;
        }
        uint8_t* sum_data = (uint8_t*)malloc(12 + seg_len);
        memcpy(sum_data, f + 26, 8);
        sum_data[8] = 0; sum_data[9] = proto == 0 ? 0x11 : 0x06;
        put16(sum_data + 10, seg_len);
        memcpy(sum_data + 12, s, seg_len);
        put16(s + cks_at, ora_get_checksum(sum_data, 12 + seg_len));
        free(sum_data);
    }
    if (kind & 0x80) {
        const uint64_t bit = draw(key, 4) % (8ull * (len - 14)) + 8ull * 14;
        f[bit >> 3] ^= (uint8_t)(1u << (bit & 7));
    }
}
