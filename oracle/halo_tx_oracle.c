/*
 * halo_tx_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline for SURVEY.md §8f
 * row f2, the forward/transmit rewrite). Linked into oracle/liboracle.so next to the rx
 * restatement; the product library never links or calls it.
 *
 * Followed reference lines (paths under /root/reference), restated one Go function at a time
 * on (pointer, length) slices; `append` into `sumData` becomes a copy into a heap buffer:
 *   HandleIpv4PktTtl     protocol/ipv4.go:134-145
 *   ReCalcIpv4CheckSum   protocol/ipv4.go:148-161
 *   ReCalcIcmpCheckSum   protocol/ipv4.go:164-174
 *   ReCalcTcpCheckSum    protocol/ipv4.go:177-200
 *   ReCalcUdpCheckSum    protocol/ipv4.go:203-226
 *   NatChangeSrc / Dst   protocol/ipv4.go:249-275, :277-302
 *   step order           engine/ipv4_engine.go:108-269 (Ipv4RouteForward: DNAT, TTL, SNAT)
 *   eth_tx SW checksum   cgo/dpdk.c:333-365 with offloads off, calling DPDK 20.11.10 LTS
 *                        (README.md:103, not vendored, not in this image) rte_ipv4_cksum and
 *                        rte_ipv4_udptcp_cksum from lib/librte_net/rte_ip.h, restated from the
 *                        published header: header length from IHL (rte_ipv4_hdr_len), IPv4
 *                        checksum = ~raw_sum, L4 length = total_length - IHL*4 (0 when
 *                        total_length < IHL*4), pseudo header {src, dst, 0, proto, l4_len},
 *                        result 0 -> 0xFFFF for UDP only (RFC 768).
 *
 * Pinning: the Go functions cannot run here (no Go toolchain); GetCheckSum is pinned by the
 * RFC 1071 known answer, the rewrite semantics by this restatement and the independent Python
 * one in oracle/ref_py.py agreeing on tests/golden/tx_*.  DPDK is absent, so the DPDK fill is
 * pinned only by RFC 768/1071 arithmetic and by agreeing with ReCalc* on well-formed packets
 * (tests/test_oracle.py); DESIGN.md §5 says "parity unpinned by reference execution".
 *
 * Build-defined behaviour where the reference has none (documented in include/halo_rx.h):
 *   - DPDK writes/reads past send_len into the mbuf when total_length or IHL point beyond the
 *     frame; here the affected checksum is left zero and HALO_TX_R_OVERRUN is reported.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/halo_rx.h"

#define ORA_API __attribute__((visibility("default")))

uint16_t ora_get_checksum(const uint8_t* data, size_t len); /* halo_rx_oracle.c (utils.go:11-31) */

static uint16_t be16(const uint8_t* p) { return (uint16_t)(((uint16_t)p[0] << 8) | p[1]); }

/* protocol/ipv4.go:148-161 */
/* Each helper returns 1 when its length guard returned early (HALO_TX_R_SKIPPED), else 0. */
static int recalc_ipv4(uint8_t* pkt, size_t len, int csum_enable) {
    if (len < 20) return 1;
    pkt[10] = 0x00;
    pkt[11] = 0x00;
    if (!csum_enable) return 0;
    uint16_t sum = ora_get_checksum(pkt, 20);
    pkt[10] = (uint8_t)(sum >> 8);
    pkt[11] = (uint8_t)sum;
    return 0;
}

/* protocol/ipv4.go:164-174 (CheckSumEnable is not consulted) */
static int recalc_icmp(uint8_t* pkt, size_t len) {
    if (len < 24) return 1;
    pkt[22] = 0x00;
    pkt[23] = 0x00;
    uint16_t sum = ora_get_checksum(pkt + 20, len - 20);
    pkt[22] = (uint8_t)(sum >> 8);
    pkt[23] = (uint8_t)sum;
    return 0;
}

/* protocol/ipv4.go:177-200 (TCP: guard 38, field 36, proto 6) and :203-226 (UDP: guard 28,
 * field 26, proto 17). totalLen-20 is Go int arithmetic truncated to two bytes. */
static int recalc_l4(uint8_t* pkt, size_t len, int csum_enable, size_t guard, size_t field, uint8_t proto) {
    if (len < guard) return 1;
    pkt[field] = 0x00;
    pkt[field + 1] = 0x00;
    if (!csum_enable) return 0;
    uint8_t* sum_data = (uint8_t*)malloc(12 + len - 20);
    if (!sum_data) abort();
    memcpy(sum_data, pkt + 12, 4);
    memcpy(sum_data + 4, pkt + 16, 4);
    sum_data[8] = 0x00;
    sum_data[9] = proto;
    int total_len = (int)be16(pkt + 2);
    sum_data[10] = (uint8_t)((total_len - 20) >> 8);
    sum_data[11] = (uint8_t)(total_len - 20);
    memcpy(sum_data + 12, pkt + 20, len - 20);
    uint16_t sum = ora_get_checksum(sum_data, 12 + len - 20);
    free(sum_data);
    pkt[field] = (uint8_t)(sum >> 8);
    pkt[field + 1] = (uint8_t)sum;
    return 0;
}

/* protocol/ipv4.go:134-145. Returns the bool result; *skip as the helpers above. */
static int handle_ipv4_pkt_ttl(uint8_t* pkt, size_t len, int csum_enable, int* skip) {
    if (len < 9) { *skip |= 1; return 0; }
    if (pkt[8] <= 1) return 0;
    pkt[8] -= 0x01;
    *skip |= recalc_ipv4(pkt, len, csum_enable);
    return 1;
}

/* protocol/ipv4.go:249-275 (src) and :277-302 (dst). */
static int nat_change(uint8_t* pkt, size_t len, uint32_t ip, uint16_t port, int dst, int csum_enable) {
    if (len < 26) return 1;
    uint8_t* a = pkt + (dst ? 16 : 12);
    a[0] = (uint8_t)(ip >> 24);
    a[1] = (uint8_t)(ip >> 16);
    a[2] = (uint8_t)(ip >> 8);
    a[3] = (uint8_t)ip;
    int skip = recalc_ipv4(pkt, len, csum_enable);
    switch (pkt[9]) {
    case 1: /* IPH_PROTO_ICMP: the echo identifier is both NAT keys */
        pkt[24] = (uint8_t)(port >> 8);
        pkt[25] = (uint8_t)port;
        skip |= recalc_icmp(pkt, len);
        break;
    case 6:
        pkt[dst ? 22 : 20] = (uint8_t)(port >> 8);
        pkt[dst ? 23 : 21] = (uint8_t)port;
        skip |= recalc_l4(pkt, len, csum_enable, 38, 36, 6);
        break;
    case 17:
        pkt[dst ? 22 : 20] = (uint8_t)(port >> 8);
        pkt[dst ? 23 : 21] = (uint8_t)port;
        skip |= recalc_l4(pkt, len, csum_enable, 28, 26, 17);
        break;
    }
    return skip;
}

/* DPDK 20.11 rte_raw_cksum: 16-bit words in host (little-endian) order, a trailing byte as
 * the low byte of a word, folded to 16 bits; returned in host order of the LE words. */
static uint16_t rte_raw_cksum_le(const uint8_t* p, size_t len) {
    uint32_t sum = 0;
    size_t i = 0;
    for (; i + 1 < len; i += 2) sum += (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8);
    if (len & 1) sum += p[i];
    while (sum >> 16) sum = (sum & 0xffff) + (sum >> 16);
    return (uint16_t)sum;
}

/* cgo/dpdk.c:333-365 with port_conf.txmode.offloads == 0. Returns HALO_TX_R_OVERRUN or 0. */
static uint8_t dpdk_tx_fill(uint8_t* frame, size_t L) {
    if (L < 14 || be16(frame + 12) != 0x0800) return 0;  /* ether_type != IPv4: untouched */
    if (L < 34) return HALO_TX_R_OVERRUN;                 /* the IPv4 header itself is cut */
    uint8_t* ip = frame + 14;
    uint8_t rc = 0;
    ip[10] = ip[11] = 0;                                   /* hdr_checksum = 0 */
    const size_t ihl4 = (size_t)(ip[0] & 0x0f) * 4;      /* rte_ipv4_hdr_len */
    if (14 + ihl4 <= L) {
        uint16_t c = (uint16_t)~rte_raw_cksum_le(ip, ihl4);  /* rte_ipv4_cksum */
        ip[10] = (uint8_t)c;                                 /* stored as a host-order u16 */
        ip[11] = (uint8_t)(c >> 8);
    } else {
        rc |= HALO_TX_R_OVERRUN;
    }
    const uint8_t proto = ip[9];
    size_t field;
    if (proto == 17) field = 20 + 6;       /* rte_udp_hdr.dgram_cksum at ipv4_hdr + 20 */
    else if (proto == 6) field = 20 + 16;  /* rte_tcp_hdr.cksum */
    else return rc;
    if (14 + field + 2 > L) return rc | HALO_TX_R_OVERRUN;
    ip[field] = ip[field + 1] = 0;
    const uint32_t l3_len = be16(ip + 2);
    if (l3_len < ihl4) return rc;          /* rte_ipv4_udptcp_cksum returns 0 */
    const uint32_t l4_len = l3_len - (uint32_t)ihl4;
    if (34 + (size_t)l4_len > L) return rc | HALO_TX_R_OVERRUN;
    uint32_t cksum = rte_raw_cksum_le(ip + 20, l4_len);
    uint8_t psd[12];                       /* rte_ipv4_phdr_cksum(ipv4_hdr, 0) */
    memcpy(psd, ip + 12, 8);
    psd[8] = 0;
    psd[9] = proto;
    psd[10] = (uint8_t)(l4_len >> 8);
    psd[11] = (uint8_t)l4_len;
    cksum += rte_raw_cksum_le(psd, 12);
    cksum = ((cksum & 0xffff0000u) >> 16) + (cksum & 0xffffu);
    cksum = (~cksum) & 0xffffu;
    if (cksum == 0 && proto == 17) cksum = 0xffff;
    ip[field] = (uint8_t)cksum;
    ip[field + 1] = (uint8_t)(cksum >> 8);
    return rc;
}

/* One frame, the steps of op->steps in the Ipv4RouteForward order. Returns HALO_TX_R_*. */
ORA_API uint8_t ora_tx_frame(uint8_t* frame, uint32_t L, const halo_tx_op_t* op, uint32_t flags) {
    const int en = (flags & HALO_RX_CSUM_ENABLE) != 0;
    const unsigned st = op->steps;
    uint8_t* pkt = frame + 14;
    const size_t len = L >= 14 ? L - 14 : 0;  /* pkt = frame[14:], engine/ipv4_engine.go:31-37 */
    int skip = 0;
    uint8_t r = 0;
    if (L < 14) {  /* no IPv4 packet at all: every Go step returns on its guard */
        if (st & (HALO_TX_NAT_DST | HALO_TX_TTL | HALO_TX_NAT_SRC | HALO_TX_RECALC)) r |= HALO_TX_R_SKIPPED;
        return r;  /* (and the TTL step, if set, ends the chain) */
    }
    if (st & HALO_TX_NAT_DST) skip |= nat_change(pkt, len, op->dst_ip, op->dst_port, 1, en);
    if (st & HALO_TX_TTL) {
        int alive = handle_ipv4_pkt_ttl(pkt, len, en, &skip);
        if (!alive) return skip ? HALO_TX_R_SKIPPED : 0;  /* TTL-exceeded branch, ipv4_engine.go:132-142 */
        r |= HALO_TX_R_TTL_ALIVE;
    }
    if (st & HALO_TX_NAT_SRC) skip |= nat_change(pkt, len, op->src_ip, op->src_port, 0, en);
    if (st & HALO_TX_RECALC) {
        skip |= recalc_ipv4(pkt, len, en);
        if (len >= 10) {
            switch (pkt[9]) {
            case 1: skip |= recalc_icmp(pkt, len); break;
            case 6: skip |= recalc_l4(pkt, len, en, 38, 36, 6); break;
            case 17: skip |= recalc_l4(pkt, len, en, 28, 26, 17); break;
            }
        }
    }
    if (skip) r |= HALO_TX_R_SKIPPED;
    if (st & HALO_TX_DPDK_FILL) r |= dpdk_tx_fill(frame, L);
    return r;
}

typedef struct {
    uint8_t* bytes;
    const uint32_t* offsets_dw;
    const uint16_t* lens;
    const halo_tx_op_t* ops;
    uint32_t flags;
    uint8_t* result;
    uint64_t first, last;
} tx_job_t;

static void* tx_job(void* arg) {
    tx_job_t* j = (tx_job_t*)arg;
    for (uint64_t i = j->first; i < j->last; ++i) {
        uint8_t r = ora_tx_frame(j->bytes + ((uint64_t)j->offsets_dw[i] << 2), j->lens[i], &j->ops[i], j->flags);
        if (j->result) j->result[i] = r;
    }
    return NULL;
}

/* In place, ragged dword offsets; threads <= 1 runs on the calling thread. */
ORA_API int ora_tx_batch(uint8_t* bytes, const uint32_t* offsets_dw, const uint16_t* lens, uint32_t n,
                         const halo_tx_op_t* ops, uint32_t flags, uint8_t* result, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    tx_job_t* jobs = (tx_job_t*)calloc((size_t)threads, sizeof(tx_job_t));
    pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !tid) { free(jobs); free(tid); return -1; }
    for (int t = 0; t < threads; ++t) {
        tx_job_t* j = &jobs[t];
        j->bytes = bytes; j->offsets_dw = offsets_dw; j->lens = lens; j->ops = ops; j->flags = flags;
        j->result = result;
        j->first = (uint64_t)n * t / threads;
        j->last = (uint64_t)n * (t + 1) / threads;
    }
    int rc = 0, started = 0;
    for (int t = 1; t < threads; ++t) {
        if (pthread_create(&tid[t], NULL, tx_job, &jobs[t]) != 0) { rc = -1; break; }
        started = t;
    }
    if (rc == 0) tx_job(&jobs[0]);
    for (int t = 1; t <= started; ++t) pthread_join(tid[t], NULL);
    free(jobs);
    free(tid);
    return rc;
}

/* ================================================================================================
 * The Build* half of row f2: locally originated packets, restated one Go function at a time
 * (TEST INFRASTRUCTURE ONLY; the product is halo_tx_build_batch_device in tx_build.hip).
 *   BuildUdpPkt   protocol/udp.go:52-91      BuildTcpPkt  protocol/tcp.go:73-123
 *   BuildIcmpPkt  protocol/icmp.go:66-89     BuildIpv4Pkt protocol/ipv4.go:89-131 (iphId, :33)
 *   BuildEthFrm   protocol/ethernet.go:58-82
 *   drivers       NetIf.TxUdp/TxTcp/TxIcmp (engine/{udp,tcp,icmp}_engine.go), TxIpv4
 *                 (engine/ipv4_engine.go:50-99: the LoChan copy for the NetIf's own address),
 *                 TxEthernet (engine/ethernet_engine.go:34-50)
 * Every Tx* driver passes an empty buffer (`make([]byte, 0, cap)`), so each Build* writes its
 * header at offset 0 of its own slice; `append` becomes a write at the running length.
 * ============================================================================================== */

/* protocol/udp.go:52-91. Returns the packet length, or -1 (payload len must <= 1472). */
static long build_udp(uint8_t* pkt, const uint8_t* payload, size_t plen, uint16_t src_port, uint16_t dst_port,
                      const uint8_t src[4], const uint8_t dst[4], int csum_enable) {
    if (plen > 1472) return -1;
    size_t n = 0;
    pkt[n++] = (uint8_t)(src_port >> 8); pkt[n++] = (uint8_t)src_port;
    pkt[n++] = (uint8_t)(dst_port >> 8); pkt[n++] = (uint8_t)dst_port;
    const uint16_t udp_len = (uint16_t)(plen + 8);
    pkt[n++] = (uint8_t)(udp_len >> 8); pkt[n++] = (uint8_t)udp_len;
    pkt[n++] = 0x00; pkt[n++] = 0x00;
    memcpy(pkt + n, payload, plen);
    n += plen;
    if (csum_enable) {
        uint8_t* sum_data = (uint8_t*)malloc(12 + n);  /* fakeHeader + pkt (:74-84) */
        memcpy(sum_data, src, 4);
        memcpy(sum_data + 4, dst, 4);
        sum_data[8] = 0x00; sum_data[9] = 0x11;
        sum_data[10] = (uint8_t)(udp_len >> 8); sum_data[11] = (uint8_t)udp_len;
        memcpy(sum_data + 12, pkt, n);
        const uint16_t sum = ora_get_checksum(sum_data, 12 + n);
        free(sum_data);
        pkt[6] = (uint8_t)(sum >> 8); pkt[7] = (uint8_t)sum;
    } else {
        pkt[6] = 0x00; pkt[7] = 0x00;
    }
    return (long)n;
}

/* protocol/tcp.go:73-123. Returns the packet length, or -1 (payload len must <= 1460). */
static long build_tcp(uint8_t* pkt, const uint8_t* payload, size_t plen, uint16_t src_port, uint16_t dst_port,
                      const uint8_t src[4], const uint8_t dst[4], uint32_t seq, uint32_t ack, uint8_t flags,
                      int csum_enable) {
    if (plen > 1460) return -1;
    size_t n = 0;
    pkt[n++] = (uint8_t)(src_port >> 8); pkt[n++] = (uint8_t)src_port;
    pkt[n++] = (uint8_t)(dst_port >> 8); pkt[n++] = (uint8_t)dst_port;
    pkt[n++] = (uint8_t)(seq >> 24); pkt[n++] = (uint8_t)(seq >> 16); pkt[n++] = (uint8_t)(seq >> 8); pkt[n++] = (uint8_t)seq;
    pkt[n++] = (uint8_t)(ack >> 24); pkt[n++] = (uint8_t)(ack >> 16); pkt[n++] = (uint8_t)(ack >> 8); pkt[n++] = (uint8_t)ack;
    pkt[n++] = 0x50; pkt[n++] = flags;       /* data offset 5 words + flags (:96) */
    pkt[n++] = 0x01; pkt[n++] = 0x00;        /* window 256 (:98) */
    pkt[n++] = 0x00; pkt[n++] = 0x00;        /* checksum */
    pkt[n++] = 0x00; pkt[n++] = 0x00;        /* urgent pointer */
    memcpy(pkt + n, payload, plen);
    n += plen;
    if (csum_enable) {
        const size_t total = 20 + plen;      /* totalLen (:113) */
        uint8_t* sum_data = (uint8_t*)malloc(12 + n);
        memcpy(sum_data, src, 4);
        memcpy(sum_data + 4, dst, 4);
        sum_data[8] = 0x00; sum_data[9] = 0x06;
        sum_data[10] = (uint8_t)(total >> 8); sum_data[11] = (uint8_t)total;
        memcpy(sum_data + 12, pkt, n);
        const uint16_t sum = ora_get_checksum(sum_data, 12 + n);
        free(sum_data);
        pkt[16] = (uint8_t)(sum >> 8); pkt[17] = (uint8_t)sum;
    } else {
        pkt[16] = 0x00; pkt[17] = 0x00;
    }
    return (long)n;
}

/* protocol/icmp.go:66-89 (icmpId: two bytes). Always checksummed. -1: payload len must <= 1472. */
static long build_icmp(uint8_t* pkt, const uint8_t* payload, size_t plen, uint8_t type, const uint8_t id[2],
                       uint16_t seq) {
    if (plen > 1472) return -1;
    size_t n = 0;
    pkt[n++] = type;
    pkt[n++] = 0x00;
    pkt[n++] = 0x00; pkt[n++] = 0x00;
    pkt[n++] = id[0]; pkt[n++] = id[1];
    pkt[n++] = (uint8_t)(seq >> 8); pkt[n++] = (uint8_t)seq;
    memcpy(pkt + n, payload, plen);
    n += plen;
    const uint16_t sum = ora_get_checksum(pkt, n);
    pkt[2] = (uint8_t)(sum >> 8); pkt[3] = (uint8_t)sum;
    return (long)n;
}

/* protocol/ipv4.go:89-131; *iph_id is the package global iphId (:33), incremented before use. */
static long build_ipv4(uint8_t* pkt, const uint8_t* payload, size_t plen, uint8_t proto, const uint8_t src[4],
                       const uint8_t dst[4], uint16_t* iph_id, int csum_enable) {
    if (plen > 1480) return -1;
    size_t n = 0;
    pkt[n++] = 0x45; pkt[n++] = 0x00;
    const uint16_t ip_len = (uint16_t)(plen + 20);
    pkt[n++] = (uint8_t)(ip_len >> 8); pkt[n++] = (uint8_t)ip_len;
    *iph_id = (uint16_t)(*iph_id + 1);
    pkt[n++] = (uint8_t)(*iph_id >> 8); pkt[n++] = (uint8_t)*iph_id;
    pkt[n++] = 0x00; pkt[n++] = 0x00;
    pkt[n++] = 0x80;
    pkt[n++] = proto;
    pkt[n++] = 0x00; pkt[n++] = 0x00;
    memcpy(pkt + n, src, 4); n += 4;
    memcpy(pkt + n, dst, 4); n += 4;
    if (csum_enable) {
        const uint16_t sum = ora_get_checksum(pkt, n);
        pkt[10] = (uint8_t)(sum >> 8); pkt[11] = (uint8_t)sum;
    } else {
        pkt[10] = 0x00; pkt[11] = 0x00;
    }
    memcpy(pkt + n, payload, plen);
    n += plen;
    return (long)n;
}

/* protocol/ethernet.go:58-82: dst, src, EtherType, payload, zero padding to 60. */
static long build_eth(uint8_t* frm, const uint8_t* payload, size_t plen, const uint8_t dst_mac[6],
                      const uint8_t src_mac[6], uint16_t eth_proto) {
    if (plen > 1500) return -1;
    size_t n = 0;
    memcpy(frm, dst_mac, 6); n += 6;
    memcpy(frm + n, src_mac, 6); n += 6;
    frm[n++] = (uint8_t)(eth_proto >> 8); frm[n++] = (uint8_t)eth_proto;
    memcpy(frm + n, payload, plen);
    n += plen;
    while (n < 60) frm[n++] = 0x00;
    return (long)n;
}

static void be32_put(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

/* One descriptor through Tx{Udp,Tcp,Icmp} -> TxIpv4 -> TxEthernet (or TxIpv4's LoChan copy).
 * Writes the frame into out[0 .. *out_len) and returns HALO_TX_B_*; `out` holds >= 1514 B. */
ORA_API uint8_t ora_tx_build_frame(const halo_tx_build_desc_t* d, const uint8_t* payload_base,
                                   const uint8_t src_mac[6], uint32_t flags, uint16_t* iph_id, uint8_t* out,
                                   uint16_t* out_len) {
    const int csum = (flags & HALO_RX_CSUM_ENABLE) != 0;
    const uint8_t* payload = payload_base + d->payload_off;
    uint8_t src[4], dst[4], l4[1514], ip[1514];
    be32_put(src, d->src_ip);
    be32_put(dst, d->dst_ip);
    long l4n;
    *out_len = 0;
    if (d->proto == 0x11) {
        l4n = build_udp(l4, payload, d->payload_len, d->src_port, d->dst_port, src, dst, csum);
    } else if (d->proto == 0x06) {
        l4n = build_tcp(l4, payload, d->payload_len, d->src_port, d->dst_port, src, dst, d->seq, d->ack, d->aux, csum);
    } else if (d->proto == 0x01) {
        const uint8_t id[2] = {(uint8_t)(d->src_port >> 8), (uint8_t)d->src_port};
        l4n = build_icmp(l4, payload, d->payload_len, d->aux, id, d->dst_port);
    } else {
        return HALO_TX_B_PROTO;
    }
    if (l4n < 0) return HALO_TX_B_PAYLOAD_LEN;
    const long ipn = build_ipv4(ip, l4, (size_t)l4n, d->proto, src, dst, iph_id, csum);
    if (ipn < 0) return HALO_TX_B_PAYLOAD_LEN; /* unreachable: every L4 limit keeps ipv4 payload <= 1480 */
    if (d->mode == HALO_TX_BUILD_LOOPBACK) {    /* engine/ipv4_engine.go:72-79: copy of ipv4Pkt */
        memcpy(out, ip, (size_t)ipn);
        *out_len = (uint16_t)ipn;
        return HALO_TX_B_OK;
    }
    const long fn = build_eth(out, ip, (size_t)ipn, d->dst_mac, src_mac, 0x0800);
    *out_len = (uint16_t)fn;
    return HALO_TX_B_OK;
}

/* Serial batch in descriptor order (iphId is a sequence): frames into slots of out_stride bytes.
 * A frame longer than its slot (build-defined; Go has no slots) gets HALO_TX_B_SLOT and is
 * refused before Build* runs: no iphId step, nothing stored. */
ORA_API int ora_tx_build_batch(const halo_tx_build_desc_t* desc, uint32_t n, const uint8_t* payload, uint32_t flags,
                               const uint8_t src_mac[6], uint8_t* frames, uint32_t out_stride, uint16_t* out_lens,
                               uint8_t* result, uint16_t* iph_id) {
    uint8_t tmp[1514];
    for (uint32_t i = 0; i < n; ++i) {
        const halo_tx_build_desc_t* d = &desc[i];
        /* the slot check needs only the descriptor: frame length from the Build* arithmetic */
        const uint32_t l4 = (d->proto == 0x06 ? 20u : 8u) + d->payload_len;
        const uint32_t fl = d->mode == HALO_TX_BUILD_LOOPBACK ? 20u + l4 : (34u + l4 < 60u ? 60u : 34u + l4);
        uint16_t len = 0;
        uint8_t r;
        const int known = d->proto == 0x11 || d->proto == 0x06 || d->proto == 0x01;
        const uint32_t lim = d->proto == 0x06 ? 1460u : 1472u;
        if (known && d->payload_len <= lim && fl > out_stride) {
            r = HALO_TX_B_SLOT; /* refused before Build*: no iphId step */
        } else {
            r = ora_tx_build_frame(d, payload, src_mac, flags, iph_id, tmp, &len);
            if (r == HALO_TX_B_OK) memcpy(frames + (uint64_t)i * out_stride, tmp, len);
        }
        if (out_lens) out_lens[i] = r == HALO_TX_B_OK ? len : 0;
        if (result) result[i] = r;
    }
    return 0;
}

/* ================================================================================================
 * IcmpTtlDeepNat (engine/icmp_engine.go:55-86): called by Ipv4RouteForward on the received
 * frame's Ethernet payload before its own DNAT (engine/ipv4_engine.go:111-130). ParseIpv4Pkt ->
 * ICMP only -> ParseIcmpPkt -> ICMP_TTL only -> quote (icmpPayload) of at least 28 bytes ->
 * NatGetFlowByWan(quoted dst, its dst port, quoted src, its src port, quoted proto) -> when a
 * flow exists: NatChangeSrc(icmpPayload, LanHost) and NatChangeDst(ethPayload, LanHost, 0).
 * ParseIpv4Pkt and ParseIcmpPkt are the rx restatement's (ora_rx_frame with HALO_RX_L3_START on
 * the Ethernet payload); the NAT table is the caller's: `found` / lan_ip / lan_port are what the
 * lookup returned. */
ORA_API void ora_rx_frame(const uint8_t* frame, uint32_t len, uint32_t flags, const halo_rx_netif_t* netif,
                          halo_rx_result_t* r);

/* The checks up to the lookup, as a record: status (OK, the failing rx status, IP_PROTO = not
 * ICMP, ICMP_TYPE = not ICMP_TTL, L4_LEN = quote < 28 B), ip_proto = the quoted protocol and the
 * lookup's arguments in received-packet orientation: src_ip/sport = the quoted packet's
 * destination (the remote end), dst_ip/dport = its source (the WAN side) — so a NAT_WAN flow key
 * of the record is NatGetFlowByWan's key. */
ORA_API void ora_icmp_quote(const uint8_t* frame, uint32_t L, uint32_t flags, halo_rx_result_t* q) {
    memset(q, 0, sizeof *q);
    q->ethertype = 0x0800;
    q->ip_proto = 0xff;
    if (L < 14) { q->status = HALO_RX_ETH_LEN; return; }
    const uint8_t* pkt = frame + 14;
    halo_rx_netif_t nif;
    memset(&nif, 0, sizeof nif);
    halo_rx_result_t r;
    ora_rx_frame(pkt, L - 14, (flags & HALO_RX_CSUM_ENABLE) | HALO_RX_L3_START, &nif, &r);
    if (r.status >= HALO_RX_IP_LEN && r.status <= HALO_RX_IP_TOTLEN_OVERRUN) { q->status = r.status; return; }
    if (r.ip_proto != 0x01) { q->status = HALO_RX_IP_PROTO; return; }
    if (r.status != HALO_RX_OK) { q->status = r.status; return; }  /* ParseIcmpPkt failed */
    if (r.l4_aux != 0x0b) { q->status = HALO_RX_ICMP_TYPE; return; }
    const uint8_t* ic = pkt + 28;          /* icmpPayload = ipv4Payload[8:] */
    const uint32_t ilen = r.payload_len;   /* totalLen - 28 */
    if (ilen < 28) { q->status = HALO_RX_L4_LEN; return; }
    q->ip_proto = ic[9];
    q->src_ip = ((uint32_t)ic[16] << 24) | ((uint32_t)ic[17] << 16) | ((uint32_t)ic[18] << 8) | ic[19];
    q->dst_ip = ((uint32_t)ic[12] << 24) | ((uint32_t)ic[13] << 16) | ((uint32_t)ic[14] << 8) | ic[15];
    uint16_t wan_port = 0, remote_port = 0;  /* NatGetSrcDstPort(icmpPayload), ipv4.go:229-246 */
    switch (ic[9]) {
        case 0x01: wan_port = remote_port = be16(ic + 24); break;
        case 0x06:
        case 0x11: wan_port = be16(ic + 20); remote_port = be16(ic + 22); break;
        default: break;
    }
    q->sport = remote_port;
    q->dport = wan_port;
}

/* In place; returns isIcmpTtl. */
ORA_API int ora_icmp_deep_nat(uint8_t* frame, uint32_t L, uint32_t flags, uint32_t lan_ip, uint16_t lan_port,
                              int found) {
    halo_rx_result_t q;
    ora_icmp_quote(frame, L, flags, &q);
    if (q.status != HALO_RX_OK || !found) return 0;
    const int en = (flags & HALO_RX_CSUM_ENABLE) != 0;
    uint8_t* pkt = frame + 14;
    const uint32_t total_len = be16(pkt + 2);
    nat_change(pkt + 28, total_len - 28, lan_ip, lan_port, 0, en); /* NatChangeSrc(icmpPayload, ...) */
    nat_change(pkt, L - 14, lan_ip, 0, 1, en);                      /* NatChangeDst(ethPayload, ..., 0) */
    return 1;
}
