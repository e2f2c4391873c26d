/*
 * gpurx_shim.h — the C side of package gpurx's cgo preamble (included by gpurx.go and parse.go;
 * static inline, so each cgo file gets its own copy). Compiled and run against include/halo_rx.h
 * and libhalo_rx.so by tests/test_go_binding.py, since this image has no Go toolchain.
 */
#ifndef GPURX_SHIM_H
#define GPURX_SHIM_H
#include <stddef.h>
#include <string.h>

#include "halo_rx.h"

// The Go mirrors below must keep these layouts.
_Static_assert(sizeof(halo_rx_result_t) == 32, "halo_rx_result_t is 32 bytes");
_Static_assert(offsetof(halo_rx_result_t, src_ip) == 8, "halo_rx_result_t.src_ip");
_Static_assert(offsetof(halo_rx_result_t, payload_off) == 20, "halo_rx_result_t.payload_off");
_Static_assert(offsetof(halo_rx_result_t, l4_ack) == 28, "halo_rx_result_t.l4_ack");
_Static_assert(sizeof(halo_rx_netif_t) == 16, "halo_rx_netif_t is 16 bytes");

// gpurx_netif: a halo_rx_netif_t from NetIf.MacAddr, IpAddrToU(NetIf.IpAddr), NatEnable.
static inline halo_rx_netif_t gpurx_netif(const uint8_t* mac, uint32_t ip, int nat_enable) {
    halo_rx_netif_t n;
    memset(&n, 0, sizeof n);
    memcpy(n.mac, mac, 6);
    n.ip = ip;
    n.nat_enable = nat_enable ? 1u : 0u;
    return n;
}

// gpurx_parse_one: one frame (l3 = 0) or one bare IPv4 packet (l3 = 1) through the host entry
// point, as a batch of one. The netif only sets the dispatch flags, which the Parse* wrappers
// do not read.
static inline int gpurx_parse_one(halo_rx_host_ctx_t* ctx, const uint8_t* buf, uint16_t len, int csum, int l3,
                                  halo_rx_result_t* out) {
    const uint64_t off = 0;
    const uint8_t mac[6] = {0, 0, 0, 0, 0, 0};
    const halo_rx_netif_t n = gpurx_netif(mac, 0, 0);
    const uint32_t flags = (csum ? HALO_RX_CSUM_ENABLE : 0u) | (l3 ? HALO_RX_L3_START : 0u);
    return halo_rx_parse_batch_host(ctx, buf, &off, &len, 1, flags, &n, out, NULL);
}

#endif /* GPURX_SHIM_H */
