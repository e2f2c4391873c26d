package gpurx

// #include "gpurx_shim.h"
import "C"

import "unsafe"

// The forward and transmit calls (SURVEY.md §8f rows f2-f4) a batched Ipv4RouteForward /
// Tx* would make, on device-resident batches: frames, offsets (u32 dwords), lengths and records in
// HBM, addressed by device pointers. All are asynchronous on the null stream.

// RouteBatch is NetIf.FindRoute -> RouteTable.FindRoute (engine/ipv4_engine.go:351-390) for every
// record's destination: ids index the RouteEntry objects registered with halo_route_update in
// RouteTable.AddRoute order (HALO_ROUTE_NONE / HALO_ROUTE_PANIC as FindRoute's nil / div-by-zero).
func RouteBatch(t *C.halo_route_table_t, dRecords unsafe.Pointer, n int, dIds unsafe.Pointer) error {
	return halo(C.halo_route_lookup_records_device(t, (*C.halo_rx_result_t)(dRecords), C.uint32_t(n),
		(*C.uint32_t)(dIds), nil))
}

// NatKeys is NatWanFlowHash.GetHashCode with NatGetFlowByWan's key normalisation
// (engine/ipv4_engine.go:471-479, :554-581) for every record, and its bucket in a table of nb
// buckets (hashmap/hashmap.go:64), so the Go side probes buckets without hashing.
func NatKeys(dRecords unsafe.Pointer, n int, natType int, dHash, dBucket unsafe.Pointer, nb uint32) error {
	return halo(C.halo_flow_hash_device((*C.halo_rx_result_t)(dRecords), C.uint32_t(n), C.HALO_FLOW_NAT_WAN,
		C.uint32_t(natType), (*C.uint64_t)(dHash), C.uint32_t(nb), (*C.uint32_t)(dBucket), nil))
}

// ParseWithNatKeys is the receive parse and NatKeys in one pass over the frames (records equal to
// the plain parse's; the keys are hashed before the records leave registers).
func ParseWithNatKeys(dFrames, dOffsets, dLens unsafe.Pointer, n int, netif *NetIfCfg, dOut, dHash, dBucket unsafe.Pointer,
	natType int, nb uint32) error {
	nif, err := netif.c()
	if err != nil {
		return err
	}
	return halo(C.halo_rx_parse_flow_batch_device((*C.uint8_t)(dFrames), (*C.uint32_t)(dOffsets),
		(*C.uint16_t)(dLens), C.uint32_t(n), csumFlag(), &nif, 0, (*C.halo_rx_result_t)(dOut), nil,
		C.HALO_FLOW_NAT_WAN, C.uint32_t(natType), (*C.uint64_t)(dHash), C.uint32_t(nb), (*C.uint32_t)(dBucket), nil))
}

// Rewrite is NatChangeDst / HandleIpv4PktTtl / NatChangeSrc / ReCalc* and eth_tx's checksum fill
// (protocol/ipv4.go:134-302, cgo/dpdk.c:333-365) for every frame, in place, in Ipv4RouteForward's
// order; dOps holds one halo_tx_op_t per frame (the addresses and ports the NAT tables resolved).
func Rewrite(dFrames, dOffsets, dLens, dOps, dResult unsafe.Pointer, n int, maxLen uint32) error {
	return halo(C.halo_tx_fixup_batch_device((*C.uint8_t)(dFrames), (*C.uint32_t)(dOffsets), (*C.uint16_t)(dLens),
		C.uint32_t(n), (*C.halo_tx_op_t)(dOps), csumFlag(), C.uint32_t(maxLen), (*C.uint8_t)(dResult), nil))
}

// BuildBatch is TxUdp / TxTcp / TxIcmp -> TxIpv4 -> TxEthernet for n descriptors
// (halo_tx_build_desc_t); iphId lives in device memory (dIphId, u16) and advances by the number
// of packets built, in descriptor order (protocol/ipv4.go:33,89-131).
func BuildBatch(dDesc unsafe.Pointer, n int, dPayload unsafe.Pointer, srcMac []byte, dFrames unsafe.Pointer,
	stride int, dLens, dResult, dIphId, dWs unsafe.Pointer, wsBytes uint64, maxPayload uint32) error {
	netif := NetIfCfg{MacAddr: srcMac, IpAddr: []byte{0, 0, 0, 0}}
	nif, err := netif.c()
	if err != nil {
		return err
	}
	return halo(C.halo_tx_build_batch_device((*C.halo_tx_build_desc_t)(dDesc), C.uint32_t(n), (*C.uint8_t)(dPayload),
		csumFlag(), &nif, C.uint32_t(maxPayload), (*C.uint8_t)(dFrames), C.uint32_t(stride), (*C.uint16_t)(dLens),
		(*C.uint8_t)(dResult), (*C.uint16_t)(dIphId), dWs, C.uint64_t(wsBytes), nil))
}

// BuildWorkspace is the device scratch BuildBatch needs for n descriptors.
func BuildWorkspace(n int) uint64 { return uint64(C.halo_tx_build_workspace(C.uint32_t(n))) }

// DeepNat is IcmpTtlDeepNat (engine/icmp_engine.go:55-86) for a batch: with dNat == nil it writes
// the quote records (NatGetFlowByWan's arguments; hash them with NatKeys), then, called again with
// the lookups' results, rewrites the frames in place.
func DeepNat(dFrames, dOffsets, dLens, dNat, dQuote, dApplied unsafe.Pointer, n int) error {
	return halo(C.halo_tx_icmp_deep_nat_batch_device((*C.uint8_t)(dFrames), (*C.uint32_t)(dOffsets),
		(*C.uint16_t)(dLens), C.uint32_t(n), (*C.halo_tx_deep_nat_t)(dNat), csumFlag(),
		(*C.halo_rx_result_t)(dQuote), (*C.uint8_t)(dApplied), nil))
}
