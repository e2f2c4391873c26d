package gpurx

// #include "gpurx_shim.h"
import "C"

import (
	"errors"
	"unsafe"
)

// RingRx is a GPU consumer of one of halo's SPSC packet rings (mem.RingBuffer = ring_buffer_t,
// mem/ring_buffer.go:18-26, cgo/ring_buffer.h:20-55): the C lcore keeps producing exactly as
// before (cgo/dpdk.c:280-307); one Poll replaces every ReadPacket + RxEthernet between the
// consumer's tail and the producer's head, and the frames stay in the ring until Commit.
type RingRx struct{ r *C.halo_rx_ring_t }

// AttachRing replaces mem.NewRingBufferConsumer(rb, offset) (mem/ring_buffer.go:226-246).
// capacity is ReadPacket's len(data): 1514 for the DPDK driver (dpdk/dpdk.go:139) and
// engine.Wire. The ring is registered for DMA (it must start on a page boundary; DPDK's hugepage
// rings do).
func AttachRing(device int, rb unsafe.Pointer, offset int64, capacity uint32) (*RingRx, error) {
	return attachRing(device, rb, offset, capacity, C.HALO_RING_REGISTER)
}

// AttachRingResident is AttachRing with a resident consumer kernel (HALO_RING_PERSISTENT): polls
// of up to 16384 frames (engine.Wire's 1k-frame PacketHandle batches) are served without a kernel
// launch or stream synchronisation (~11 us instead of ~19 us per 1k frames, DESIGN.md §12.5).
// The kernel exits after 20 ms without a poll and is relaunched by the next one.
func AttachRingResident(device int, rb unsafe.Pointer, offset int64, capacity uint32) (*RingRx, error) {
	return attachRing(device, rb, offset, capacity, C.HALO_RING_REGISTER|C.HALO_RING_PERSISTENT)
}

func attachRing(device int, rb unsafe.Pointer, offset int64, capacity uint32, flags C.uint32_t) (*RingRx, error) {
	var r *C.halo_rx_ring_t
	if err := halo(C.halo_rx_ring_attach(C.int(device), rb, C.int64_t(offset), C.uint32_t(capacity), 0, 0,
		flags, &r)); err != nil {
		return nil, err
	}
	return &RingRx{r}, nil
}

// Poll parses every frame repeated ReadPacket calls would return now; pos[i] is frame i's record
// position in the ring stream (its bytes start 4 bytes later, modulo the ring size). out and pos
// must hold the attach's max_frames entries (default: ring size / 8).
func (x *RingRx) Poll(netif *NetIfCfg, out []Result, pos []uint64) (int, error) {
	if len(out) == 0 || len(pos) < len(out) {
		return 0, errors.New("gpurx: empty result or position slice")
	}
	nif, err := netif.c()
	if err != nil {
		return 0, err
	}
	var info C.halo_rx_ring_scan_t
	if err := halo(C.halo_rx_ring_poll(x.r, csumFlag(), &nif, (*C.halo_rx_result_t)(unsafe.Pointer(&out[0])), nil,
		(*C.uint64_t)(unsafe.Pointer(&pos[0])), &info)); err != nil {
		return 0, err
	}
	return int(info.n_frames), nil
}

// Commit hands the polled records back to the producer (ReadPacket's tail store).
func (x *RingRx) Commit() error { return halo(C.halo_rx_ring_commit(x.r)) }

// RingStats mirrors halo_rx_ring_stats_t as a Go type callers outside this package can name (cgo
// types are private to the package that declares them).
type RingStats struct {
	Polls           uint64 // polls that found records
	Frames          uint64 // frames returned
	SmallPolls      uint64 // polls on the small path (one launch, or a resident request)
	ServiceRequests uint64 // small polls served by the resident consumer
	ServiceLaunches uint64 // resident consumer launches (first use, after idle exits and device drains)
	WalkNs          uint64 // small polls: the host's ReadPacket walk of the length fields
	WaitNs          uint64 // small polls: launch + synchronisation, or request to completion
	ServiceGpuNs    uint64 // resident consumer: GPU time per request, summed
}

// Stats reports the consumer's poll counters and where small polls spent their time
// (halo_rx_ring_get_stats).
func (x *RingRx) Stats() (RingStats, error) {
	var st C.halo_rx_ring_stats_t
	if err := halo(C.halo_rx_ring_get_stats(x.r, &st)); err != nil {
		return RingStats{}, err
	}
	return RingStats{Polls: uint64(st.polls), Frames: uint64(st.frames), SmallPolls: uint64(st.small_polls),
		ServiceRequests: uint64(st.service_requests), ServiceLaunches: uint64(st.service_launches),
		WalkNs: uint64(st.walk_ns), WaitNs: uint64(st.wait_ns), ServiceGpuNs: uint64(st.service_gpu_ns)}, nil
}

// Detach synchronises and frees the consumer (the ring memory must outlive it).
func (x *RingRx) Detach() error { return halo(C.halo_rx_ring_detach(x.r)) }
