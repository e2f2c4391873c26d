package gpurx

/*
#cgo LDFLAGS: -L${SRCDIR}/../../halo_amd/lib -lhalo_rx_cpu
#include "gpurx_shim.h"
#include "halo_rx_cpu.h"
*/
import "C"

import (
	"errors"
	"unsafe"
)

// ParseFramesCPU is ParseFramesBatch on the calling core (halo_rx_parse_batch_cpu,
// include/halo_rx_cpu.h, libhalo_rx_cpu.so): the same Results, bit for bit, with no GPU round
// trip. It is the explicit choice for a poll below the crossover where a GPU call costs more than
// the frames (INTEGRATION.md §1a: a few hundred 64 B frames); it is never taken behind the caller's
// back, and the GPU entry points still fail without a device. l3 parses bare IPv4 packets (a NetIf's
// LoChan, as ParsePacketsL3). Offsets may have any alignment; no state, safe from any goroutine.
func ParseFramesCPU(buf []byte, off []uint64, lens []uint16, netif *NetIfCfg, l3 bool, out []Result) error {
	if len(off) != len(lens) || len(out) < len(lens) {
		return errors.New("gpurx: offsets, lengths and results disagree")
	}
	if len(lens) == 0 {
		return nil
	}
	for i, o := range off {
		if o+uint64(lens[i]) > uint64(len(buf)) {
			return errors.New("gpurx: a frame reaches past the end of buf")
		}
	}
	if len(buf) == 0 {
		buf = make([]byte, 4) // every frame is empty: any valid address will do
	}
	n, err := netif.c()
	if err != nil {
		return err
	}
	flags := csumFlag()
	if l3 {
		flags |= C.HALO_RX_L3_START
	}
	return halo(C.halo_rx_parse_batch_cpu((*C.uint8_t)(unsafe.Pointer(&buf[0])), (*C.uint64_t)(unsafe.Pointer(&off[0])),
		(*C.uint16_t)(unsafe.Pointer(&lens[0])), C.uint32_t(len(lens)), flags, &n,
		(*C.halo_rx_result_t)(unsafe.Pointer(&out[0])), nil))
}

// ParseBatchCPU is Ctx.ParseBatch on the calling core: every frame of b through ParseFramesCPU
// (l3: bare IPv4 packets), then Dispatch / DispatchLoopback into b.Res and b.Act.
func ParseBatchCPU(b *Batch, netif *NetIfCfg, l3 bool) error {
	n := b.Len()
	if err := ParseFramesCPU(b.Buf, b.Off, b.Lens, netif, l3, b.Res[:n]); err != nil {
		return err
	}
	return dispatch(l3, b.Res[:n], netif, b.Act[:n])
}

// parseOneCPU is parseOne (parse.go) on the calling core: one frame, or one bare IPv4 packet when
// l3, with no NetIf (the Parse* wrappers read no dispatch flag). Lengths past 65535 are capped as
// parseOne caps them: every such length gets the same ETH_LEN / IP_LEN verdict.
func parseOneCPU(buf []byte, l3 bool) (Result, error) {
	n := len(buf)
	if n > 0xFFFF {
		n = 0xFFFF
	}
	var r [1]Result
	netif := &NetIfCfg{MacAddr: make([]byte, 6), IpAddr: make([]byte, 4)}
	err := ParseFramesCPU(buf[:n], []uint64{0}, []uint16{uint16(n)}, netif, l3, r[:])
	return r[0], err
}
