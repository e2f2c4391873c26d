package gpurx

// #include "gpurx_shim.h"
import "C"

import (
	"encoding/binary"
	"errors"
	"sync"
	"unsafe"

	"github.com/flswld/halo/protocol"
)

// Single-frame Parse* with the reference's signatures and results (protocol/{ethernet,ipv4,udp,
// tcp,icmp}.go), for callers that hold one frame or packet at a time: an Ipv4PktFwdHook
// (engine/engine.go:132, example/example.go:162-168) or code written against package protocol.
// Each frame goes through the GPU as a batch of one on a package-level context (Device) whose
// resident consumer serves it: ~7.6 us per frame (DESIGN.md §13.1), against ~22 ns for the one-core
// C port of the reference's own parse — a GPU round trip per packet is ~350x slower than parsing it
// on the calling core. These wrappers exist for ported code that needs the reference's signatures;
// a forward hook that parses every forwarded packet belongs on Ctx.ParseFramesBatch over batches of
// a few hundred frames or more (the crossover, §13.1), or on ParseFramesCPU (cpu.go), which gives
// the same Results on the calling core. These wrappers never switch to the CPU by themselves.
// protocol.CheckSumEnable is read at every call, as the reference reads it.

// Device is the GPU the single-frame wrappers use (set before the first call).
var Device = 0

// SingleFrameCPU, when set, makes the single-frame wrappers parse on the calling core through the
// CPU entry point (ParseFramesCPU: the same Result, ~30 ns instead of a ~7.6 us GPU round trip). It
// is the caller's choice, read at every call; the default keeps them on the GPU.
var SingleFrameCPU = false

var (
	oneMu  sync.Mutex
	oneCtx *Ctx
)

func parseOne(buf []byte, l3 bool) (Result, error) {
	if SingleFrameCPU {
		return parseOneCPU(buf, l3)
	}
	oneMu.Lock()
	defer oneMu.Unlock()
	if oneCtx == nil {
		x, err := NewCtx(Device)
		if err != nil {
			return Result{}, err
		}
		// one frame per call: served by the resident consumer (~8 us, no launch or synchronisation)
		if err := x.SetResident(64, 1<<16); err != nil {
			x.Close()
			return Result{}, err
		}
		oneCtx = x
	}
	n := len(buf)
	if n > 0xFFFF { // every length past the caps gets the same ETH_LEN / IP_LEN verdict
		n = 0xFFFF
	}
	var empty [4]byte
	p := &empty[0]
	if n > 0 {
		p = &buf[0]
	}
	csum, l := C.int(0), C.int(0)
	if protocol.CheckSumEnable {
		csum = 1
	}
	if l3 {
		l = 1
	}
	var r Result
	rc := C.gpurx_parse_one(oneCtx.c, (*C.uint8_t)(unsafe.Pointer(p)), C.uint16_t(n), csum, l,
		(*C.halo_rx_result_t)(unsafe.Pointer(&r)))
	return r, halo(rc)
}

// ParseEthFrm is protocol.ParseEthFrm (protocol/ethernet.go:29-55).
func ParseEthFrm(frm []byte) (payload []byte, dstMac []byte, srcMac []byte, ethProto uint16, err error) {
	r, e := parseOne(frm, false)
	if e != nil {
		return nil, nil, nil, protocol.ETH_PROTO_UNKNOWN, e
	}
	if r.Status == StatusEthLen || r.Status == StatusEthType {
		return nil, nil, nil, protocol.ETH_PROTO_UNKNOWN, r.Err()
	}
	return frm[14:], frm[0:6], frm[6:12], r.EthProto, nil
}

// ParseIpv4Pkt is protocol.ParseIpv4Pkt (protocol/ipv4.go:48-86). For a totalLen outside
// [20, len(pkt)] it evaluates the reference's own slice expression pkt[20:totalLen], so it panics
// or returns the bytes past len(pkt) exactly where the reference does.
func ParseIpv4Pkt(pkt []byte) (payload []byte, ipHeadProto uint8, srcAddr []byte, dstAddr []byte, err error) {
	r, e := parseOne(pkt, true)
	if e != nil {
		return nil, protocol.IPH_PROTO_UNKNOWN, nil, nil, e
	}
	switch r.Status {
	case StatusIpLen, StatusIpVer, StatusIpFrag, StatusIpProto, StatusIpHdrCksum:
		return nil, protocol.IPH_PROTO_UNKNOWN, nil, nil, r.Err()
	case StatusIpTotLenUnderflow, StatusIpTotLenOverrun:
		totalLen := int(binary.BigEndian.Uint16(pkt[2:4]))
		return pkt[20:totalLen], pkt[9], pkt[12:16], pkt[16:20], nil
	}
	return pkt[20:r.IpTotalLen], r.IpHeadProto, pkt[12:16], pkt[16:20], nil
}

// ipWrap puts seg behind a minimal valid IPv4 header (0x45, DF, the protocol, the addresses, the
// header checksum) so that the L3 parse hands exactly seg to the L4 parser: pkt[20:totalLen] = seg
// and the pseudo header carries src / dst. Only the verdicts for seg are read back.
func ipWrap(seg []byte, proto uint8, src, dst []byte) []byte {
	pkt := make([]byte, 20, 20+len(seg))
	pkt[0], pkt[6], pkt[8], pkt[9] = 0x45, 0x40, 64, proto
	binary.BigEndian.PutUint16(pkt[2:4], uint16(20+len(seg)))
	copy(pkt[12:16], src)
	copy(pkt[16:20], dst)
	s := uint32(0)
	for k := 0; k < 20; k += 2 {
		s += uint32(binary.BigEndian.Uint16(pkt[k : k+2]))
	}
	for s>>16 != 0 {
		s = s&0xFFFF + s>>16
	}
	binary.BigEndian.PutUint16(pkt[10:12], ^uint16(s))
	return append(pkt, seg...)
}

var errAddr = errors.New("gpurx: srcAddr and dstAddr must be 4-byte IPv4 addresses")

// l4 parses seg as protocol `proto` and returns its record and the reference's error for it.
func l4(seg []byte, proto uint8, src, dst []byte) (Result, error) {
	if len(src) != 4 || len(dst) != 4 {
		return Result{}, errAddr
	}
	r, e := parseOne(ipWrap(seg, proto, src, dst), true)
	if e != nil {
		return r, e
	}
	switch r.Status {
	case StatusOK:
		return r, nil
	case StatusIpLen, StatusL4Len: // IpLen: 20 + len(seg) > 1500, i.e. len(seg) > 1480
		return r, errors.New(ErrorText(StatusL4Len, proto))
	}
	return r, errors.New(ErrorText(r.Status, proto))
}

// ParseUdpPkt is protocol.ParseUdpPkt (protocol/udp.go:21-49).
func ParseUdpPkt(pkt []byte, srcAddr []byte, dstAddr []byte) (payload []byte, srcPort uint16, dstPort uint16, err error) {
	r, e := l4(pkt, protocol.IPH_PROTO_UDP, srcAddr, dstAddr)
	if e != nil {
		return nil, 0, 0, e
	}
	return pkt[8:], r.SrcPort, r.DstPort, nil
}

// ParseTcpPkt is protocol.ParseTcpPkt (protocol/tcp.go:36-70); the payload starts at the
// data-offset nibble used as BYTES, as tcp.go:49,68 does.
func ParseTcpPkt(pkt []byte, srcAddr []byte, dstAddr []byte) (payload []byte, srcPort uint16, dstPort uint16,
	seqNum uint32, ackNum uint32, flags uint8, err error) {
	r, e := l4(pkt, protocol.IPH_PROTO_TCP, srcAddr, dstAddr)
	if e != nil {
		return nil, 0, 0, 0, 0, 0, e
	}
	return pkt[r.PayloadOff-20:], r.SrcPort, r.DstPort, r.Seq, r.Ack, r.L4Aux, nil
}

// ParseIcmpPkt is protocol.ParseIcmpPkt (protocol/icmp.go:33-63); the checksum is always verified.
func ParseIcmpPkt(pkt []byte) (payload []byte, icmpType uint8, icmpId []byte, icmpSeq uint16, err error) {
	zero := []byte{0, 0, 0, 0}
	r, e := l4(pkt, protocol.IPH_PROTO_ICMP, zero, zero)
	if e != nil {
		return nil, protocol.ICMP_UNKNOWN, nil, 0, e
	}
	return pkt[8:], r.L4Aux, pkt[4:6], uint16(r.Seq), nil
}
