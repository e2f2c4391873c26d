// Package gpurx batches halo's receive parse + checksum (protocol.ParseEthFrm -> ParseIpv4Pkt ->
// ParseUdpPkt / ParseTcpPkt / ParseIcmpPkt with protocol.CheckSumEnable, and the branch inputs of
// engine.RxEthernet / RxIpv4) onto an MI355X GPU through the C ABI of include/halo_rx.h, which
// libhalo_rx.so implements with hand-written gfx950 kernels.
//
// It sits next to halo's only other cgo package, dpdk (dpdk/dpdk.go), and follows its rules: C
// never keeps a Go pointer past a call, and the slices handed to C hold no Go pointers.
//
//   - Ctx.ParseFramesBatch / ParsePacketsL3: one call per batch of frames (or LoChan packets).
//   - Dispatch / DispatchLoopback: the engine's per-frame decision over the records.
//   - parse.go: ParseEthFrm / ParseIpv4Pkt / ParseUdpPkt / ParseTcpPkt / ParseIcmpPkt with the
//     reference's signatures, for one frame at a time (an Ipv4PktFwdHook, ported code).
//   - ../engine/packet_handle_batched.go: the batched NetIf.PacketHandle built on these.
//
// The Go toolchain is absent from the image this was written in; tests/test_go_binding.py
// compiles and runs the C side of the preamble against halo_rx.h and libhalo_rx.so, and checks
// that every C name and every gpurx name the Go files use is defined.
package gpurx

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../halo_amd/lib -lhalo_rx -Wl,-rpath,${SRCDIR}/../../halo_amd/lib
#include "gpurx_shim.h"
*/
import "C"

import (
	"errors"
	"sync"
	"unsafe"

	"github.com/flswld/halo/protocol"
)

// Result mirrors halo_rx_result_t (32 bytes, little-endian, no Go pointers): the return values
// of ParseEthFrm / ParseIpv4Pkt / Parse{Udp,Tcp,Icmp}Pkt / NatGetSrcDstPort for one frame, each
// filled only when its layer succeeded; payload slices are (PayloadOff, PayloadLen) into the frame.
type Result struct {
	Status      uint8
	Flags       uint8
	EthProto    uint16
	IpHeadProto uint8
	L4Aux       uint8 // TCP flags or ICMP type
	IpTotalLen  uint16
	SrcAddr     uint32 // protocol.IpAddrToU form
	DstAddr     uint32
	SrcPort     uint16 // NatGetSrcDstPort; ICMP: the echo id twice
	DstPort     uint16
	PayloadOff  uint16
	PayloadLen  uint16
	Seq         uint32 // TCP seqNum, or ICMP id<<16 | seq
	Ack         uint32
}

var _ [32]byte = [unsafe.Sizeof(Result{})]byte{}

// Record status: the first failing check in reference order (halo_rx_status_t).
const (
	StatusOK                = 0
	StatusEthLen            = 1  // ethernet.go:31
	StatusEthType           = 2  // ethernet.go:39-50
	StatusIpLen             = 3  // ipv4.go:49
	StatusIpVer             = 4  // ipv4.go:52
	StatusIpFrag            = 5  // ipv4.go:59
	StatusIpProto           = 6  // ipv4.go:63-72
	StatusIpHdrCksum        = 7  // ipv4.go:74-78
	StatusIpTotLenUnderflow = 8  // ipv4.go:84: Go panics (slice bounds)
	StatusIpTotLenOverrun   = 9  // ipv4.go:84: Go reads stale bytes or panics
	StatusL4Len             = 10 // udp.go:22 / tcp.go:37 / icmp.go:34
	StatusIcmpType          = 11 // icmp.go:38-47
	StatusIcmpCode          = 12 // icmp.go:49
	StatusL4Cksum           = 13 // udp.go:42 / tcp.go:63 / icmp.go:53
)

// Record flags: what RxEthernet / RxIpv4 branch on.
const (
	FlagMacMatch = 0x01 // engine/ethernet_engine.go:22
	FlagIpBcast  = 0x02 // engine/ipv4_engine.go:24
	FlagDstIsOwn = 0x04 // engine/ipv4_engine.go:31
)

// Engine actions (halo_rx_action_t): the branch the reference engine takes for a record.
const (
	ActDropEth      = 0  // ParseEthFrm error: logged, dropped
	ActIgnoreMac    = 1  // not this NetIf's MAC
	ActArp          = 2  // HandleArp
	ActIgnoreType   = 3  // 802.3 / IPv6
	ActDropIp       = 4  // ParseIpv4Pkt error: logged, dropped
	ActBcastUdp     = 5  // RxUdpBroadcast, UDP parse OK
	ActDropBcastUdp = 6  // RxUdpBroadcast, UDP parse error: logged
	ActIgnoreBcast  = 7  // x.x.x.255, not UDP
	ActForward      = 8  // Ipv4RouteForward
	ActLocalIcmp    = 9  // RxIcmp, parse OK
	ActLocalUdp     = 10 // RxUdp, parse OK
	ActLocalTcp     = 11 // RxTcp, parse OK
	ActDropL4       = 12 // local L4 parse error: logged, dropped
	ActLoNotOwn     = 13 // LoChan drain: not this NetIf's address, skipped
)

var errText = [...]string{
	StatusEthLen:     "ethernet frame len must >= 42 and <= 1514 bytes", // ethernet.go:32
	StatusEthType:    "unknown ethernet protocol",                       // ethernet.go:49
	StatusIpLen:      "ip packet len must >= 20 and <= 1500 bytes",      // ipv4.go:50
	StatusIpVer:      "not support type of ip packet",                   // ipv4.go:53
	StatusIpFrag:     "not support ip frg",                              // ipv4.go:60
	StatusIpProto:    "unknown ip protocol",                             // ipv4.go:71
	StatusIpHdrCksum: "header check sum error",                          // ipv4.go:76
	StatusIcmpType:   "not support type of icmp packet",                 // icmp.go:46
	StatusIcmpCode:   "not support type of icmp packet",                 // icmp.go:50
	StatusL4Cksum:    "check sum error",                                 // udp.go:43 / tcp.go:64 / icmp.go:54
}

// ErrorText is the error string the reference function that failed returns for a record's status
// ("" for OK and the build-defined totalLen statuses). The L4 length check has one text per
// protocol, picked by the record's IpHeadProto.
func ErrorText(status, ipHeadProto uint8) string {
	if status == StatusL4Len {
		switch ipHeadProto {
		case protocol.IPH_PROTO_UDP:
			return "udp packet len must >= 8 and <= 1480 bytes" // udp.go:23
		case protocol.IPH_PROTO_TCP:
			return "tcp packet len must >= 20 and <= 1480 bytes" // tcp.go:38
		case protocol.IPH_PROTO_ICMP:
			return "icmp packet len must >= 8 and <= 1480 bytes" // icmp.go:35
		}
		return ""
	}
	if int(status) < len(errText) {
		return errText[status]
	}
	return ""
}

// Err is ErrorText as an error (nil when the text is empty).
func (r *Result) Err() error {
	if t := ErrorText(r.Status, r.IpHeadProto); t != "" {
		return errors.New(t)
	}
	return nil
}

// Payload is the innermost payload slice the parse returned, inside frame.
func (r *Result) Payload(frame []byte) []byte {
	return frame[r.PayloadOff : int(r.PayloadOff)+int(r.PayloadLen)]
}

func halo(rc C.int) error {
	if rc != 0 {
		return errors.New("gpurx: " + C.GoString(C.halo_rx_strerror(rc)))
	}
	return nil
}

// NetIfCfg is what the parse and the dispatch need of an engine.NetIf.
type NetIfCfg struct {
	MacAddr   []byte // NetIf.MacAddr (6 bytes)
	IpAddr    []byte // NetIf.IpAddr (4 bytes)
	NatEnable bool   // NetIfConfig.NatEnable
}

func (n *NetIfCfg) c() (C.halo_rx_netif_t, error) {
	if len(n.MacAddr) != 6 || len(n.IpAddr) != 4 {
		return C.halo_rx_netif_t{}, errors.New("gpurx: MacAddr must be 6 bytes and IpAddr 4")
	}
	nat := C.int(0)
	if n.NatEnable {
		nat = 1
	}
	return C.gpurx_netif((*C.uint8_t)(unsafe.Pointer(&n.MacAddr[0])), C.uint32_t(protocol.IpAddrToU(n.IpAddr)), nat), nil
}

// Ctx is a host context on one device (halo_rx_host_ctx_t: pinned staging and two streams). A Ctx
// serialises its own calls; use one per PacketHandle goroutine.
type Ctx struct {
	mu sync.Mutex
	c  *C.halo_rx_host_ctx_t
}

// NewCtx creates a host context on `device` (chunk sizes: the library's defaults).
func NewCtx(device int) (*Ctx, error) {
	var c *C.halo_rx_host_ctx_t
	if err := halo(C.halo_rx_host_ctx_create(C.int(device), 0, 0, &c)); err != nil {
		return nil, err
	}
	return &Ctx{c: c}, nil
}

// SetResident serves batches of up to maxFrames frames (<= 16384; 0 turns it off) with a kernel
// resident on the GPU instead of a launch per batch (halo_rx_host_ctx_set_resident): the frames are
// packed into pinned staging and one request line is written, so a PacketHandle-sized batch costs
// ~8 us instead of ~33-37 us (DESIGN.md §13.1). The kernel keeps 8 CUs while batches keep coming
// and leaves 20 ms after the last one. maxBytes bounds the staging (0: min(1516 * maxFrames, 64 MiB)).
func (x *Ctx) SetResident(maxFrames int, maxBytes uint64) error {
	x.mu.Lock()
	defer x.mu.Unlock()
	return halo(C.halo_rx_host_ctx_set_resident(x.c, C.uint32_t(maxFrames), C.uint64_t(maxBytes)))
}

// DeviceSynchronize waits for all work on `device` after stopping the library's resident consumers
// there (halo_rx_device_synchronize). A plain hipDeviceSynchronize from the caller would wait for
// those kernels too, which end only 20 ms after their last request.
func DeviceSynchronize(device int) error { return halo(C.halo_rx_device_synchronize(C.int(device))) }

// Release drains `device` and hands back its status-histogram tree keys (halo_rx_release); the
// trees, rings, contexts and captured graphs stay valid.
func Release(device int) error { return halo(C.halo_rx_release(C.int(device))) }

// Close frees the context.
func (x *Ctx) Close() {
	x.mu.Lock()
	defer x.mu.Unlock()
	if x.c != nil {
		C.halo_rx_host_ctx_destroy(x.c)
		x.c = nil
	}
}

func csumFlag() C.uint32_t {
	if protocol.CheckSumEnable {
		return C.HALO_RX_CSUM_ENABLE
	}
	return 0
}

func (x *Ctx) parse(buf []byte, off []uint64, lens []uint16, netif *NetIfCfg, flags C.uint32_t, out []Result) error {
	if len(off) != len(lens) || len(out) < len(lens) {
		return errors.New("gpurx: offsets, lengths and results disagree")
	}
	if len(lens) == 0 {
		return nil
	}
	if len(buf) == 0 {
		buf = make([]byte, 4) // every frame is empty: any valid address will do
	}
	n, err := netif.c()
	if err != nil {
		return err
	}
	x.mu.Lock()
	defer x.mu.Unlock()
	return halo(C.halo_rx_parse_batch_host(x.c, (*C.uint8_t)(unsafe.Pointer(&buf[0])),
		(*C.uint64_t)(unsafe.Pointer(&off[0])), (*C.uint16_t)(unsafe.Pointer(&lens[0])), C.uint32_t(len(lens)),
		flags, &n, (*C.halo_rx_result_t)(unsafe.Pointer(&out[0])), nil))
}

// ParseFramesBatch parses and verifies frames buf[off[i] : off[i]+lens[i]] exactly as
// ParseEthFrm -> ParseIpv4Pkt -> Parse{Udp,Tcp,Icmp}Pkt would, one Result per frame, with
// protocol.CheckSumEnable's current value (ICMP is always verified, icmp.go:53).
func (x *Ctx) ParseFramesBatch(buf []byte, off []uint64, lens []uint16, netif *NetIfCfg, out []Result) error {
	return x.parse(buf, off, lens, netif, csumFlag(), out)
}

// ParsePacketsL3 is ParseFramesBatch for bare IPv4 packets (a NetIf's LoChan: engine.go:353-381):
// every buffer starts at its IPv4 header (HALO_RX_L3_START). Starts must be 4-byte aligned
// relative to each other for the fast paths; PackAligned lays packets out that way.
func (x *Ctx) ParsePacketsL3(buf []byte, off []uint64, lens []uint16, netif *NetIfCfg, out []Result) error {
	return x.parse(buf, off, lens, netif, csumFlag()|C.HALO_RX_L3_START, out)
}

func dispatch(loopback bool, res []Result, netif *NetIfCfg, acts []uint8) error {
	if len(acts) < len(res) {
		return errors.New("gpurx: actions shorter than results")
	}
	if len(res) == 0 {
		return nil
	}
	n, err := netif.c()
	if err != nil {
		return err
	}
	r := (*C.halo_rx_result_t)(unsafe.Pointer(&res[0]))
	a := (*C.uint8_t)(unsafe.Pointer(&acts[0]))
	if loopback {
		return halo(C.halo_rx_dispatch_loopback(r, C.uint32_t(len(res)), &n, a, nil))
	}
	return halo(C.halo_rx_dispatch(r, C.uint32_t(len(res)), &n, a, nil))
}

// Dispatch maps records to the branch RxEthernet -> RxIpv4 takes for each (Act* codes).
func Dispatch(res []Result, netif *NetIfCfg, acts []uint8) error { return dispatch(false, res, netif, acts) }

// DispatchLoopback maps LoChan records (ParsePacketsL3) to PacketHandle's drain decisions.
func DispatchLoopback(res []Result, netif *NetIfCfg, acts []uint8) error {
	return dispatch(true, res, netif, acts)
}

// Batch is a reusable batch: frames copied back to back (4-byte aligned starts, as halo's ring
// records are, mem/ring_buffer.go:47-50), their records and actions.
type Batch struct {
	Buf  []byte
	Off  []uint64
	Lens []uint16
	Res  []Result
	Act  []uint8
}

// NewBatch allocates room for max frames of up to 1514 bytes.
func NewBatch(max int) *Batch {
	return &Batch{Buf: make([]byte, 0, max*1516), Off: make([]uint64, 0, max), Lens: make([]uint16, 0, max),
		Res: make([]Result, max), Act: make([]uint8, max)}
}

// Reset empties the batch, keeping its memory.
func (b *Batch) Reset() { b.Buf, b.Off, b.Lens = b.Buf[:0], b.Off[:0], b.Lens[:0] }

// Len is the number of frames in the batch.
func (b *Batch) Len() int { return len(b.Lens) }

// Add copies one frame in (EthRxFunc's slice aliases a reused buffer: dpdk/dpdk.go:184-194,
// engine/engine.go:544, so it must be copied before the next poll — the one copy the reference
// already makes out of the ring). Frames longer than 65535 bytes are cut to 65535: the record's
// length field is a u16, and every length past 1514 (9014 with the jumbo extension) gets the same
// ETH_LEN verdict, so the verdicts are unchanged; Frame(k) then returns the first 65535 bytes.
func (b *Batch) Add(frame []byte) {
	if len(frame) > 0xFFFF {
		frame = frame[:0xFFFF]
	}
	b.Off = append(b.Off, uint64(len(b.Buf)))
	b.Lens = append(b.Lens, uint16(len(frame)))
	b.Buf = append(b.Buf, frame...)
	for len(b.Buf)%4 != 0 {
		b.Buf = append(b.Buf, 0)
	}
	if len(b.Lens) > len(b.Res) {
		b.Res = append(b.Res, Result{})
		b.Act = append(b.Act, 0)
	}
}

// Frame k of the batch.
func (b *Batch) Frame(k int) []byte { return b.Buf[b.Off[k] : b.Off[k]+uint64(b.Lens[k])] }

// PackAligned lays packets out back to back at 4-byte aligned offsets.
func PackAligned(pkts [][]byte) *Batch {
	b := NewBatch(len(pkts))
	for _, p := range pkts {
		b.Add(p)
	}
	return b
}

// ParseBatch parses every frame of b (ParseFramesBatch, or ParsePacketsL3 when l3) and dispatches
// the records (Dispatch / DispatchLoopback) into b.Res and b.Act.
func (x *Ctx) ParseBatch(b *Batch, netif *NetIfCfg, l3 bool) error {
	n := b.Len()
	var err error
	if l3 {
		err = x.ParsePacketsL3(b.Buf, b.Off, b.Lens, netif, b.Res[:n])
	} else {
		err = x.ParseFramesBatch(b.Buf, b.Off, b.Lens, netif, b.Res[:n])
	}
	if err != nil {
		return err
	}
	return dispatch(l3, b.Res[:n], netif, b.Act[:n])
}
