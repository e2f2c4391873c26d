package engine

// The batched NetIf.PacketHandle: a file a halo maintainer adds to package engine (next to
// engine.go) to receive through package gpurx. It keeps PacketHandle's loop, its EthRxFunc
// surface and its observable behaviour — the same handlers, service callbacks, TX replies and log
// lines, in the same order — but parses each batch of frames in one GPU call and then acts on the
// records frame by frame, exactly where RxEthernet -> RxIpv4 -> Rx{Icmp,Udp,Tcp} would have.
//
// Reference: engine/engine.go:339-385 (PacketHandle and its LoChan drain),
// engine/ethernet_engine.go:13-31 (RxEthernet), engine/ipv4_engine.go:18-47 (RxIpv4),
// engine/{udp,tcp,icmp}_engine.go (RxUdp / RxUdpBroadcast, RxTcp, RxIcmp).

import (
	"fmt"

	"github.com/flswld/halo/cpu"
	"github.com/flswld/halo/gpurx"
	"github.com/flswld/halo/protocol"
)

// BatchConfig tunes PacketHandleBatched.
type BatchConfig struct {
	// Batch is the most frames one GPU call parses (0: 4096).
	Batch int
	// DrainEvery is the number of EthRxFunc polls between LoChan drains. 99 is PacketHandle's own
	// cadence (engine.go:353: n == 100-1): a batch then ends at every 99th poll and the drain runs
	// there, so handlers, drains and their TX see exactly the reference's order. 0 drains after
	// every batch, and a batch also ends at the first poll that returns nil.
	DrainEvery int
	// Launched turns the resident consumer off: every batch is then a launch + synchronisation
	// (~33-37 us for <= 256 frames instead of ~8 us, DESIGN.md §13.1), and no kernel stays on the
	// GPU between batches.
	Launched bool
	// CPUBelow sends a batch (or LoChan drain) of fewer frames to the CPU entry point
	// (gpurx.ParseBatchCPU, halo_rx_parse_batch_cpu): the same records on this goroutine's core,
	// ~9 ns per frame against ~8 us per GPU round trip, so below ~3,800 frames it is the faster
	// path (INTEGRATION.md §1a). 0 keeps every batch on the GPU.
	CPUBelow int
}

// parse is ParseBatch on the GPU, or on the CPU entry point below cfg.CPUBelow frames.
func (cfg *BatchConfig) parse(x *gpurx.Ctx, b *gpurx.Batch, netif *gpurx.NetIfCfg, l3 bool) error {
	if b.Len() < cfg.CPUBelow {
		return gpurx.ParseBatchCPU(b, netif, l3)
	}
	return x.ParseBatch(b, netif, l3)
}

// PacketHandleBatched replaces `go netIf.PacketHandle()` (engine.go:299) for a NetIf whose frames
// are parsed on the GPU by x.
//
// One difference in timing, not in results for unchanged configuration: the reference parses and
// acts on each frame before it polls the next, while a batch is parsed as a whole before its
// handlers run, with the NetIf's MAC / IP / NatEnable as they were at the start of the batch. A
// handler that changes them (RxDhcp storing a leased address, engine/dhcp_engine.go) takes effect
// from the next batch; the frames after it in the same batch were judged (DST_IS_OWN, MAC_MATCH)
// against the old address. With DrainEvery 99 a batch spans at most 99 polls. A failed GPU call
// drops its whole batch with one log line where the reference would have handled each frame.
func (i *NetIf) PacketHandleBatched(x *gpurx.Ctx, cfg BatchConfig) {
	if i.Config.BindCpuCore >= 0 {
		cpu.BindCpuCore(i.Config.BindCpuCore)
	}
	if cfg.Batch <= 0 {
		cfg.Batch = 4096
	}
	if !cfg.Launched && cfg.Batch <= 16384 {
		if err := x.SetResident(cfg.Batch, 0); err != nil {
			Log(fmt.Sprintf("gpurx resident consumer unavailable, batches are launched: %v\n", err))
		}
	}
	netif := &gpurx.NetIfCfg{MacAddr: i.MacAddr, IpAddr: i.IpAddr, NatEnable: i.Config.NatEnable}
	b := gpurx.NewBatch(cfg.Batch)
	n := 0 // polls since the last drain: PacketHandle's n
	for !i.Router.Stop.Load() {
		b.Reset()
		for b.Len() < cfg.Batch {
			f := i.Config.EthRxFunc()
			n++
			if f != nil {
				b.Add(f) // EthRxFunc's slice aliases a reused buffer: copied before the next poll
			}
			if cfg.DrainEvery > 0 && n >= cfg.DrainEvery {
				break
			}
			if f == nil && cfg.DrainEvery == 0 {
				break
			}
		}
		if b.Len() > 0 {
			if err := cfg.parse(x, b, netif, false); err != nil {
				Log(fmt.Sprintf("gpurx parse error: %v\n", err))
			} else {
				for k := 0; k < b.Len(); k++ {
					i.dispatchParsed(b.Frame(k), &b.Res[k], b.Act[k])
				}
			}
		}
		if cfg.DrainEvery == 0 || n >= cfg.DrainEvery {
			i.drainLoChanBatched(x, netif, &cfg)
			n = 0
		}
	}
	i.Router.StopWaitGroup.Done()
}

// dispatchParsed is RxEthernet -> RxIpv4 for one frame whose record the GPU produced: the parse
// calls are replaced by reads of r, the branches by the action halo_rx_dispatch derived from it
// (tests/test_abi.py::test_dispatch_matches_oracle_engine checks that order).
func (i *NetIf) dispatchParsed(frm []byte, r *gpurx.Result, act uint8) {
	if i.Router.Config.DebugLog {
		Log(fmt.Sprintf("rx eth frm, if: %v, len: %v, data: %02x\n", i.Config.Name, len(frm), frm))
	}
	switch act {
	case gpurx.ActDropEth:
		Log(fmt.Sprintf("parse ethernet frame error: %v\n", r.Err()))
	case gpurx.ActArp:
		i.HandleArp(frm[14:], frm[6:12])
	case gpurx.ActDropIp:
		Log(fmt.Sprintf("parse ip packet error: %v\n", r.Err()))
	case gpurx.ActBcastUdp:
		udpPayload := r.Payload(frm)
		if r.DstPort == DhcpClientPort || r.DstPort == DhcpServerPort {
			i.RxDhcp(udpPayload, r.SrcPort, r.DstPort, frm[26:30])
		}
	case gpurx.ActDropBcastUdp:
		Log(fmt.Sprintf("parse udp packet error: %v\n", r.Err()))
	case gpurx.ActForward:
		ok := i.Ipv4RouteForward(frm[14:], frm[26:30], frm[30:34], r.IpHeadProto)
		if !ok && r.IpHeadProto == protocol.IPH_PROTO_ICMP {
			i.deliverParsed(frm, 14, r) // RxIcmp(ipv4Payload, ipv4SrcAddr)
		}
	case gpurx.ActLocalIcmp, gpurx.ActLocalUdp, gpurx.ActLocalTcp, gpurx.ActDropL4:
		i.deliverParsed(frm, 14, r)
	}
	// ActIgnoreMac, ActIgnoreType, ActIgnoreBcast: the reference does nothing
}

// deliverParsed is RxIcmp / RxUdp / RxTcp (engine/{icmp,udp,tcp}_engine.go) after their parse
// call, for a record whose L4 verdict the GPU produced. `buf` is the frame (ipOff 14) or, from the
// LoChan drain, the bare IPv4 packet (ipOff 0) the record's offsets refer to.
func (i *NetIf) deliverParsed(buf []byte, ipOff int, r *gpurx.Result) {
	src := buf[ipOff+12 : ipOff+16] // ipv4SrcAddr
	var err error
	if r.Status != gpurx.StatusOK {
		err = r.Err()
	}
	switch r.IpHeadProto {
	case protocol.IPH_PROTO_ICMP:
		if err != nil {
			Log(fmt.Sprintf("parse icmp packet error: %v\n", err))
			return
		}
		if r.L4Aux == protocol.ICMP_REQUEST {
			icmp := buf[ipOff+20:]
			i.TxIcmp(r.Payload(buf), protocol.ICMP_REPLY, icmp[4:6], uint16(r.Seq), src)
		}
	case protocol.IPH_PROTO_UDP:
		if err != nil {
			Log(fmt.Sprintf("parse udp packet error: %v\n", err))
			return
		}
		handleFunc, exist := i.UdpServiceMap[r.DstPort]
		if !exist {
			return
		}
		handleFunc(UdpSession{RemoteIp: r.SrcAddr, RemotePort: r.SrcPort}, r.Payload(buf))
	case protocol.IPH_PROTO_TCP:
		if err != nil {
			Log(fmt.Sprintf("parse tcp packet error: %v\n", err))
			return
		}
		handleFunc, exist := i.TcpServiceMap[r.DstPort]
		if !exist {
			return
		}
		flags := r.L4Aux
		if flags&protocol.TCP_FLAGS_SYN != 0 && flags&protocol.TCP_FLAGS_ACK == 0 {
			i.TxTcp(nil, r.DstPort, r.SrcPort, src, 1234567890, r.Seq+1, protocol.TCP_FLAGS_SYN|protocol.TCP_FLAGS_ACK)
		} else if flags&protocol.TCP_FLAGS_SYN != 0 && flags&protocol.TCP_FLAGS_ACK != 0 {
			i.TxTcp(nil, r.DstPort, r.SrcPort, src, 1234567891, r.Seq+1, protocol.TCP_FLAGS_ACK)
		}
		handleFunc(TcpSession{RemoteIp: r.SrcAddr, RemotePort: r.SrcPort}, r.Payload(buf), r.Seq, r.Ack, flags)
	}
}

// drainLoChanBatched is PacketHandle's loopback drain (engine.go:353-381): until LoChan is empty,
// take what is queued (at most cfg.Batch packets per call; on the CPU entry point below
// cfg.CPUBelow), parse it with HALO_RX_L3_START and act
// per packet in order — ParseIpv4Pkt error: logged; not this NetIf's address: skipped; else the
// local RxIcmp / RxUdp / RxTcp. Handlers that queue more loopback packets are drained in the same
// call, as the reference's select loop drains them.
func (i *NetIf) drainLoChanBatched(x *gpurx.Ctx, netif *gpurx.NetIfCfg, cfg *BatchConfig) {
	max := cfg.Batch
	for {
		var pkts [][]byte
	take:
		for len(pkts) < max {
			select {
			case p := <-i.LoChan:
				pkts = append(pkts, p)
			default:
				break take
			}
		}
		if len(pkts) == 0 {
			return
		}
		b := gpurx.PackAligned(pkts)
		if err := cfg.parse(x, b, netif, true); err != nil {
			Log(fmt.Sprintf("gpurx parse error: %v\n", err))
			return
		}
		for k := range pkts {
			r := &b.Res[k]
			switch b.Act[k] {
			case gpurx.ActDropIp:
				Log(fmt.Sprintf("parse ip packet error: %v\n", r.Err()))
			case gpurx.ActLoNotOwn:
			case gpurx.ActLocalIcmp, gpurx.ActLocalUdp, gpurx.ActLocalTcp, gpurx.ActDropL4:
				i.deliverParsed(b.Frame(k), 0, r)
			}
		}
	}
}
