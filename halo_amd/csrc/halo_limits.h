// halo_limits.h — the reference's protocol limits and constants, shared by the kernels
// (halo_common.h) and the HIP-free host logic (host_logic.h).
#pragma once
#include <stdint.h>

namespace halo {

// Reference limits (protocol/ethernet.go:31, protocol/ipv4.go:49, protocol/udp.go:22,
// protocol/tcp.go:37, protocol/icmp.go:34) and the build-defined jumbo extension.
constexpr uint32_t kEthMin = 42, kEthMax = 1514, kIpMax = 1500, kL4Max = 1480;
constexpr uint32_t kEthMaxJumbo = 9014, kIpMaxJumbo = 9000, kL4MaxJumbo = 8980;

// EtherTypes (protocol/ethernet.go:16-22), IP protocol ids (protocol/ipv4.go:27-32),
// ICMP types (protocol/icmp.go:25-30).
constexpr uint16_t kEthIeee8023 = 0x05DC, kEthIpv4 = 0x0800, kEthArp = 0x0806,
                   kEthIpv6 = 0x86DD, kEthUnknown = 0xFFFF;
constexpr uint8_t kIpIcmp = 0x01, kIpTcp = 0x06, kIpUdp = 0x11, kIpUnknown = 0xFF;
constexpr uint8_t kIcmpRequest = 0x08, kIcmpReply = 0x00, kIcmpTtl = 0x0B;

constexpr uint64_t kRbHeader = 128;  // sizeof(RingBuffer), mem/ring_buffer.go:18-26

}  // namespace halo
