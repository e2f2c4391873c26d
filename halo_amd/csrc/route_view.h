// route_view.h — the device side of a synced route table (route_lpm.hip): the DIR-24-8 lookup of
// NetIf.FindRoute (engine/ipv4_engine.go:351-390) shared by the standalone lookup kernels and the
// rx kernels' fused pass (halo_rx_parse_route_batch_device), so both return the same route ids.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/halo_rx.h"

namespace halo {

constexpr uint32_t kExt = 0x80000000u;     // tbl24 entry: index of a tbl8 block
constexpr uint32_t kDirect = 0x40000000u;  // entry: the route id itself (a one-route list)

struct LpmView {
    const uint32_t* tbl24;
    const uint32_t* tbl8;
    const uint2* lists;  // (start, count) per ECMP list
    const uint32_t* ids;
};

// Go hash/fnv New32a over the 4 address bytes (RouteTable.IpHash, engine/engine.go:159)
__device__ __forceinline__ uint32_t fnv1a32(uint32_t ip) {
    uint32_t h = 2166136261u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        h ^= (ip >> (24 - 8 * k)) & 0xFFu;
        h *= 16777619u;
    }
    return h;
}

__device__ __forceinline__ uint32_t find_route(const LpmView& v, uint32_t ip) {
    uint32_t e = v.tbl24[ip >> 8];
    if (e & kExt) e = v.tbl8[(size_t)(e & ~kExt) * 256 + (ip & 0xFFu)];
    if (e == 0) return HALO_ROUTE_NONE;
    if (e & kDirect) return e & ~kDirect;
    const uint2 l = v.lists[e - 1];
    if (l.y == 0) return HALO_ROUTE_PANIC;  // Go's divide-by-zero panic on an emptied list
    return v.ids[l.x + fnv1a32(ip) % l.y];
}

// The device view of a table synced with halo_route_sync_device (HALO_E_INVAL otherwise). Take it
// under a RouteViewLock held until the kernel using it is enqueued: a concurrent sync then cannot
// rewrite that generation before the device has drained the launch.
int route_view(const halo_route_table_t* t, LpmView* out);
class RouteViewLock {
public:
    explicit RouteViewLock(const halo_route_table_t* t);
    ~RouteViewLock();
    RouteViewLock(const RouteViewLock&) = delete;
    RouteViewLock& operator=(const RouteViewLock&) = delete;

private:
    const halo_route_table_t* t_;
};

}  // namespace halo
