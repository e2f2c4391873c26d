// route_lpm.hip — SURVEY.md §8f row f4: the forward path's route lookup (NetIf.FindRoute ->
// RouteTable.FindRoute, engine/ipv4_engine.go:351-390) on gfx950.
//
// Control plane (host): the reference's binary trie, kept node for node as UpdateRoute builds it
// (engine/ipv4_engine.go:304-348) — prefix depth 32 - ctz(mask), the path of the OLD route's
// destination bits, a non-nil (possibly emptied) route list per touched node, list order =
// insertion order. FindRoute's answer for an address is the deepest node with a non-nil list on
// the address's path, so the trie is a plain longest-prefix-match set and compiles to a DIR-24-8
// table: tbl24[ip >> 8] holds either a list reference or a pointer to a 256-entry block indexed
// by ip & 0xFF. The compile is a DFS that fills each absent subtree's address range with the
// list inherited from above (16M first-level entries, 64 MB of HBM: a dependent pair of 4-byte
// reads per lookup, served mostly from the 256 MB Infinity Cache).
//
// Data plane (device): per address, one or two table reads; a one-route list is stored in the
// table as the route id itself, otherwise the ECMP pick of FindRoute follows:
// ids[start + fnv32a(ip) % count] (Go hash/fnv New32a over the 4 address bytes, the
// RouteTable.IpHash of engine/engine.go:159); count 0 is the reference's divide-by-zero panic,
// reported as HALO_ROUTE_PANIC.
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <vector>

#include "halo_common.h"
#include "route_view.h"

struct halo_route_table {
    struct Node {
        int32_t child[2] = {-1, -1};
        bool has_list = false;  // RouteList != nil
        std::vector<uint32_t> ids;
    };
    std::vector<Node> nodes;  // nodes[0] = Root
    std::vector<halo_route_entry_t> routes;
    mutable std::mutex mu;  // RouteTable.Lock
    // Device copies, double-buffered: lookups read gen[active]; a sync compiles into the other
    // generation (after the device has drained every lookup that could still read it) and then
    // publishes it, so a lookup in flight never sees a table being rewritten or freed.
    struct Gen {
        uint32_t* d_tbl24 = nullptr;
        uint32_t* d_tbl8 = nullptr;
        size_t tbl8_cap = 0;
        uint2* d_lists = nullptr;  // (start, count) per list
        size_t lists_cap = 0;
        uint32_t* d_ids = nullptr;
        size_t ids_cap = 0;
    } gen[2];
    int device = -1;
    std::atomic<int> active{-1};  // published generation, -1 before the first sync
    std::mutex sync_mu;           // one sync at a time
    // Lookups hold it shared from route_view until their kernel is enqueued (RouteViewLock); a sync
    // holds it exclusively while it drains the device and rewrites the unpublished generation, so
    // no lookup can be enqueued against a generation between its view and the drain.
    mutable std::shared_mutex view_mu;
};

namespace halo {
namespace {


struct Compiler {
    const halo_route_table& t;
    std::vector<uint32_t>& tbl24;
    std::vector<uint32_t>& tbl8;
    std::vector<uint2>& lists;
    std::vector<uint32_t>& ids;

    // table value of a node with a non-nil list: kDirect | id for a one-route list (no ECMP pick:
    // the lookup is then a single table read), else the list reference (index + 1)
    uint32_t list_of(const halo_route_table::Node& n) {
        if (n.ids.size() == 1 && n.ids[0] < kDirect) return kDirect | n.ids[0];
        const uint32_t start = (uint32_t)ids.size();
        ids.insert(ids.end(), n.ids.begin(), n.ids.end());
        lists.push_back(make_uint2(start, (uint32_t)n.ids.size()));
        return (uint32_t)lists.size();
    }
    static void fill(std::vector<uint32_t>& v, size_t lo, size_t hi, uint32_t x) {
        for (size_t k = lo; k < hi; ++k) v[k] = x;
    }
    // node at depth 24 < d <= 32 under a tbl8 block; `low` = the address bits after the 24th
    void walk8(int32_t ni, uint32_t depth, uint32_t low, uint32_t inherited, size_t blk) {
        const auto& n = t.nodes[ni];
        const uint32_t v = n.has_list ? list_of(n) : inherited;
        if (depth == 32) {
            tbl8[blk * 256 + low] = v;
            return;
        }
        for (uint32_t b = 0; b < 2; ++b) {
            const uint32_t sub = low * 2 + b;  // (depth + 1 - 24) bits
            const uint32_t shift = 31 - depth;
            if (n.child[b] >= 0) walk8(n.child[b], depth + 1, sub, v, blk);
            else fill(tbl8, blk * 256 + ((size_t)sub << shift), blk * 256 + ((size_t)(sub + 1) << shift), v);
        }
    }
    // node at depth d <= 24 with address prefix `prefix` (d bits)
    void walk(int32_t ni, uint32_t depth, uint32_t prefix, uint32_t inherited) {
        const auto& n = t.nodes[ni];
        const uint32_t v = n.has_list ? list_of(n) : inherited;
        if (depth == 24) {
            if (n.child[0] < 0 && n.child[1] < 0) {
                tbl24[prefix] = v;
                return;
            }
            const size_t blk = tbl8.size() / 256;
            tbl8.resize(tbl8.size() + 256, 0u);
            tbl24[prefix] = kExt | (uint32_t)blk;
            for (uint32_t b = 0; b < 2; ++b) {
                if (n.child[b] >= 0) walk8(n.child[b], 25, b, v, blk);
                else fill(tbl8, blk * 256 + (size_t)b * 128, blk * 256 + (size_t)(b + 1) * 128, v);
            }
            return;
        }
        for (uint32_t b = 0; b < 2; ++b) {
            const uint32_t sub = prefix * 2 + b;
            const uint32_t shift = 23 - depth;
            if (n.child[b] >= 0) walk(n.child[b], depth + 1, sub, v);
            else fill(tbl24, (size_t)sub << shift, (size_t)(sub + 1) << shift, v);
        }
    }
};

// four addresses per lane (one 16-byte load), grid-stride
__global__ void __launch_bounds__(256) lpm_kernel(const LpmView v, const uint32_t* ips, uint32_t n, uint32_t* out) {
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t n4 = n / 4;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += stride) {
        const uint4 a = reinterpret_cast<const uint4*>(ips)[q];
        uint4 r;
        r.x = find_route(v, a.x);
        r.y = find_route(v, a.y);
        r.z = find_route(v, a.z);
        r.w = find_route(v, a.w);
        reinterpret_cast<uint4*>(out)[q] = r;
    }
    for (uint32_t i = n4 * 4 + blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = find_route(v, ips[i]);
}

// dst_ip of each halo_rx_result_t (dword 3): the forward path's FindRoute(ipv4DstAddr)
__global__ void __launch_bounds__(256) lpm_records_kernel(const LpmView v, const halo_rx_result_t* recs, uint32_t n,
                                                          uint32_t* out) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = find_route(v, reinterpret_cast<const uint32_t*>(recs)[8ull * i + 3]);
}

uint32_t lpm_blocks(uint64_t threads) {
    const uint64_t b = (threads + 255) / 256;
    const uint64_t kMax = 256ull * 8 * 8;
    return (uint32_t)(b > kMax ? kMax : (b ? b : 1));
}

bool same_route(const halo_route_entry_t& a, const halo_route_entry_t& b) {
    return a.dst_ip == b.dst_ip && a.network_mask == b.network_mask && a.next_hop == b.next_hop && a.netif == b.netif;
}

template <typename T>
int grow(T*& p, size_t& cap, size_t need) {
    if (need <= cap) return HALO_OK;
    size_t c = cap ? cap : 256;
    while (c < need) c *= 2;
    T* q = nullptr;
    if (hipMalloc(&q, c * sizeof(T)) != hipSuccess) return HALO_E_NOMEM;
    if (p) (void)hipFree(p);
    p = q;
    cap = c;
    return HALO_OK;
}

struct DeviceScope {  // run on `dev`, restore the caller's current device
    int prev = -1;
    explicit DeviceScope(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceScope() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace
}  // namespace halo

extern "C" HALO_API int halo_route_table_create(halo_route_table_t** out) {
    if (!out) return HALO_E_INVAL;
    auto* t = new (std::nothrow) halo_route_table;
    if (!t) return HALO_E_NOMEM;
    t->nodes.emplace_back();  // Root: new(TrieNode) (engine/engine.go:158)
    *out = t;
    return HALO_OK;
}

extern "C" HALO_API int halo_route_table_destroy(halo_route_table_t* t) {
    if (!t) return HALO_E_INVAL;
    if (t->device >= 0) {
        halo::DeviceScope ds(t->device);
        halo::ParkResidents park(t->device);  // through the frees: hipFree waits for every kernel
        (void)halo::drain_device(t->device);  // no lookup may still read the tables
        for (auto& g : t->gen) {
            if (g.d_tbl24) (void)hipFree(g.d_tbl24);
            if (g.d_tbl8) (void)hipFree(g.d_tbl8);
            if (g.d_lists) (void)hipFree(g.d_lists);
            if (g.d_ids) (void)hipFree(g.d_ids);
        }
    }
    delete t;
    return HALO_OK;
}

extern "C" HALO_API int halo_route_update(halo_route_table_t* t, const halo_route_entry_t* old_route,
                                          const halo_route_entry_t* new_route, uint32_t* new_id) {
    if (!t || !old_route) return HALO_E_INVAL;
    std::lock_guard<std::mutex> g(t->mu);  // RouteTable.Lock
    uint32_t depth = 0;
    const uint32_t mask = old_route->network_mask;
    if (mask) depth = 32u - (uint32_t)__builtin_ctz(mask);  // the maskSize loop of :309-317
    int32_t ni = 0;
    for (uint32_t i = 0; i < depth; ++i) {
        const uint32_t bit = (old_route->dst_ip >> (31 - i)) & 1u;
        int32_t c = t->nodes[ni].child[bit];
        if (c < 0) {
            c = (int32_t)t->nodes.size();
            t->nodes.emplace_back();
            t->nodes[ni].child[bit] = c;
        }
        ni = c;
    }
    auto& node = t->nodes[ni];
    std::vector<uint32_t> list;
    list.reserve(node.ids.size() + 1);
    for (uint32_t id : node.ids)
        if (!halo::same_route(t->routes[id], *old_route)) list.push_back(id);
    if (new_route) {
        const uint32_t id = (uint32_t)t->routes.size();
        if (id >= HALO_ROUTE_PANIC) return HALO_E_RANGE;
        t->routes.push_back(*new_route);
        list.push_back(id);
        if (new_id) *new_id = id;
    }
    node.ids.swap(list);
    node.has_list = true;
    return HALO_OK;
}

extern "C" HALO_API int halo_route_get(const halo_route_table_t* t, uint32_t id, halo_route_entry_t* out) {
    if (!t || !out) return HALO_E_INVAL;
    std::lock_guard<std::mutex> g(t->mu);
    if (id >= t->routes.size()) return HALO_E_RANGE;
    *out = t->routes[id];
    return HALO_OK;
}

extern "C" HALO_API int halo_route_sync_device(halo_route_table_t* t, int device) {
    if (!t || device < 0) return HALO_E_INVAL;
    if (t->device >= 0 && t->device != device) return HALO_E_INVAL;  // one device per table
    int rc;
    {
        int cnt = 0;
        if (hipGetDeviceCount(&cnt) != hipSuccess || device >= cnt) return HALO_E_NODEV;
    }
    halo::DeviceScope ds(device);
    if ((rc = halo::check_device())) return rc;
    halo::ParkResidents park(device);  // the drains, table growth (hipFree) and copies below
    std::vector<uint32_t> tbl24(1u << 24, 0u), tbl8, ids;
    std::vector<uint2> lists;
    {
        std::lock_guard<std::mutex> g(t->mu);
        halo::Compiler c{*t, tbl24, tbl8, lists, ids};
        c.walk(0, 0, 0, 0u);
    }
    std::lock_guard<std::mutex> sg(t->sync_mu);
    std::unique_lock<std::shared_mutex> vl(t->view_mu);  // no lookup between its view and its launch
    const int cur = t->active.load(std::memory_order_acquire);
    // the generation written now was last published before `cur`: lookups launched while it was
    // active may still be running on any stream of the device, so drain the device first
    // (resident consumers are stopped for it, so a persistent ring's kernel cannot hold the write
    // lock, and the lookups behind it, for its 20 ms idle window: ADVICE r3)
    if (cur >= 0 && halo::drain_device(device) != HALO_OK) return HALO_E_HIP;
    auto& g = t->gen[cur < 0 ? 0 : 1 - cur];
    if (!g.d_tbl24 && hipMalloc(&g.d_tbl24, tbl24.size() * sizeof(uint32_t)) != hipSuccess) return HALO_E_NOMEM;
    t->device = device;
    if ((rc = halo::grow(g.d_tbl8, g.tbl8_cap, tbl8.size() ? tbl8.size() : 1))) return rc;
    if ((rc = halo::grow(g.d_lists, g.lists_cap, lists.size() ? lists.size() : 1))) return rc;
    if ((rc = halo::grow(g.d_ids, g.ids_cap, ids.size() ? ids.size() : 1))) return rc;
    if (hipMemcpy(g.d_tbl24, tbl24.data(), tbl24.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess ||
        (tbl8.size() &&
         hipMemcpy(g.d_tbl8, tbl8.data(), tbl8.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) ||
        (lists.size() &&
         hipMemcpy(g.d_lists, lists.data(), lists.size() * sizeof(uint2), hipMemcpyHostToDevice) != hipSuccess) ||
        (ids.size() && hipMemcpy(g.d_ids, ids.data(), ids.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess))
        return HALO_E_HIP;
    // hipMemcpy from pageable memory returns once the host buffer is consumed, not when the copy
    // has landed: wait for it before publishing
    if (halo::drain_device(device) != HALO_OK) return HALO_E_HIP;
    t->active.store(cur < 0 ? 0 : 1 - cur, std::memory_order_release);
    return HALO_OK;
}

namespace halo {
RouteViewLock::RouteViewLock(const halo_route_table_t* t) : t_(t) {
    if (t_) t_->view_mu.lock_shared();
}
RouteViewLock::~RouteViewLock() {
    if (t_) t_->view_mu.unlock_shared();
}

int route_view(const halo_route_table_t* t, LpmView* out) {
    if (!t || !out) return HALO_E_INVAL;
    const int a = t->active.load(std::memory_order_acquire);
    if (a < 0) return HALO_E_INVAL;  // never synced
    const auto& g = t->gen[a];
    *out = LpmView{g.d_tbl24, g.d_tbl8, g.d_lists, g.d_ids};
    return HALO_OK;
}
}  // namespace halo

extern "C" HALO_API int halo_route_lookup_device(const halo_route_table_t* t, const uint32_t* d_ips, uint32_t n,
                                                 uint32_t* d_route_ids, halo_stream_t stream) {
    halo::RouteViewLock lk(t);
    halo::LpmView v;
    if (halo::route_view(t, &v)) return HALO_E_INVAL;
    if (n == 0) return HALO_OK;
    if (!d_ips || !d_route_ids) return HALO_E_INVAL;
    if ((reinterpret_cast<uintptr_t>(d_ips) | reinterpret_cast<uintptr_t>(d_route_ids)) & 15u) return HALO_E_INVAL;
    int rc = halo::check_device();
    if (rc) return rc;
    hipLaunchKernelGGL(halo::lpm_kernel, dim3(halo::lpm_blocks((n + 3) / 4)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), v, d_ips, n, d_route_ids);
    return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
}

extern "C" HALO_API int halo_route_lookup_records_device(const halo_route_table_t* t,
                                                         const halo_rx_result_t* d_records, uint32_t n,
                                                         uint32_t* d_route_ids, halo_stream_t stream) {
    halo::RouteViewLock lk(t);
    halo::LpmView v;
    if (halo::route_view(t, &v)) return HALO_E_INVAL;
    if (n == 0) return HALO_OK;
    if (!d_records || !d_route_ids) return HALO_E_INVAL;
    int rc = halo::check_device();
    if (rc) return rc;
    hipLaunchKernelGGL(halo::lpm_records_kernel, dim3(halo::lpm_blocks(n)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), v, d_records, n, d_route_ids);
    return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
}
