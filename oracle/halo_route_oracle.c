/*
 * halo_route_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline for SURVEY.md
 * §8f row f4, route lookup). Linked into oracle/liboracle.so; never into the product.
 *
 * Restates the reference's binary-trie route table literally (paths under /root/reference):
 *   RouteTable / TrieNode / RouteEntry  engine/ipv4_engine.go:270-290
 *   AddRoute / DeleteRoute              :293-301 (UpdateRoute(r, r) / UpdateRoute(r, nil))
 *   UpdateRoute                         :304-348 (depth = 32 - ctz(mask) for mask != 0; the path
 *                                        follows the OLD route's dst bits; a non-nil, possibly
 *                                        empty list replaces the node's list)
 *   FindRoute                           :351-383 (deepest non-nil list on the address's path;
 *                                        ECMP pick lastMatch[fnv32a(ip) % len])
 *   IpHash = fnv.New32a()               engine/engine.go:159 (Go stdlib hash/fnv FNV-1a 32)
 *   IpAddrToU                           protocol/utils.go:34-44
 *
 * A route entry is identified by the id it got when it was inserted (the reference returns the
 * *RouteEntry pointer). FindRoute's `r.IpHash.Sum32() % uint32(len(lastMatch))` divides by zero
 * when the deepest non-nil list is empty (a node whose routes were all deleted): Go panics; the
 * restatement returns HALO_ROUTE_PANIC.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/halo_rx.h"

#define ORA_API __attribute__((visibility("default")))

typedef struct ora_node {
    struct ora_node *left, *right;
    int has_list;     /* RouteList != nil */
    uint32_t n, cap;  /* len / cap of RouteList */
    uint32_t* ids;    /* route ids, list order */
} ora_node_t;

typedef struct {
    ora_node_t* root;
    halo_route_entry_t* routes; /* by id */
    uint32_t n_routes, cap_routes;
} ora_rt_t;

ORA_API ora_rt_t* ora_route_create(void) {
    ora_rt_t* t = (ora_rt_t*)calloc(1, sizeof(ora_rt_t));
    t->root = (ora_node_t*)calloc(1, sizeof(ora_node_t));
    return t;
}

static void free_node(ora_node_t* n) {
    if (!n) return;
    free_node(n->left);
    free_node(n->right);
    free(n->ids);
    free(n);
}

ORA_API void ora_route_destroy(ora_rt_t* t) {
    if (!t) return;
    free_node(t->root);
    free(t->routes);
    free(t);
}

/* UpdateRoute (engine/ipv4_engine.go:304-348). Returns the new route's id (or UINT32_MAX). */
ORA_API uint32_t ora_route_update(ora_rt_t* t, const halo_route_entry_t* old_r, const halo_route_entry_t* new_r) {
    ora_node_t* node = t->root;
    int mask_size = 0;
    const uint32_t mask = old_r->network_mask;
    if (mask != 0) {
        for (int i = 1; i <= 32; i++) {
            mask_size++;
            if (i == 32 || (uint32_t)(mask << i) == 0) break;  /* Go: mask<<32 == 0 for a uint32 */
        }
    }
    for (int i = 0; i < mask_size; i++) {
        const uint32_t bit = (old_r->dst_ip >> (31 - i)) & 1u;  /* DstIpAddr[i/8] >> (7 - i%8) */
        ora_node_t** child = bit ? &node->right : &node->left;
        if (!*child) *child = (ora_node_t*)calloc(1, sizeof(ora_node_t));
        node = *child;
    }
    /* newRouteList := make(..., 0, len(node.RouteList)): non-nil even when it ends up empty */
    uint32_t* list = (uint32_t*)malloc(sizeof(uint32_t) * (node->n + 1));
    uint32_t m = 0;
    for (uint32_t k = 0; k < node->n; k++) {
        const halo_route_entry_t* e = &t->routes[node->ids[k]];
        if (e->dst_ip == old_r->dst_ip && e->network_mask == old_r->network_mask && e->next_hop == old_r->next_hop &&
            e->netif == old_r->netif)
            continue;
        list[m++] = node->ids[k];
    }
    uint32_t id = UINT32_MAX;
    if (new_r) {
        if (t->n_routes == t->cap_routes) {
            t->cap_routes = t->cap_routes ? 2 * t->cap_routes : 64;
            t->routes = (halo_route_entry_t*)realloc(t->routes, sizeof(halo_route_entry_t) * t->cap_routes);
        }
        id = t->n_routes++;
        t->routes[id] = *new_r;
        list[m++] = id;
    }
    free(node->ids);
    node->ids = list;
    node->n = m;
    node->has_list = 1;
    return id;
}

/* Go hash/fnv New32a over the 4 address bytes */
static uint32_t fnv1a32(uint32_t ip) {
    uint32_t h = 2166136261u;
    for (int k = 0; k < 4; k++) {
        h ^= (ip >> (24 - 8 * k)) & 0xffu;
        h *= 16777619u;
    }
    return h;
}

/* FindRoute (engine/ipv4_engine.go:351-383): route id, HALO_ROUTE_NONE or HALO_ROUTE_PANIC */
ORA_API uint32_t ora_route_find(const ora_rt_t* t, uint32_t ip) {
    const ora_node_t* node = t->root;
    const ora_node_t* last = NULL;
    for (int i = 0; i < 32; i++) {
        if (node->has_list) last = node;
        const uint32_t bit = (ip >> (31 - i)) & 1u;
        const ora_node_t* next = bit ? node->right : node->left;
        if (!next) break;
        node = next;
    }
    if (node->has_list) last = node;
    if (!last) return HALO_ROUTE_NONE;
    if (last->n == 0) return HALO_ROUTE_PANIC;
    return last->ids[fnv1a32(ip) % last->n];
}

ORA_API void ora_route_find_batch(const ora_rt_t* t, const uint32_t* ips, uint32_t n, uint32_t* out) {
    for (uint32_t i = 0; i < n; i++) out[i] = ora_route_find(t, ips[i]);
}
