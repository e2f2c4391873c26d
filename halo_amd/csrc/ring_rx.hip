// ring_rx.hip — halo's SPSC packet ring as the source of a receive batch (SURVEY.md §8f row f1;
// BASELINE config 1 drains exactly such a ring through engine.Wire).
//
// The reference drains the ring one record per call: ReadPacket (mem/ring_buffer.go:298-352, the
// Go twin of cgo/ring_buffer.h:294-348) copies the next record into a reused 1514-byte buffer
// (dpdk.EthQueueRxPkt, dpdk/dpdk.go:183-199; engine.Wire.Rx, engine/engine.go:535-545) and
// PacketHandle parses it (engine/engine.go:339-351). Here a consumer takes everything between its
// cursor and the producer's head in one poll: the span goes to HBM raw (one DMA, two around the
// wrap), the GPU finds the record boundaries, the rx kernel (rx_parse.hip) parses the frames where
// they lie, and the records come back in one copy. The host reads `head`, writes `tail`, and never
// touches a frame byte.
//
// Record boundaries on the GPU. Walking records is a chain: the record whose length field is span
// dword a continues at a + ceil((4 + len) / 4) (u32 length + bytes, 4-byte aligned:
// mem/ring_buffer.go:47-50) unless ReadPacket would return false there. It is resolved over
// 4096-dword tiles by guess and verify:
//   A. guess  — every tile guesses where the walk enters it (the first position that passes
//               ReadPacket's checks and whose chain does not stop inside the tile; tile 0: the
//               span's start), walks from there and keeps its records and a summary;
//   B. link   — one workgroup checks the guesses by induction from tile 0 (tile t's guess is right
//               iff the verified walk through tile t - 1 enters t there), walks a tile again from
//               its real entry where the guess was wrong, and prefix-sums the records;
//   C. copy   — every tile writes its records as (dword offset, length) at its place.
// 0.033 ms for 1M 64 B records (68 MB). Three launches because a kernel boundary (~4.5 us) is
// cheaper here than workgroups waiting on each other's device-scope messages: one-launch walks
// (a linker workgroup; a decoupled look-back) and B + C in one launch were built, bit-exact, and
// measured slower.
// The previous resolution (tile maps of every entry position by pointer jumping, composed into
// superblocks, chained, expanded back down, then emitted: 0.19 ms against 0.033 for 1M 64 B
// records) is recorded in DESIGN.md §10.4 / §14.2 and was removed from the library.
// Every step applies ReadPacket's checks in ReadPacket's order, so the frames taken, the stop and
// the new tail are those of repeated ReadPacket calls (tests/test_gpu_ring.py, against the oracle,
// which tests/test_ring_oracle.py checks against the reference's own cgo/ring_buffer.h).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <new>
#include <thread>
#include <vector>

#include "halo_common.h"

namespace halo {
namespace {

constexpr uint32_t kTile = 4096;                 // span dwords per tile (16 KB)
constexpr uint32_t kThreads = 256;
constexpr uint32_t kLdsStop = 0x8000u;           // nxt entry: the walk stops at this position
constexpr uint32_t kMaxCapacity = 4 * kTile - 8; // the longest record must fit a tile's entry window
constexpr uint64_t kMaxSpan = (16ull << 30) - (64ull << 10);  // dword offsets stay below 2^32
constexpr uint64_t kPieceBytes = 16ull << 20;    // DMA piece (1024 tiles) whose maps start on arrival
constexpr uint64_t kSmallPoll = 4ull << 20;      // default: polls up to this size take the small path
constexpr uint64_t kSmallPollMax = 16ull << 20;

struct Scan {
    const uint32_t* span;   // the ring bytes [tail, tail + used) in stream order, as dwords
    uint32_t n_dw;          // used / 4
    uint32_t n_tiles;
    uint32_t cap;           // receive buffer capacity: len(data) of ReadPacket
    uint32_t max_frames;
    uint64_t half;          // RingBuffer.size / 2
    uint32_t half32;        // min(half, 2^32 - 1)
    uint32_t lim;           // min(half32, cap): the longest length a record may have
    uint32_t lim_dw;        // its dwords, (lim + 7) / 4
    uint2* tile_entry;      // [n_tiles]: (records before the tile, records the tile takes), from B
    struct RingCtl* ctl;    // total and the tile the walk ends in
    uint2* sum;             // [n_tiles]: (guess | exit << 16, records | why << 12 | longest << 16)
    uint32_t* tmp;          // [n_tiles][kTile / 2]: a tile's records, position | length << 16
    halo_rx_ring_scan_t* info;
    uint32_t* off_dw;       // frame i's bytes start at span dword off_dw[i]
    uint16_t* lens;
};

// Dwords of the record whose length field is span dword a (value `len`), or 0 where ReadPacket
// returns false, with the reason: the checks of mem/ring_buffer.go:309-335, in that order.
// 32-bit arithmetic throughout (the walk is VALU-bound): the record's dwords are
// ceil((4 + len) / 4) = (len >> 2) + 1 + (len & 3 != 0) without overflow, and size/2 is clamped
// to 2^32 - 1 (a u32 length can only exceed it when it is smaller).
__device__ __forceinline__ uint32_t record_dwords(const Scan& s, uint32_t a, uint32_t len, uint32_t& why) {
    if (a >= s.n_dw) { why = HALO_RING_STOP_EMPTY; return 0; }                                  // usedSpace < 4
    if (len == 0 || len > s.half32) { why = HALO_RING_STOP_BAD_LEN; return 0; }
    const uint32_t dw = (len >> 2) + 1u + ((len & 3u) != 0u);                                   // ringBufferRecordSize / 4
    if (s.n_dw - a < dw) { why = HALO_RING_STOP_PARTIAL; return 0; }                            // usedSpace < totalSize
    if (len > s.cap) { why = HALO_RING_STOP_CAPACITY; return 0; }                              // len(data) < packetLen
    return dw;
}

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

// Span dwords [a, a+4) (zero past the span's end).
__device__ __forceinline__ uint4 span_quad(const Scan& s, uint32_t a) {
    if (a + 4 <= s.n_dw) {
        const u32x4a4 x = *reinterpret_cast<const u32x4a4*>(s.span + a);
        return make_uint4(x.x, x.y, x.z, x.w);
    }
    return make_uint4(a < s.n_dw ? s.span[a] : 0u, a + 1 < s.n_dw ? s.span[a + 1] : 0u,
                      a + 2 < s.n_dw ? s.span[a + 2] : 0u, a + 3 < s.n_dw ? s.span[a + 3] : 0u);
}

// Tile tables. nxt[q]: the position of the record after the one whose length
// field is tile position q (bits 0-12; >= kTile: the next tile's position + kTile) with that
// length's low two bits (bits 13-14: with the record's dwords they give the length back), or
// kLdsStop when q fails ReadPacket's checks (the reason is worked out again, for the one position
// a walk stops at, by stop_why). list: the positions >= lo that pass.
constexpr uint32_t kListMax = kTile / 2;  // records of >= 2 dwords: at most this many per tile
constexpr uint32_t kNone = 0xFFFFu;      // tile summary: no position of the tile passes the checks
constexpr uint32_t kPosMask = 0x1FFFu;   // kTile + W - 1 < 2^13
constexpr uint32_t kGuessTries = 4;      // chains a tile tries as its guessed entry
static_assert(kTile + (kMaxCapacity + 7) / 4 <= kPosMask + 1, "nxt positions fit 13 bits");

// The length field of the record at tabulated position q (it passed the checks): its dwords and
// the low bits kept in nxt[q].
__device__ __forceinline__ uint32_t nxt_len(uint32_t q, uint32_t v) {
    const uint32_t dw = (v & kPosMask) - q, r = (v >> 13) & 3u;
    return ((dw - 1u - (r != 0u)) << 2) | r;
}

// Why ReadPacket stops at span dword a (a position whose nxt is kLdsStop).
__device__ __forceinline__ uint32_t stop_why(const Scan& s, uint32_t a) {
    uint32_t why = HALO_RING_STOP_EMPTY;
    if (a < s.n_dw) record_dwords(s, a, s.span[a], why);
    return why;
}

// One tile's tables, shared by the workgroup that walks it (12 KB: eight 4-wave workgroups per CU;
// a set per wave held the guess kernel at three waves per SIMD, 31 us for 1M 64 B records).
struct TileTab {
    uint16_t nxt[kTile];
    uint16_t list[kListMax];
    uint32_t part[16];  // per-wave candidate counts, then the first link break
    uint32_t cq[2];     // the walk's records and end, from the wave that walked serially
};

// Tabulates tile t (nxt, and list = the positions >= lo that pass, in order) with the whole
// workgroup of W waves; returns how many pass (list holds the first kListMax). Lane l of wave w
// takes the 16-byte chunks w * kTile / W + 256 u + 4 l: the tile's bytes are read once, with every
// load of a lane in flight together.
//
// The walk is VALU-bound here (round 5: 612 VALU a wave, 38 a position), so the common tile takes a
// shorter test: when the tile ends at least one longest record (lim = min(size / 2, capacity)) before
// the span does, a position passes exactly when 1 <= len <= lim — no record can run past the span
// from it, and EMPTY / PARTIAL cannot apply — which is one compare whose lane mask is also the
// position's ballot. The record's dwords are (len + 7) >> 2 (= ceil((4 + len) / 4)).
template <int W>
constexpr uint32_t kTabQ = kTile / (W * 256);  // 16-byte chunks per lane

template <int W>
__device__ __forceinline__ void tile_load(const Scan& s, uint32_t t, uint4 (&v)[kTabQ<W>]) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t at = t * kTile + w * (kTile / W) + 4 * lane;
    if (t * kTile + kTile <= s.n_dw) {  // uniform
#pragma unroll
        for (uint32_t u = 0; u < kTabQ<W>; ++u) {
            const u32x4a4 x = *reinterpret_cast<const u32x4a4*>(s.span + at + 256 * u);
            v[u] = make_uint4(x.x, x.y, x.z, x.w);
        }
    } else {
#pragma unroll
        for (uint32_t u = 0; u < kTabQ<W>; ++u) v[u] = span_quad(s, at + 256 * u);
    }
}

template <int W, bool INNER>
__device__ __forceinline__ uint32_t tabulate_as(const Scan& s, uint32_t t, TileTab& tb, uint32_t lo,
                                                const uint4 (&v)[kTabQ<W>]) {
    constexpr uint32_t Q = kTabQ<W>;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint32_t tbase = t * kTile, wbase = w * (kTile / W);
    bool m[Q][4];  // position q + j holds a record and is at or past lo
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t u = 0; u < Q; ++u) {
        const uint32_t q = wbase + 256 * u + 4 * lane;
        const uint32_t d[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        uint32_t nx[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            bool pass;
            if constexpr (INNER) {
                pass = d[j] - 1u < s.lim;
            } else {
                uint32_t why;
                pass = record_dwords(s, tbase + q + j, d[j], why) != 0;
            }
            nx[j] = pass ? ((q + j + ((d[j] + 7u) >> 2)) | ((d[j] & 3u) << 13)) : kLdsStop;
            m[u][j] = pass && q + j >= lo;
            cnt += (uint32_t)__popcll(__ballot(m[u][j]));
        }
        *reinterpret_cast<uint2*>(&tb.nxt[q]) = make_uint2(nx[0] | (nx[1] << 16), nx[2] | (nx[3] << 16));
    }
    if (lane == 0) tb.part[w] = cnt;
    __syncthreads();
    uint32_t n_act = 0, k = 0;  // this wave's first list slot: the candidates of the waves before
#pragma unroll
    for (uint32_t x = 0; x < (uint32_t)W; ++x) {
        k += x < w ? tb.part[x] : 0u;
        n_act += tb.part[x];
    }
    // ordered compaction (wave, then chunk, then lane, then j)
#pragma unroll
    for (uint32_t u = 0; u < Q; ++u) {
        uint32_t slot = k, total = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // + the candidates of the lanes before this one
            const uint64_t b = __ballot(m[u][j]);
            slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, slot));
            total += (uint32_t)__popcll(b);
        }
        const uint32_t q = wbase + 256 * u + 4 * lane;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (m[u][j] && slot < kListMax) tb.list[slot] = (uint16_t)(q + j);
            slot += m[u][j] ? 1u : 0u;
        }
        k += total;
    }
    __syncthreads();
    return n_act;
}

template <int W>
__device__ __forceinline__ uint32_t tile_tabulate(const Scan& s, uint32_t t, TileTab& tb, uint32_t lo,
                                                  const uint4 (&v)[kTabQ<W>]) {
    if ((uint64_t)t * kTile + kTile + s.lim_dw <= s.n_dw) return tabulate_as<W, true>(s, t, tb, lo, v);  // uniform
    return tabulate_as<W, false>(s, t, tb, lo, v);
}

template <int W>
__device__ __forceinline__ uint32_t tile_tabulate(const Scan& s, uint32_t t, TileTab& tb, uint32_t lo) {
    uint4 v[kTabQ<W>];
    tile_load<W>(s, t, v);
    return tile_tabulate<W>(s, t, tb, lo, v);
}

// The first "break" at list index >= i0: the first listed candidate whose link does not reach the
// next listed one (the last one always breaks). The chain through the listed candidates from
// list[i0] is list[i0..F]; it goes on at nxt[list[F]].
template <int W>
__device__ __forceinline__ uint32_t first_break(TileTab& tb, uint32_t n_act, uint32_t i0) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    uint32_t f = ~0u;
    for (uint32_t i = i0 + tid; i < n_act; i += 64 * W)
        if ((tb.nxt[tb.list[i]] & kPosMask) != (i + 1 < n_act ? tb.list[i + 1] : 0xFFFFu)) {
            f = i;
            break;
        }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) f = min(f, (uint32_t)__shfl_xor((int)f, m, 64));
    if (lane == 0) tb.part[w] = f;
    __syncthreads();
    uint32_t F = n_act - 1;
#pragma unroll
    for (uint32_t x = 0; x < (uint32_t)W; ++x) F = min(F, tb.part[x]);
    __syncthreads();  // part is rewritten by the next call
    return F;
}

// The walk through a tabulated tile from `entry` = list[i0] (or a position that fails the checks
// or is not listed: then it takes nothing), by the whole workgroup: list[i0 .. i0 + c) become its
// records (at most `limit`) and q the position after the last one (>= kTile: it continues in the
// next tile; < kTile: it stops there, nxt[q] says why). Fast path: in ring data the positions that
// pass ReadPacket's checks are, almost always, exactly the record starts, each linking to the
// next, so the walk is list[i0..F] — found by one parallel pass over the links instead of one
// dependent LDS read per record. A position that passes the checks but is not on the chain (a
// record decoy in a payload) shows up as a link that skips over it; wave 0 then walks serially from
// where the links end.
struct TileWalk {
    uint32_t c, q;
};
template <int W>
__device__ __forceinline__ TileWalk tile_walk(TileTab& tb, uint32_t n_act, uint32_t i0, uint32_t entry,
                                              uint32_t limit, uint32_t known_F = ~0u) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    uint32_t c = 0, q = entry;
    bool serial = n_act > kListMax;  // too many candidates to list: walk serially from the entry
    if (!serial && i0 < n_act && tb.list[i0] == entry) {  // uniform
        const uint32_t F = known_F != ~0u ? known_F : first_break<W>(tb, n_act, i0), M = F + 1 - i0;
        c = min(M, limit);
        q = c < M ? tb.list[i0 + c] : tb.nxt[tb.list[F]] & kPosMask;
        // the chain goes on at a position past a decoy: continue serially from there
        serial = c == M && c < limit && q < kTile && !(tb.nxt[q] & kLdsStop);
    }
    if (serial) {  // uniform
        if (w == 0) {
            // the lanes follow the same chain (values made scalar): uniform control flow around one
            // dependent LDS read per record
            while (c < limit && q < kTile) {
                const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane((int)tb.nxt[q]);
                if (v & kLdsStop) break;
                tb.list[i0 + c++] = (uint16_t)q;
                q = v & kPosMask;
            }
            if (lane == 0) {
                tb.cq[0] = c;
                tb.cq[1] = q;
            }
        }
        __syncthreads();
        c = tb.cq[0];
        q = tb.cq[1];
    }
    __syncthreads();  // cq / list are reused by the caller's next tile
    return TileWalk{c, q};
}

__device__ __forceinline__ uint32_t len_dwords(uint32_t len) { return (len >> 2) + 1u + ((len & 3u) != 0u); }

constexpr uint32_t kTileWaves = kThreads / 64;

// ---- the record walk by guess and verify (the default) ------------------------------------------
// A. Every tile guesses its entry — the first position that passes ReadPacket's checks (tile 0:
//    the span's start) — walks from it (tile_walk) and keeps the records it found in its slot of
//    the workspace, with a summary: (guess, where the walk leaves or stops, records, why, longest).
// B. One workgroup links the summaries: tile t's guess is right when the walk through tile t - 1
//    (itself verified) enters tile t there. By induction from tile 0 every guess that matches is
//    the real entry, so a chunk of 8192 tiles is settled by one comparison per tile and a prefix
//    sum; a tile whose guess is wrong (a decoy in the record that straddles its start) is walked
//    again by the workgroup from its real entry, and the linking goes on after it.
// C. Every tile copies its records to (dword offset, length) at its place in the batch.
// Three launches, each tile read once (the map path it replaces: seven launches and a serial chain
// of map lookups between them, 0.19 ms for 1M 64 B records, profiles/r05/r5f).
struct RingCtl {
    uint32_t last_tile;  // the tile the walk ends in
    uint32_t n;          // records taken (min(total, max_frames)): C reads (last_tile, n) in one load
    uint32_t total;      // records the walk takes before it stops (max_frames ignored)
};

// A tile's walk into its workspace slot (position | length << 16) and its longest record.
__device__ __forceinline__ uint32_t keep_records(const Scan& s, uint32_t t, const TileTab& tb, uint32_t i0,
                                                 uint32_t c) {
    uint32_t* tmp = s.tmp + (uint64_t)t * kListMax;
    uint32_t mx = 0;
    for (uint32_t j = threadIdx.x; j < c; j += blockDim.x) {
        const uint32_t e = tb.list[i0 + j], len = nxt_len(e, tb.nxt[e]);
        tmp[j] = e | (len << 16);
        mx = max(mx, len);
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, m, 64));
    return mx;  // the wave's
}

// One tile of A: its tables, its guess, its walk, its records and summary.
template <int W>
__device__ __forceinline__ void guess_tile(const Scan& s, uint32_t t, TileTab& tb, uint32_t* s_mx,
                                           const uint4 (&v)[kTabQ<W>]) {
    const uint32_t tid = threadIdx.x;
    const uint32_t n_act = tile_tabulate<W>(s, t, tb, 0, v);
    // The guess: the first listed candidate whose chain of links does not stop inside the tile. The
    // dword before a record is often a decoy — a frame's last bytes and zero padding make a small
    // "length" (1.3 % of IMIX tiles, tools: a 570 B frame's last dword) — whose link lands nowhere;
    // such a chain is skipped. If every try stops, the first candidate (the walk may really stop).
    uint32_t i0 = 0, F0 = ~0u;  // the chosen chain: its first listed index and its first break
    if (t > 0 && n_act <= kListMax) {
        for (uint32_t k = 0, tries = 0; k < n_act && tries < kGuessTries; ++tries) {  // uniform
            const uint32_t F = first_break<W>(tb, n_act, k), q = tb.nxt[tb.list[F]] & kPosMask;
            if (!(q < kTile && (tb.nxt[q] & kLdsStop))) {
                i0 = k;
                F0 = F;
                break;
            }
            k = F + 1;
        }
    }
    const uint32_t g = t == 0 ? 0u : n_act ? tb.list[i0] : kNone;
    TileWalk wk{0, kNone};
    if (g != kNone) wk = tile_walk<W>(tb, n_act, i0, g, kListMax, F0);  // uniform (tile 0: i0 = 0)
    const uint32_t mx = keep_records(s, t, tb, i0, wk.c);
    if ((tid & 63u) == 0) s_mx[tid >> 6] = mx;
    __syncthreads();
    if (tid == 0) {
        uint32_t m = 0;
        for (uint32_t x = 0; x < (uint32_t)W; ++x) m = max(m, s_mx[x]);
        const uint32_t why = wk.q < kTile ? stop_why(s, t * kTile + wk.q) : 0u;
        s.sum[t] = make_uint2(g | (wk.q << 16), wk.c | (why << 12) | (m << 16));
    }
}

#ifndef HALO_RING_GUESS_WAVES
#define HALO_RING_GUESS_WAVES 4  // waves per tile in A
#endif
constexpr uint32_t kGuessWaves = HALO_RING_GUESS_WAVES;

__global__ void __launch_bounds__(kGuessWaves * 64) ring_guess_kernel(const Scan s) {
    __shared__ TileTab tb;
    __shared__ uint32_t s_mx[kGuessWaves];
    // (one tile per workgroup: workgroups that took tiles t, t + 2048, ... and loaded the next
    // one's bytes while working on the current one ran slower, 24.9 against 19.0 us for 1M 64 B
    // records, profiles/r05/r5zc: the tile's work, not its load, is what a CU waits on)
    uint4 v[kTabQ<kGuessWaves>];
    tile_load<kGuessWaves>(s, blockIdx.x, v);
    guess_tile<kGuessWaves>(s, blockIdx.x, tb, s_mx, v);
}

#ifndef HALO_RING_LINK_THREADS
#define HALO_RING_LINK_THREADS 512  // 1024: 8.7 us, 256: 10.6, 512: 8.0 for 1M 64 B records (profiles/r05/r5zt)
#endif
constexpr uint32_t kLinkThreads = HALO_RING_LINK_THREADS, kLinkWaves = kLinkThreads / 64, kLinkPer = 16;  // 512: a chunk spans 128 MB
constexpr uint32_t kLinkChunk = kLinkThreads * kLinkPer;

// B's second walk of tile J from its real entry `jin` (the guess was wrong): its records to the
// workspace, and (records, exit, why, longest) to s_fix.
__device__ __forceinline__ void relink_tile(const Scan& s, uint32_t J, uint32_t jin, TileTab& tb,
                                                      uint32_t* s_part, uint32_t* s_fix) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t n_act = tile_tabulate<kLinkWaves>(s, J, tb, jin);
    const TileWalk wk = tile_walk<kLinkWaves>(tb, n_act, 0, jin, kListMax);
    const uint32_t m = keep_records(s, J, tb, 0, wk.c);
    if (lane == 0) s_part[wv] = m;
    __syncthreads();
    if (tid == 0) {
        uint32_t mm = 0;
        for (uint32_t k = 0; k < kLinkWaves; ++k) mm = max(mm, s_part[k]);
        s_fix[0] = wk.c;
        s_fix[1] = wk.q;
        s_fix[2] = wk.q < kTile ? stop_why(s, J * kTile + wk.q) : 0u;
        s_fix[3] = mm;
    }
}

__global__ void __launch_bounds__(kLinkThreads) ring_link_kernel(const Scan s) {
    __shared__ TileTab tb;
    __shared__ uint32_t s_min[kLinkWaves], s_sum[kLinkWaves];
    __shared__ uint32_t s_q[kLinkThreads];  // each thread's last tile's exit (its successor's entry)
    __shared__ uint32_t s_fix[4];           // the special tile's records, exit, why, longest record
    __shared__ uint32_t s_cut[2];           // the tile (and records before it) max_frames cuts inside
    __shared__ uint32_t s_sj[3];            // the special tile's summary and the exit of the one before
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t mf = s.max_frames, nt = s.n_tiles;
    uint32_t t0 = 0, e = 0, base = 0;  // the next tile to link, its entry, records before it (uniform)
    uint32_t why = HALO_RING_STOP_EMPTY, last = 0;
    uint32_t mx = 0;  // the longest record of this thread's tiles that lie wholly before max_frames
    if (tid == 0) s_cut[0] = ~0u;
    // a tile's records counted into the batch: all of them, the first ones (max_frames cuts inside
    // it: its longest comes from its records at the end), or none
    auto account = [&](uint32_t j, uint32_t b, uint32_t c, uint32_t m) {
        if (b + c <= mf) mx = max(mx, m);
        else if (b < mf) {
            s_cut[0] = j;
            s_cut[1] = b;
        }
    };
    for (;;) {
        // A chunk of kLinkChunk tiles from t0, kLinkPer summaries a thread in registers: the first
        // tile that cannot be passed on its summary ("special": the entry the tile before leads to
        // is not the guess, the walk stops inside, or the span's last tile) and the records of the
        // ones before it. After a special tile the next chunk starts behind it (a re-read of the
        // summaries, from the L2): keeping the chunk's state across a tile's second walk instead
        // spilled at 1024 threads (70 us, profiles/r05/r5k).
        const uint32_t j0 = t0 + tid * kLinkPer;
        uint2 sm[kLinkPer];
        if (j0 + kLinkPer <= nt && !(reinterpret_cast<uintptr_t>(s.sum) & 15u)) {  // two summaries a load
#pragma unroll
            for (uint32_t k = 0; k < kLinkPer; k += 2) {
                const uint4 v = *reinterpret_cast<const uint4*>(s.sum + j0 + k);
                sm[k] = make_uint2(v.x, v.y);
                sm[k + 1] = make_uint2(v.z, v.w);
            }
        } else {
#pragma unroll
            for (uint32_t k = 0; k < kLinkPer; ++k) sm[k] = j0 + k < nt ? s.sum[j0 + k] : make_uint2(kNone, 0u);
        }
        uint32_t prev_q = 0;
        if (j0 > t0 && j0 <= nt) prev_q = s.sum[j0 - 1].x >> 16;
        uint32_t first = ~0u, fx = 0, fy = 0, fpe = 0;  // this thread's first special tile: summary, exit before
#pragma unroll
        for (uint32_t k = 0; k < kLinkPer; ++k) {
            const uint32_t j = j0 + k, g = sm[k].x & 0xFFFFu, q = sm[k].x >> 16;
            const uint32_t in = j == t0 ? e : prev_q - kTile;  // wraps (no match) when prev_q < kTile
            const bool special = j >= nt || in != g || q < kTile || j == nt - 1;
            if (special && first == ~0u) {
                first = j;
                fx = sm[k].x;
                fy = sm[k].y;
                fpe = prev_q;
            }
            prev_q = q;
        }
        const uint32_t my_first = first;
        s_q[tid] = prev_q;
        // block: the first special tile J (every chunk that reaches the span's last tile has one)
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) first = min(first, (uint32_t)__shfl_xor((int)first, m, 64));
        if (lane == 0) s_min[wv] = first;
        __syncthreads();
        uint32_t J = ~0u;
        for (uint32_t k = 0; k < kLinkWaves; ++k) J = min(J, s_min[k]);
        // an exclusive prefix of the records of the tiles before J
        uint32_t cnt = 0;
#pragma unroll
        for (uint32_t k = 0; k < kLinkPer; ++k) cnt += j0 + k < J ? sm[k].y & 0xFFFu : 0u;
        uint32_t x = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) s_sum[wv] = x;
        __syncthreads();
        uint32_t off = 0, chunk_total = 0;
        for (uint32_t k = 0; k < kLinkWaves; ++k) {
            if (k < wv) off += s_sum[k];
            chunk_total += s_sum[k];
        }
        uint32_t b = base + off + x - cnt;
#pragma unroll
        for (uint32_t k = 0; k < kLinkPer; ++k) {
            const uint32_t j = j0 + k, c = sm[k].y & 0xFFFu;
            if (j < J) {
                s.tile_entry[j] = make_uint2(b, c);
                account(j, b, c, sm[k].y >> 16);
                b += c;
            }
        }
        base += chunk_total;
        if (J == ~0u) {  // no special tile in the chunk (it ended before the span's last tile)
            e = s_q[kLinkThreads - 1] - kTile;
            t0 += kLinkChunk;
            __syncthreads();
            continue;
        }
        // J's summary and the exit of the tile before it, from the thread that found J (no reload)
        if (my_first == J) {
            s_sj[0] = fx;
            s_sj[1] = fy;
            s_sj[2] = fpe;
        }
        __syncthreads();
        const uint32_t jin = J == t0 ? e : s_sj[2] - kTile;  // J's real entry
        const uint2 sj = make_uint2(s_sj[0], s_sj[1]);
        __syncthreads();  // s_q / s_min / s_sum / s_sj are rewritten below and by the next chunk
        if ((sj.x & 0xFFFFu) == jin) {  // uniform. The guess was right: the walk stops in J, or J is the last tile
            if (tid == 0) {
                s_fix[0] = sj.y & 0xFFFu;
                s_fix[1] = sj.x >> 16;
                s_fix[2] = (sj.y >> 12) & 0xFu;
                s_fix[3] = sj.y >> 16;
            }
        } else {  // a decoy led the guess astray: walk J again from its real entry
            relink_tile(s, J, jin, tb, s_min, s_fix);
        }
        __syncthreads();
        const uint32_t c = s_fix[0], q = s_fix[1];
        if (tid == 0) {
            s.tile_entry[J] = make_uint2(base, c);
            account(J, base, c, s_fix[3]);
        }
        base += c;
        if (q < kTile || J == nt - 1) {  // stopped in J, or left the span (EMPTY)
            why = q < kTile ? s_fix[2] : HALO_RING_STOP_EMPTY;
            last = J;
            break;
        }
        t0 = J + 1;
        e = q - kTile;
        __syncthreads();
    }
    // the longest record taken: every whole tile's, and the cut tile's records before max_frames
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, m, 64));
    __syncthreads();
    if (lane == 0) s_min[wv] = mx;
    uint32_t mc = 0;
    if (s_cut[0] != ~0u) {
        const uint32_t* tmp = s.tmp + (uint64_t)s_cut[0] * kListMax;
        for (uint32_t j = tid; j < mf - s_cut[1]; j += kLinkThreads) mc = max(mc, tmp[j] >> 16);
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) mc = max(mc, (uint32_t)__shfl_xor((int)mc, o, 64));
    if (lane == 0) s_sum[wv] = mc;
    __syncthreads();
    if (tid == 0) {
        uint32_t m = 0;
        for (uint32_t k = 0; k < kLinkWaves; ++k) m = max(m, max(s_min[k], s_sum[k]));
        const uint32_t n = min(base, mf);
        s.ctl->total = base;
        s.ctl->last_tile = last;
        s.ctl->n = min(base, mf);
        halo_rx_ring_scan_t info;
        info.n_frames = n;
        info.stop = n < base ? HALO_RING_STOP_MAX : why;
        info.end_bytes = 0;  // C: the position after record n - 1
        info.max_len = m;
        info.pad = 0;
        *s.info = info;
    }
}

__global__ void __launch_bounds__(kThreads) ring_copy_kernel(const Scan s) {
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t t = blockIdx.x * kTileWaves + w;
    // the three reads in one round trip (the tile's entry read before the walk's end is known)
    const uint64_t tw = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(s.tile_entry + t));  // whole-workgroup padded
    const uint2 te = make_uint2((uint32_t)tw, (uint32_t)(tw >> 32));
    const uint2 ln = *reinterpret_cast<const uint2*>(s.ctl);  // (last_tile, n)
    const uint32_t last = ln.x, n = ln.y;
    if (t > last) return;  // wave-uniform: tiles past the walk's end hold nothing
    const uint32_t base = te.x;
    if (base >= n) return;
    const uint32_t cnt = min(te.y, n - base), tbase = t * kTile;
    const uint32_t* tmp = s.tmp + (uint64_t)t * kListMax;
    for (uint32_t j = lane; j < cnt; j += 64) {
        const uint32_t v = tmp[j], pos = v & 0xFFFFu, len = v >> 16;
        s.off_dw[base + j] = tbase + pos + 1;
        s.lens[base + j] = (uint16_t)len;
        if (base + j == n - 1) s.info->end_bytes = 4ull * (tbase + pos + len_dwords(len));
    }
}

struct Geom {
    uint32_t n_dw, n_tiles;
    uint64_t sum_off, tmp_off, tile_entry_off, total_off, bytes;
};

Geom geometry(uint64_t used, uint32_t cap) {
    Geom g{};
    g.n_dw = (uint32_t)(used >> 2);
    g.n_tiles = std::max<uint32_t>(1, (g.n_dw + kTile - 1) / kTile);
    (void)cap;
    uint64_t o = 0;
    g.sum_off = o;
    o += (uint64_t)g.n_tiles * sizeof(uint2);
    g.tmp_off = o;
    o += (uint64_t)g.n_tiles * kListMax * sizeof(uint32_t);
    g.tile_entry_off = o;
    o += (uint64_t)(g.n_tiles + kTileWaves - 1) / kTileWaves * kTileWaves * sizeof(uint2);  // C reads whole workgroups
    g.total_off = o;
    o += 256;
    g.bytes = o;
    return g;
}

Scan make_scan(const Geom& g, const uint8_t* d_span, uint64_t ring_size, uint32_t cap, uint32_t max_frames,
               uint8_t* ws, halo_rx_ring_scan_t* d_info, uint32_t* d_off, uint16_t* d_len) {
    Scan s{};
    s.span = reinterpret_cast<const uint32_t*>(d_span);
    s.n_dw = g.n_dw;
    s.n_tiles = g.n_tiles;
    s.cap = cap;
    s.max_frames = max_frames;  // 0: no frame may be taken
    s.half = ring_size / 2;
    s.half32 = (uint32_t)std::min<uint64_t>(s.half, 0xFFFFFFFFull);
    s.lim = std::min(s.half32, cap);
    s.lim_dw = (uint32_t)(((uint64_t)s.lim + 7) / 4);
    s.tile_entry = reinterpret_cast<uint2*>(ws + g.tile_entry_off);
    s.ctl = reinterpret_cast<RingCtl*>(ws + g.total_off);
    s.sum = reinterpret_cast<uint2*>(ws + g.sum_off);
    s.tmp = reinterpret_cast<uint32_t*>(ws + g.tmp_off);
    s.info = d_info;
    s.off_dw = d_off;
    s.lens = d_len;
    return s;
}

// The record walk of a span: the guess / link / copy kernels.
int launch_walk(const Scan& s, hipStream_t st) {
    hipLaunchKernelGGL(ring_guess_kernel, dim3(s.n_tiles), dim3(kGuessWaves * 64), 0, st, s);
    hipLaunchKernelGGL(ring_link_kernel, dim3(1), dim3(kLinkThreads), 0, st, s);
    hipLaunchKernelGGL(ring_copy_kernel, dim3((s.n_tiles + kTileWaves - 1) / kTileWaves), dim3(kThreads), 0, st, s);
    return hipGetLastError() == hipSuccess ? HALO_OK : HALO_E_HIP;
}

}  // namespace
}  // namespace halo

using halo::Geom;
using halo::Scan;

struct halo_rx_ring {
    int device = 0;
    uint8_t* mem = nullptr;   // the RingBuffer header; the data area follows
    uint8_t* data = nullptr;
    uint64_t size = 0;
    uint64_t cursor = 0;      // stream position after the frames polled so far
    uint32_t cap = 0, max_frames = 0;
    uint64_t max_bytes = 0;
    bool registered = false;
    Geom g{};                 // workspace geometry for max_bytes
    hipStream_t s_copy = nullptr, s_comp = nullptr, s_d2h = nullptr;
    std::vector<hipEvent_t> ev;  // per piece: copy landed, parse done
    uint8_t* d_span = nullptr;
    uint8_t* d_ws = nullptr;
    uint32_t* d_off = nullptr;
    uint16_t* d_len = nullptr;
    halo_rx_result_t* d_res = nullptr;
    uint32_t* d_hist = nullptr;
    halo_rx_ring_scan_t* d_info = nullptr;
    halo_rx_ring_scan_t* h_info = nullptr;  // pinned
    uint32_t* h_off = nullptr;              // pinned
    // small path (registered rings): the ring's data area as the device sees it, and pinned
    // (offset, length, record) arrays for up to small_frames frames
    uint8_t* d_data = nullptr;
    uint64_t small = 0;
    uint32_t small_frames = 0;
    uint32_t* h_soff = nullptr;
    uint16_t* h_slen = nullptr;
    halo_rx_result_t* h_sres = nullptr;
    uint32_t* d_soff = nullptr;
    uint16_t* d_slen = nullptr;
    halo_rx_result_t* d_sres = nullptr;
    // HALO_RING_PERSISTENT: the resident small-poll consumer (resident.hip, rx_parse.hip
    // ring_service_kernel) over the ring's data area and the pinned offset / length arrays
    halo::Resident* svc = nullptr;
    halo_rx_ring_stats_t stats{};
};

namespace {
// Returns false when the ring memory could not be unregistered (the caller must not free it then:
// the pages stay mapped for the device).
bool free_ring(halo_rx_ring* r) {
    halo::ParkUsed park(r->device);  // hipFree waits for the device's kernels, hipHostFree for every device's
    halo::resident_destroy(r->svc);      // stops the consumer and waits for its kernel to end
    for (hipEvent_t e : r->ev)
        if (e) (void)hipEventDestroy(e);
    if (r->s_copy) (void)hipStreamDestroy(r->s_copy);
    if (r->s_comp) (void)hipStreamDestroy(r->s_comp);
    if (r->s_d2h) (void)hipStreamDestroy(r->s_d2h);
    if (r->d_span) (void)hipFree(r->d_span);
    if (r->d_ws) (void)hipFree(r->d_ws);
    if (r->d_off) (void)hipFree(r->d_off);
    if (r->d_len) (void)hipFree(r->d_len);
    if (r->d_res) (void)hipFree(r->d_res);
    if (r->d_hist) (void)hipFree(r->d_hist);
    if (r->d_info) (void)hipFree(r->d_info);
    if (r->h_info) (void)hipHostFree(r->h_info);
    if (r->h_off) (void)hipHostFree(r->h_off);
    if (r->h_soff) (void)hipHostFree(r->h_soff);
    if (r->h_slen) (void)hipHostFree(r->h_slen);
    if (r->h_sres) (void)hipHostFree(r->h_sres);
    bool ok = true;
    if (r->registered) ok = halo::host_reg_remove(r->mem, halo::kRegRing) == HALO_OK;
    delete r;
    return ok;
}

// Device address of host memory [p, p + bytes) when it is pinned or registered in one piece,
// else nullptr (the failed query's error is cleared so later launch checks do not see it).
void* device_view(const void* p, uint64_t bytes) {
    void *d0 = nullptr, *d1 = nullptr;
    if (!p || !bytes) return nullptr;
    if (hipHostGetDevicePointer(&d0, const_cast<void*>(p), 0) != hipSuccess ||
        hipHostGetDevicePointer(&d1, const_cast<uint8_t*>(static_cast<const uint8_t*>(p)) + bytes - 1, 0) !=
            hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint8_t*>(d1) - static_cast<uint8_t*>(d0) == (ptrdiff_t)(bytes - 1) ? d0 : nullptr;
}

int alloc_small(halo_rx_ring* r, uint64_t bytes) {
    const uint32_t frames = (uint32_t)std::min<uint64_t>(bytes / 8, r->max_frames);
    if (frames > r->small_frames) {
        halo::ParkUsed park(r->device);  // hipHostFree waits for kernels on every device
        if (r->h_soff) (void)hipHostFree(r->h_soff);
        if (r->h_slen) (void)hipHostFree(r->h_slen);
        if (r->h_sres) (void)hipHostFree(r->h_sres);
        r->h_soff = nullptr;
        r->h_slen = nullptr;
        r->h_sres = nullptr;  // allocated on first use: only for callers whose array is not mapped
        r->d_sres = nullptr;
        r->small_frames = 0;
        r->d_soff = nullptr;
        r->d_slen = nullptr;
        if (r->svc) halo::resident_set_arrays(r->svc, r->d_data, nullptr, nullptr);  // freed above
        // on failure the small path is switched off (small = 0): every later poll takes the pipelined
        // path instead of walking with no arrays and returning nothing
        r->small = 0;
        if (hipHostMalloc((void**)&r->h_soff, 4ull * frames, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&r->h_slen, 2ull * frames, hipHostMallocDefault) != hipSuccess)
            return HALO_E_NOMEM;
        r->d_soff = static_cast<uint32_t*>(device_view(r->h_soff, 4ull * frames));
        r->d_slen = static_cast<uint16_t*>(device_view(r->h_slen, 2ull * frames));
        if (!r->d_soff || !r->d_slen) {
            r->d_soff = nullptr;
            r->d_slen = nullptr;
            return HALO_E_NOMEM;
        }
        r->small_frames = frames;
        if (r->svc) halo::resident_set_arrays(r->svc, r->d_data, r->d_soff, r->d_slen);
    }
    r->small = bytes;
    return HALO_OK;
}

// The small path (BASELINE config 1: 1k-frame batches through engine.Wire). The host reads the
// records' length fields exactly as ReadPacket does (mem/ring_buffer.go:309-335: 4 bytes per
// record, never a frame byte); one rx launch then parses the frames where they lie in the
// registered ring, over PCIe, and writes the records straight into the caller's array when that
// is pinned or registered. One launch and one synchronisation replace the span DMA, the seven
// walk launches, the info round trip and the record copies of the pipelined path, which are
// latency, not bandwidth, at this size. Returns 1 (nothing done) when a frame wraps around the end
// of the data area: that poll takes the pipelined path, which linearises the span.
int small_poll(halo_rx_ring* r, uint64_t used, uint32_t flags, const halo_rx_netif_t* netif,
               halo_rx_result_t* out, uint32_t* status_hist, uint64_t* positions, halo_rx_ring_scan_t* info) {
    // every record is >= 8 bytes and used <= small, so at most small_frames frames fit: the bound
    // below never cuts a walk, it only keeps the pinned arrays' size in the contract
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const halo::RingWalk w = halo::ring_walk(r->data, r->size, r->cursor, used, r->cap,
                                             std::min(r->max_frames, r->small_frames), r->h_soff, r->h_slen, positions);
    const auto t1 = clk::now();
    if (w.wraps) return 1;
    r->stats.walk_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    ++r->stats.small_polls;
    const uint32_t n = w.n, max_len = w.max_len;
    if (n) {
        const uint64_t rb = sizeof(halo_rx_result_t) * (uint64_t)n;
        // looked up per poll (not cached): the caller may unregister or reuse the array between polls.
        // A registration made through the library is found in its registry without a runtime call
        // (two hipHostGetDevicePointer calls per poll otherwise); other pinned memory by the runtime.
        auto* dout = static_cast<halo_rx_result_t*>(halo::host_reg_device_view(out, rb));
        if (!dout) dout = static_cast<halo_rx_result_t*>(device_view(out, rb));
        if (!dout && !r->h_sres) {
            const uint64_t sb = sizeof(halo_rx_result_t) * (uint64_t)r->small_frames;
            if (hipHostMalloc((void**)&r->h_sres, sb, hipHostMallocDefault) != hipSuccess) return HALO_E_NOMEM;
            if (!(r->d_sres = static_cast<halo_rx_result_t*>(device_view(r->h_sres, sb)))) return HALO_E_NOMEM;
        }
        // one length and consecutive records (no wrap between the first and the last): frame i at
        // off_dw[0] + i * stride, passed as the strided layout (no offset / length arrays to read)
        const uint32_t stride = (4u + max_len + 3u) >> 2;
        const bool uni = w.min_len == max_len &&
                         (int64_t)r->h_soff[n - 1] - (int64_t)r->h_soff[0] == (int64_t)(n - 1) * stride;
        int rc = halo::kResidentParked;
        if (r->svc && n <= halo::kSvcMaxFrames)
            rc = halo::resident_request(r->svc, n, flags, netif, dout ? dout : r->d_sres, uni ? r->h_soff[0] : 0u,
                                        uni ? stride : 0u, uni ? max_len : 0u);
        if (rc == halo::kResidentParked) {  // no resident consumer, or a device drain has it parked
            rc = uni ? halo_rx_parse_strided_device(r->d_data + 4ull * r->h_soff[0], 4ull * stride, nullptr, max_len, n,
                                                    flags, netif, dout ? dout : r->d_sres, nullptr, r->s_comp)
                     : halo_rx_parse_batch_device(r->d_data, r->d_soff, r->d_slen, n, flags, netif, max_len,
                                                  dout ? dout : r->d_sres, nullptr, r->s_comp);
            if (!rc && hipStreamSynchronize(r->s_comp) != hipSuccess) rc = HALO_E_HIP;
        }
        r->stats.wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t1).count();
        if (rc) return rc;
        if (!dout) memcpy(out, r->h_sres, rb);
        if (status_hist)
            for (uint32_t i = 0; i < n; ++i) ++status_hist[out[i].status];  // the statuses the kernel wrote
    }
    info->n_frames = n;
    info->stop = w.stop;
    info->end_bytes = w.end_bytes;
    info->max_len = max_len;
    r->cursor += w.end_bytes;
    r->stats.polls += n != 0;
    r->stats.frames += n;
    return HALO_OK;
}
}  // namespace

extern "C" HALO_API uint64_t halo_rx_ring_scan_workspace(uint64_t used, uint32_t capacity) {
    if (capacity == 0) capacity = halo::kEthMax;
    if (capacity > halo::kMaxCapacity || used > halo::kMaxSpan) return 0;
    return halo::geometry(used, capacity).bytes;
}

extern "C" HALO_API int halo_rx_ring_scan_device(const uint8_t* d_span, uint64_t used, uint64_t ring_size,
                                                 uint32_t capacity, uint32_t max_frames, uint32_t* d_offsets_dw,
                                                 uint16_t* d_lens, halo_rx_ring_scan_t* d_info, void* d_workspace,
                                                 uint64_t workspace_bytes, halo_stream_t stream) {
    if (!d_info) return HALO_E_INVAL;
    if (capacity == 0) capacity = halo::kEthMax;
    if (capacity > halo::kMaxCapacity || !halo::pow2(ring_size)) return HALO_E_INVAL;
    if ((used & 3u) || used > ring_size || used > halo::kMaxSpan) return HALO_E_INVAL;
    const Geom g = halo::geometry(used, capacity);
    if (used && (!d_span || !d_offsets_dw || !d_lens || (reinterpret_cast<uintptr_t>(d_span) & 3u) ||
                 !d_workspace || workspace_bytes < g.bytes))
        return HALO_E_INVAL;
    int rc = halo::check_device();
    if (rc) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (used == 0)
        return hipMemsetAsync(d_info, 0, sizeof(halo_rx_ring_scan_t), st) == hipSuccess ? HALO_OK : HALO_E_HIP;
    const Scan s = halo::make_scan(g, d_span, ring_size, capacity, max_frames ? max_frames : 0xFFFFFFFFu,
                                   static_cast<uint8_t*>(d_workspace), d_info, d_offsets_dw, d_lens);
    return halo::launch_walk(s, st);
}

// The walk + parse stream, at the device's highest priority: its workgroups are placed ahead of
// the record copies' blit waves as CUs free up (profiles/r01/ab_r3x_ring_e2e.log).
static bool comp_stream(hipStream_t* st) {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
        return hipStreamCreateWithPriority(st, hipStreamNonBlocking, hi) == hipSuccess;
    return hipStreamCreateWithFlags(st, hipStreamNonBlocking) == hipSuccess;
}

extern "C" HALO_API int halo_rx_ring_attach(int device, void* ring_mem, int64_t offset, uint32_t capacity,
                                            uint64_t max_bytes, uint32_t max_frames, uint32_t attach_flags,
                                            halo_rx_ring_t** out) {
    if (!out) return HALO_E_INVAL;
    *out = nullptr;
    uint64_t size = 0, tail = 0;
    uint8_t* mem = static_cast<uint8_t*>(ring_mem);
    int rc = halo::validate_ring(mem, offset, &size, &tail);
    if (rc) return rc;
    if (attach_flags & ~(HALO_RING_REGISTER | HALO_RING_PERSISTENT)) return HALO_E_INVAL;
    if ((attach_flags & HALO_RING_PERSISTENT) && !(attach_flags & HALO_RING_REGISTER)) return HALO_E_INVAL;
    // a registered ring pins the whole pages it spans: it must start on a page of its own
    const uint64_t page = halo::host_page_size();
    const uint64_t reg_bytes = (halo::kRbHeader + size + page - 1) / page * page;
    if ((attach_flags & HALO_RING_REGISTER) && (reinterpret_cast<uintptr_t>(mem) % page)) return HALO_E_INVAL;
    if (capacity == 0) capacity = halo::kEthMax;
    if (capacity > halo::kMaxCapacity) return HALO_E_INVAL;
    if (max_bytes == 0) max_bytes = std::min<uint64_t>(size, 256ull << 20);
    max_bytes = std::min<uint64_t>(std::min<uint64_t>(max_bytes, size), halo::kMaxSpan) & ~3ull;
    if (max_bytes < 8) return HALO_E_INVAL;
    if (max_frames == 0 || max_frames > max_bytes / 8) max_frames = (uint32_t)std::min<uint64_t>(max_bytes / 8, 0xFFFFFFFFull);
    if ((rc = halo_rx_init(device))) return rc;
    halo::ParkUsed park(device);  // allocations, registration (and a failed attach's frees: hipHostFree waits on every device)
    auto* r = new (std::nothrow) halo_rx_ring;
    if (!r) return HALO_E_NOMEM;
    r->device = device;
    r->mem = mem;
    r->data = mem + halo::kRbHeader;
    r->size = size;
    r->cursor = tail;
    r->cap = capacity;
    r->max_frames = max_frames;
    r->max_bytes = max_bytes;
    r->g = halo::geometry(std::min<uint64_t>(max_bytes, halo::kPieceBytes + 4ull * halo::kTile), capacity);  // a piece + a cut record
    r->ev.assign(2 * (size_t)((max_bytes + halo::kPieceBytes - 1) / halo::kPieceBytes), nullptr);
    bool ok = hipStreamCreateWithFlags(&r->s_copy, hipStreamNonBlocking) == hipSuccess &&
              comp_stream(&r->s_comp) &&
              hipStreamCreateWithFlags(&r->s_d2h, hipStreamNonBlocking) == hipSuccess;
    for (auto& e : r->ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->d_span, max_bytes + 16) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->d_ws, r->g.bytes) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->d_off, 4ull * max_frames) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->d_len, 2ull * max_frames) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->d_res, sizeof(halo_rx_result_t) * (uint64_t)max_frames) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->d_hist, 4 * HALO_RX_STATUS_COUNT) == hipSuccess;
    // complete before any non-blocking stream counts into it (a stream wait, not a device drain: a
    // resident consumer elsewhere on the device would hold a device synchronisation for 20 ms)
    ok = ok && hipMemsetAsync(r->d_hist, 0, 4 * HALO_RX_STATUS_COUNT, r->s_comp) == hipSuccess &&
         hipStreamSynchronize(r->s_comp) == hipSuccess;
    ok = ok && hipMalloc((void**)&r->d_info, sizeof(halo_rx_ring_scan_t)) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&r->h_info, sizeof(halo_rx_ring_scan_t), hipHostMallocDefault) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&r->h_off, 4ull * max_frames, hipHostMallocDefault) == hipSuccess;
    int reg_rc = HALO_OK;
    if (ok && (attach_flags & HALO_RING_REGISTER)) {
        reg_rc = halo::host_reg_add(mem, reg_bytes, halo::kRegRing);  // INVAL: shares a page with a live one
        ok = reg_rc == HALO_OK;
        r->registered = ok;
        if (ok && size <= halo::kMaxSpan + (64ull << 10)) {  // dword offsets into the data area fit u32
            r->d_data = static_cast<uint8_t*>(device_view(r->data, size));
            ok = !r->d_data || alloc_small(r, halo::kSmallPoll) == HALO_OK;
        }
        if (ok && (attach_flags & HALO_RING_PERSISTENT) && r->d_data)
            ok = halo::resident_create(device, r->d_data, r->d_soff, r->d_slen, &r->svc) == HALO_OK;
    }
    if (!ok) {
        free_ring(r);
        return reg_rc != HALO_OK ? reg_rc : HALO_E_NOMEM;
    }
    *out = r;
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_ring_detach(halo_rx_ring_t* r) {
    if (!r) return HALO_E_INVAL;
    (void)hipSetDevice(r->device);
    if (r->s_copy) (void)hipStreamSynchronize(r->s_copy);
    if (r->s_comp) (void)hipStreamSynchronize(r->s_comp);
    if (r->s_d2h) (void)hipStreamSynchronize(r->s_d2h);
    return free_ring(r) ? HALO_OK : HALO_E_HIP;
}

// One poll, pipelined over 16 MiB pieces of the span: every piece's H2D copy is queued at once on
// the copy stream; piece k is then walked from the record boundary where piece k-1's walk ended
// (a record crossing a piece end is simply PARTIAL there and taken with the next piece), parsed
// where it lies and its records copied back on a third stream — so the walk, the parse and the
// record copies of piece k overlap the transfer of the pieces after it.
extern "C" HALO_API int halo_rx_ring_poll(halo_rx_ring_t* r, uint32_t flags, const halo_rx_netif_t* netif,
                                          halo_rx_result_t* out, uint32_t* status_hist, uint64_t* positions,
                                          halo_rx_ring_scan_t* info) {
    if (!r || !netif || !out || !info) return HALO_E_INVAL;
    if (flags & ~(HALO_RX_CSUM_ENABLE | HALO_RX_JUMBO_EXT)) return HALO_E_INVAL;
    if (hipSetDevice(r->device) != hipSuccess) return HALO_E_NODEV;
    memset(info, 0, sizeof *info);
    const uint64_t head = __atomic_load_n(reinterpret_cast<const uint64_t*>(r->mem), __ATOMIC_ACQUIRE);
    uint64_t used = head - r->cursor;
    if (used > r->size) {  // ReadPacket: usedSpace > size -> false
        info->stop = HALO_RING_STOP_BAD_CURSOR;
        return HALO_OK;
    }
    used = std::min(used, r->max_bytes) & ~3ull;
    if (used == 0) return HALO_OK;  // EMPTY
    if (used <= r->small && r->d_data) {
        const int rc = small_poll(r, used, flags, netif, out, status_hist, positions, info);
        if (rc <= 0) return rc;  // 1: a frame wraps around the data area's end -> pipelined path
    }
    const uint64_t mask = r->size - 1, pos = r->cursor & mask;
    const uint32_t n_pieces = (uint32_t)((used + halo::kPieceBytes - 1) / halo::kPieceBytes);
    int rc = HALO_OK;
    // 1. every piece's copy, in order, on the copy stream
    for (uint32_t k = 0; k < n_pieces && rc == HALO_OK; ++k) {
        const uint64_t b0 = (uint64_t)k * halo::kPieceBytes, b1 = std::min(used, b0 + halo::kPieceBytes);
        uint64_t src = (pos + b0) & mask, len = b1 - b0, dst = b0;
        while (len && rc == HALO_OK) {  // up to the end of the data area, then from its start
            const uint64_t c = std::min(len, r->size - src);
            if (hipMemcpyAsync(r->d_span + dst, r->data + src, c, hipMemcpyHostToDevice, r->s_copy) != hipSuccess)
                rc = HALO_E_HIP;
            dst += c;
            len -= c;
            src = 0;
        }
        if (!rc && hipEventRecord(r->ev[2 * k], r->s_copy) != hipSuccess) rc = HALO_E_HIP;
    }
    // 2. walk, parse and return piece by piece
    uint64_t off = 0;         // span bytes consumed: the record boundary the next walk starts at
    uint32_t done = 0;        // frames taken
    std::vector<std::pair<uint32_t, uint64_t>> spans;  // (first frame, span offset) per piece (positions)
    for (uint32_t k = 0; k < n_pieces && rc == HALO_OK; ++k) {
        const uint64_t avail = std::min(used, (uint64_t)(k + 1) * halo::kPieceBytes) - off;
        if (hipStreamWaitEvent(r->s_comp, r->ev[2 * k], 0) != hipSuccess) { rc = HALO_E_HIP; break; }
        const Geom g = halo::geometry(avail, r->cap);
        const Scan sc = halo::make_scan(g, r->d_span + off, r->size, r->cap, r->max_frames - done, r->d_ws, r->d_info,
                                        r->d_off + done, r->d_len + done);
        if ((rc = halo::launch_walk(sc, r->s_comp))) break;
        if (hipMemcpyAsync(r->h_info, r->d_info, sizeof *info, hipMemcpyDeviceToHost, r->s_comp) != hipSuccess ||
            hipStreamSynchronize(r->s_comp) != hipSuccess) { rc = HALO_E_HIP; break; }
        const halo_rx_ring_scan_t pi = *r->h_info;
        if (pi.n_frames) {
            spans.emplace_back(done, off);
            rc = halo_rx_parse_batch_device(r->d_span + off, r->d_off + done, r->d_len + done, pi.n_frames, flags,
                                            netif, pi.max_len, r->d_res + done, status_hist ? r->d_hist : nullptr,
                                            r->s_comp);
            if (rc) break;
            if (hipEventRecord(r->ev[2 * k + 1], r->s_comp) != hipSuccess ||
                hipStreamWaitEvent(r->s_d2h, r->ev[2 * k + 1], 0) != hipSuccess ||
                hipMemcpyAsync(out + done, r->d_res + done, sizeof(halo_rx_result_t) * pi.n_frames,
                               hipMemcpyDeviceToHost, r->s_d2h) != hipSuccess) { rc = HALO_E_HIP; break; }
        }
        done += pi.n_frames;
        off += pi.end_bytes;
        info->max_len = std::max(info->max_len, pi.max_len);
        info->stop = pi.stop;
        // a record cut by the piece's end (PARTIAL) or a piece ending on a record boundary
        // (EMPTY) continues with the next piece; anything else ends the walk
        if (pi.stop != HALO_RING_STOP_PARTIAL && pi.stop != HALO_RING_STOP_EMPTY) break;
    }
    if (!rc && positions && done &&
        hipMemcpyAsync(r->h_off, r->d_off, 4ull * done, hipMemcpyDeviceToHost, r->s_d2h) != hipSuccess)
        rc = HALO_E_HIP;
    if (hipStreamSynchronize(r->s_copy) != hipSuccess && !rc) rc = HALO_E_HIP;
    if (hipStreamSynchronize(r->s_comp) != hipSuccess && !rc) rc = HALO_E_HIP;
    if (hipStreamSynchronize(r->s_d2h) != hipSuccess && !rc) rc = HALO_E_HIP;
    if (rc) return rc;
    if (positions) {
        for (size_t j = 0; j < spans.size(); ++j) {
            const uint32_t f1 = j + 1 < spans.size() ? spans[j + 1].first : done;
            for (uint32_t i = spans[j].first; i < f1; ++i)
                positions[i] = r->cursor + spans[j].second + 4ull * (r->h_off[i] - 1u);
        }
    }
    if (status_hist && done) {
        uint32_t h[HALO_RX_STATUS_COUNT];
        // on the stream the parses ran on: hipMemset / hipMemcpy go to the null stream, which a
        // non-blocking stream does not wait for (a reset could land after the next poll's counts)
        if (hipMemcpyAsync(h, r->d_hist, sizeof h, hipMemcpyDeviceToHost, r->s_comp) != hipSuccess ||
            hipMemsetAsync(r->d_hist, 0, sizeof h, r->s_comp) != hipSuccess ||
            hipStreamSynchronize(r->s_comp) != hipSuccess)
            return HALO_E_HIP;
        for (int j = 0; j < HALO_RX_STATUS_COUNT; ++j) status_hist[j] += h[j];
    }
    info->n_frames = done;
    info->end_bytes = off;
    r->cursor += off;
    r->stats.polls += done != 0;
    r->stats.frames += done;
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_ring_get_stats(const halo_rx_ring_t* r, halo_rx_ring_stats_t* out) {
    if (!r || !out) return HALO_E_INVAL;
    *out = r->stats;
    if (r->svc) {
        const halo::ResidentStats s = halo::resident_stats(r->svc);
        out->service_requests = s.requests;
        out->service_launches = s.launches;
        out->service_gpu_ns = s.gpu_ns;
    }
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_ring_set_service_timeout(halo_rx_ring_t* r, uint64_t us) {
    if (!r || !r->svc) return HALO_E_INVAL;
    halo::resident_set_timeout(r->svc, us);
    return HALO_OK;
}

extern "C" HALO_API int halo_rx_ring_set_small_poll(halo_rx_ring_t* r, uint64_t bytes) {
    if (!r || bytes > halo::kSmallPollMax) return HALO_E_INVAL;
    if (bytes && !r->d_data) return HALO_E_INVAL;  // needs a ring attached with HALO_RING_REGISTER
    if (hipSetDevice(r->device) != hipSuccess) return HALO_E_NODEV;
    if (!bytes) {
        r->small = 0;
        return HALO_OK;
    }
    return alloc_small(r, bytes);
}

extern "C" HALO_API int halo_rx_ring_commit(halo_rx_ring_t* r) {
    if (!r) return HALO_E_INVAL;
    __atomic_store_n(reinterpret_cast<uint64_t*>(r->mem + 64), r->cursor, __ATOMIC_RELEASE);
    return HALO_OK;
}

// ---- several devices, one host batch ------------------------------------------
extern "C" HALO_API int halo_rx_shard_multi(halo_rx_host_ctx_t* const* ctxs, uint32_t n_ctx, const uint8_t* bytes,
                                            const uint64_t* offsets, const uint16_t* lens, uint32_t n, uint32_t flags,
                                            const halo_rx_netif_t* netif, halo_rx_result_t* out,
                                            uint32_t* status_hist, uint32_t* shard_first) {
    if (!ctxs || n_ctx == 0 || n_ctx > 1024 || !netif) return HALO_E_INVAL;
    for (uint32_t k = 0; k < n_ctx; ++k)
        if (!ctxs[k]) return HALO_E_INVAL;
    if (n && (!bytes || !offsets || !lens || !out)) return HALO_E_INVAL;
    // contiguous index ranges balanced by frame bytes
    std::vector<uint32_t> first(n_ctx + 1, n);
    halo::shard_bounds(lens, n, n_ctx, first.data());
    if (shard_first)
        for (uint32_t j = 0; j <= n_ctx; ++j) shard_first[j] = first[j];
    std::vector<int> rcs(n_ctx, HALO_OK);
    std::vector<std::vector<uint32_t>> hists(n_ctx, std::vector<uint32_t>(HALO_RX_STATUS_COUNT, 0));
    auto run = [&](uint32_t j) {
        const uint32_t f0 = first[j], cnt = first[j + 1] - first[j];
        if (cnt)
            rcs[j] = halo_rx_parse_batch_host(ctxs[j], bytes, offsets + f0, lens + f0, cnt, flags, netif, out + f0,
                                              status_hist ? hists[j].data() : nullptr);
    };
    std::vector<std::thread> th;
    th.reserve(n_ctx);
    for (uint32_t j = 1; j < n_ctx; ++j) th.emplace_back(run, j);
    run(0);
    for (auto& t : th) t.join();
    for (uint32_t j = 0; j < n_ctx; ++j)
        if (rcs[j]) return rcs[j];
    if (status_hist)
        for (uint32_t j = 0; j < n_ctx; ++j)
            for (int s = 0; s < HALO_RX_STATUS_COUNT; ++s) status_hist[s] += hists[j][s];
    return HALO_OK;
}
