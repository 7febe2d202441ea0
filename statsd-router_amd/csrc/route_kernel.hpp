// route_kernel.hpp — device side of the MI355X statsd-router hot path (included by sr_route.hip
// and by tools/ablate_route.hip; everything lives in namespace srk).
//
// Reference path (hulu/statsd-router, /root/reference):
//   udp_read_cb        sr-main.c:149-191  framing + newline tokeniser + length gate 5 < L < 1450
//   process_data_line  sr-main.c:137-147  ':' presence -> INVALID_FORMAT
//   hash               sr-main.c:120-134  sdbm over the name (signed char, u64 wrap)
//   find_downstream    sr-main.c:86-117   hash-seeded partial Fisher-Yates probe over alive shards
//
// Input: a batch of framed datagrams back to back in HBM. Every framed datagram ends in '\n'
// (host framing, sr_frame_datagram), so the lines of the batch are its '\n'-terminated pieces and
// datagram boundaries are irrelevant here. Output: one 8-byte sr_record per line, in input order.
//
// One kernel, one pass over the bytes:
//   * A launch routes up to 32 batches. Blocks 0 .. nb-1 are per-batch SCANNERS; every other block
//     routes one 16 KiB TILE with 256 threads (4 waves), 64 contiguous bytes per thread, up to 7
//     workgroups per CU (71-72 VGPRs, ~22.5 KiB of LDS). With 8+ batches each batch's tiles and its
//     scanner share one XCD class (blocks b and b + 8 land on the same XCD).
//   * Tile entry: four buffer_load_dwordx4 per thread (+ 2 KiB of halo before the tile) into a padded
//     LDS image (17-dword rows: conflict-free per-thread rows); '\n' and ':' bit masks of the
//     thread's 64 bytes from the load registers (8 VALU per dword for both patterns); the tile's '\n'
//     count published at once in a status granule for the scanner.
//   * Record numbering: the scanner polls its batch's tile counts (two polls in flight, 64 tiles per
//     poll) and publishes each tile's first record index (bases granule: plain store when the tile
//     shares the scanner's XCD, sc1 otherwise); a second scanner wave does the stores. A tile reads
//     its base part-way through its hashing, long after it is normally published; a tile that never
//     published within a spin budget is counted by the scanner itself (no dispatch-order assumption).
//   * Line state per thread (lines before its chunk, first ':' of the line open at its start) from
//     two u32 DPP wave scans plus the earlier waves' totals; the line straddling into the tile (at
//     most one) is located in the halo (or in global memory for lines longer than it).
//   * Lines, in windows of 256 tile-local lines: (end, first ':') staged in LDS, then every line
//     hashed from the LDS image: sdbm with SDWA byte-pair products and one 64x64 multiply per 8
//     bytes (sdbm_img), a name of n bytes being ceil(n/64) 64-byte segments combined with K^len.
//     Two lane layouts, one instantiation each (identical records): KV_UNIFORM gives every line of
//     a tile the same G lanes (from the tile's mean line length); KV_SEGMENTS gives a tile of mixed
//     lengths one lane per segment, lines packed back to back over the lanes, a line's hash the
//     difference of an inclusive wave scan of segment hashes (route_host.hpp picks per launch).
//   * Shard pick: h % N through a 64-bit magic reciprocal when every shard is alive; otherwise the
//     reference's probe: its first two picks here (reciprocals and alive words in LDS pad dwords),
//     a line needing a third deferred by record index to probe_defer_kernel (16-entry register
//     overlay), and one needing more than 16 dead probes to probe_wide_kernel (the probe on a full
//     LDS permutation). The dead shards the probes visit (sr-main.c:106) are noted by the probes
//     themselves (LDS words per tile, ORed per batch by probe_defer_kernel); beyond 1024 shards
//     probed_dead_kernel replays the probes from the hashes after the launch.
//   * Every workgroup arrives on 8-way sharded counters without waiting; the last block waits for
//     all arrivals and advances the context's epoch, so stale granules of earlier launches are never
//     mistaken for current ones, with or without graph replay.
// No MFMA: HBM-bound byte work on VALU + LDS.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sr_route.h"

namespace srk {

constexpr int kBlock = 256;                  // threads per workgroup of the product kernel (4 waves)
constexpr int kLaneBytes = 64;               // bytes per lane
constexpr int kTile = kBlock * kLaneBytes;   // 16 KiB per tile
constexpr int kOverlay = 16;                 // register overlay entries of the probe
constexpr int kNone = 0x1FFFF;               // "no colon" marker (above any tile position)
constexpr int kSpinBudget = 1 << 14;         // polls before a missing predecessor is proxied
constexpr uint32_t kFlagAgg = 1u, kFlagIncl = 2u;
constexpr uint16_t kRoutePending = 0xFFFCu;  // internal: resolved by probe_defer_kernel / probe_wide_kernel
constexpr uint32_t kRouteDefer = 0xFFFBu;    // internal: probe_shard stopped after its first two picks
constexpr uint64_t K = 65599ull;             // sdbm multiplier: (h<<6)+(h<<16)-h (sr-main.c:131)
constexpr int kPowLo = 64, kPowHi = 24;     // K^i (i < 64) and K^(64 i) (i < 24: exponents below 1536)
constexpr int kPowInv = 4;                   // K^-z (z < 4)

// ablation switches (tools/ablate_route.hip); the product instantiates ABL_NONE
enum : unsigned {
    ABL_NONE = 0,
    ABL_NO_LOOKBACK = 1u,   // base = 0 (records overwrite each other)
    ABL_NO_LINES = 2u,      // skip per-line staging / hashing / records
    ABL_NO_PROLOGUE = 4u,   // skip the straddling-line prologue
    ABL_NO_SCAN = 8u,       // skip masks/Horner/scans (counts only)
    ABL_LOAD_ONLY = 16u,    // load the tile into LDS and count '\n' only
    ABL_STAMPS = 32u,       // diagnostic: s_memrealtime at phase boundaries into RouteParams::dbg
    ABL_NO_XCD_LOCAL = 64u, // deal every launch's tiles round-robin even when it has 8+ batches
    ABL_NO_HASH = 256u,     // ablation: skip the sdbm (h = 0); staging, probe and records stay
    ABL_LDS_PAD = 131072u,  // occupancy experiment: 4 KiB of unused LDS per workgroup
    ABL_OLD_MASKS = 65536u,  // round-1 v0.5 piece masks (one SWAR test per pattern)
    ABL_OLD_SCANNER = 32768u, // round-1 v0.5 scanner: one wave polls and publishes
    ABL_FAKE_BASE = 4096u,  // ablation: base = t * (this tile's count), exact only for uniform tiles (C2)
    ABL_EARLY_BASE = 2048u,  // also read the record base when staging ends (round-1 v0.6a/b; no gain once
                             // the pipelined scanner publishes ahead of need)
    ABL_AGENT_GRANULES = 262144u,  // every count / base granule stored sc1 (round-1 v0.5), whatever the XCDs
    ABL_SCAN_SERIAL = 524288u,  // round-1 v0.6 scanner: 256 granules per round trip, one poll in flight
    ABL_NO_MID_BASE = 2097152u,  // no base read part-way through the hash (round-1 v0.8)
    ABL_OLD_HASH = 1024u,   // round-1 v0.5 per-segment sdbm (v_alignbyte reads, compiler-extracted bytes)
};

// Product kernel variants (same records, bit for bit): KV_SEGMENTS lays a tile of mixed line
// lengths out one lane per 64-byte name segment (route_host.hpp picks the variant per launch).
// KV_ALIVE: a launch whose every shard is alive (the shard is h % N): no probe, overlay, deferral or
// probed-dead marks in the kernel, and none of their registers.
// KV_PICKS: a launch with dead shards whose probes end after the first picks (one dead shard: two
// picks always find a live one; two or more: the deferral of probe_defer_kernel) runs a variant
// with chunk_probe in place of probe_shard, whose 16-entry overlay loop it cannot reach.
enum : unsigned { KV_UNIFORM = 0u, KV_SEGMENTS = 4194304u, KV_ALIVE = 268435456u, KV_PICKS = 536870912u };
// KV_DEFER1: the common dead-shard launch, two or more of at most 64 shards dead with every probe that
// meets a dead shard deferred after one pick (probe_defer_kernel redoes it whole and notes the dead
// shards it visits): the probe is h % N and one test of the alive word (a kernel argument), with no
// reciprocal or alive pads in LDS, no marks and no pending list (a variant of the picks-only and
// chunk kernels).
constexpr unsigned KV_DEFER1 = 2147483648u;
// KV_DEAD1: exactly one dead shard (RouteParams::dead_k): find_downstream's two picks in closed form,
// the second pick's reciprocal a kernel argument (magic_n1), no alive or reciprocal pads in LDS.
constexpr unsigned KV_DEAD1 = 134217728u;
// KV_HIST1: the KV_DEAD1 uniform / segment variant that also counts the tile histograms of a route + pack
// launch (RouteParams::hist); a variant of its own because the counting costs the route-only variant
// 3 % in SGPR spills (every-shard-alive variants count them at no cost)
constexpr unsigned KV_HIST1 = 1048576u;
template <unsigned ABL>
constexpr bool kCountsHist = (ABL & KV_ALIVE) != 0 || ((ABL & KV_DEAD1) != 0 && (ABL & KV_HIST1) != 0);

constexpr uint64_t ipow(uint64_t b, unsigned e) {
    uint64_t r = 1;
    while (e) {
        if (e & 1) r *= b;
        b *= b;
        e >>= 1;
    }
    return r;
}
constexpr uint64_t inv_odd(uint64_t a) {  // a^-1 mod 2^64 for odd a (Newton)
    uint64_t x = a;
    for (int i = 0; i < 6; ++i) x *= 2 - a * x;
    return x;
}
constexpr uint64_t kK16 = ipow(K, 16), kK32 = ipow(K, 32), kK48 = ipow(K, 48), kK64 = ipow(K, 64);
constexpr uint64_t kK4096 = ipow(K, 4096);
constexpr uint64_t kK4 = ipow(K, 4);
constexpr int32_t kK2lo = (int32_t)(K * K - (1ull << 32));   // K^2 = 2^32 + 0x7E0F81
static_assert(K * K == (1ull << 32) + 0x7E0F81ull, "K^2 split");
constexpr uint64_t kKinv = inv_odd(K);
static_assert(K * kKinv == 1ull, "K inverse");

struct Magic {          // exact n / d for 64-bit n (Granlund-Montgomery, round-up variant)
    uint64_t m;
    uint32_t shift;
    uint32_t kind;      // 0: q = n >> shift; 1: q = mulhi >> shift; 2: add-indicator form
};

struct PendingLine {
    uint32_t rec;
    uint32_t batch;
    uint64_t hash;
};

// Per-context device control block, zeroed once at sr_open. Counters on separate 128-B lines.
struct Control {
    uint32_t epoch;
    uint32_t pad1;
    uint32_t pending;
    uint32_t pad0[29];
    uint32_t done[8][32];
    uint64_t scan_xcc[32];   // per batch: the XCD its scanner runs on (kFlagXcc granule)
    uint32_t layout[8][32];  // KV_SEGMENTS launches, sharded: [0] tiles that weighed the segment
                             // layout, [1] tiles it saves two or more rounds (published per launch
                             // by the last block)
};

// One batch of a launch. A launch routes up to kMaxBatches independent batches: tiles
// [tile0, tile0 + ntiles) of the grid belong to batch i, each batch with its own look-back chain
// (status granules at the same grid indices) and its own records and line count.
constexpr int kMaxBatches = 32;
constexpr int kHistKeys = 17;  // RouteParams::hist: up to 16 shards + the unrouted key
constexpr int kPerClass = 8;   // batches per XCD class: <= 4 with 8+ batches (XCD-local), <= 7 below
struct BatchDesc {
    const uint8_t *bytes;
    sr_record *recs;
    uint64_t *hashes;        // may be null
    uint64_t *n_out;         // device: line count of the batch
    uint32_t nbytes;
    uint32_t max_records;
    uint32_t tile0;          // first tile in its XCD class's sequence (class 0 only: the launch's)
    uint32_t ntiles;
    uint32_t sbase;          // first status / base granule of the batch
    uint32_t cls;            // XCD class: the tiles of the batch are blocks nb + cls + 8 i
    uint32_t pad;
    uint64_t *probed_dead;   // may be null: bit k set = dead shard k was probed by some line
                             // (find_downstream zeroes its active buffer, sr-main.c:106)
    uint64_t *dhash;         // RouteParams::defer: the hashes of deferred lines, by record index
};

struct RouteParams {
    uint32_t nb;             // batches in this launch
    uint32_t total_blocks;   // grid size: nb scanners + every batch's tiles (+ padding blocks)
    uint32_t xcd_local;      // 1: tile blocks dealt to 8 XCD classes, each batch within one class
    uint32_t nds;            // number of downstreams
    uint32_t dead;           // dead downstreams in the alive snapshot
    uint32_t pending_cap;
    uint32_t nwords_check;   // probed_dead_kernel: bitmap words checked for completion (0: never)
    uint32_t nwords;         // alive / probed-dead bitmap words
    uint32_t defer;          // probes past their first `picks` picks are deferred (probe_defer_kernel)
    uint32_t picks;          // with defer: picks the route kernel makes itself (1 or 2)
    uint32_t mark;           // the probes note the dead shards they visit (sr-main.c:106), for the bitmaps
    uint32_t mark_tiles;     // ... the route kernel's too (LDS words, then its tile slot): not when every
                             // probe that meets a dead shard is deferred (one pick), which probe_defer_kernel
                             // then redoes whole, noting its dead picks itself
    Magic magic_n;           // for h % nds (fast path)
    const uint64_t *alive;   // bitmap
    const Magic *magic;      // [0..nds], index i -> divisor i
    const uint64_t *kpow;    // kPowLo + kPowHi + kPowInv entries: K^i (i < 64), K^(64 i) (i < 24), K^-z (z < 4)
    Control *ctl;
    uint64_t *status;        // per-tile '\n' count granules {epoch, flag, count} (written by the tile)
    uint64_t *bases;         // per-tile first-record granules {epoch, flag, base} (written by the scanner)
    PendingLine *pending;
    uint64_t *tile_pd;       // mark: per tile (status granule index), its probed-dead words
    uint64_t *dbg;           // ABL_STAMPS builds only: 16 timestamp slots per tile
    uint32_t *layout_out;    // host-mapped {sequence, tiles weighed, tiles segmented} of the last
                             // KV_SEGMENTS launch (null: not published)
    // route_chunk_kernel (chunk_kernel.hpp): K^-z (z <= 64), then per lane K^(64 (255 - l)) and
    // K^-(64 (255 - l)); per tile the tail-line granules {meta, hash lo, hash hi, -}; polls of a
    // predecessor's tail granules before the tile computes that line itself (0: always)
    const uint64_t *cpow;
    uint64_t *tail;
    uint32_t lb_spin;
    uint32_t pad_lb;
    // route_chunk_kernel (SR_KNOB_PREFETCH): a tile workgroup also touches one dword per 128-byte line of
    // the tile `prefetch` tiles further on in its batch (the one its XCD runs about that many tiles
    // later), so that tile's loads find it in L2 / the memory-side cache; 0: off
    uint32_t prefetch;
    uint32_t pad_pf;
    uint64_t alive_w0;       // KV_DEFER1: the alive bitmap's first word (nds <= 64)
    Magic magic_n1;          // KV_DEAD1: for h % (nds - 1)
    uint32_t dead_k;         // KV_DEAD1: the dead shard
    uint32_t pad_dk;
    // route + pack launches (sr_route_pack_many; every shard alive, at most kHistKeys - 1 shards): per
    // tile its records' key histogram (shard, or nds = unrouted), key-major per batch at
    // hist[(nds + 1) * sbase + key * ntiles + t], for the packing's sort (mtu_kernel.hpp); null: off
    uint32_t *hist;
    // per block residue r = B mod 8, the batches of the tiles those blocks run, in tile order:
    // (the first B / 8 past the batch's tiles << 6) | batch index; ~0u after the last (one scalar
    // load, issued with the header's, finds a tile's batch: launch_header_batch)
    uint32_t cls_tab[8][kPerClass];
    BatchDesc b[kMaxBatches];
};

// ---------------------------------------------------------------------------------------
// Helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t sdbm_step(uint64_t h, uint32_t byte) {
    // sr-main.c:131: h = (h << 6) + (h << 16) - h + c, with c a *signed* char (sr-main.c:122)
    const int64_t c = (int8_t)byte;
    return (h << 16) + (h << 6) - h + (uint64_t)c;
}

// Four Horner steps at once (bytes in memory order = little-endian byte order of x):
//   h*K^4 + (c0*K + c1)*K^2 + (c2*K + c3),   K^2 = 2^32 + 0x7E0F81.
// The pair terms are exact 32-bit multiply-adds; only the final step needs 64-bit multiplies,
// so the dword costs one 64x64 product instead of four (the 64-bit multiplies are the slow ops).
__device__ __forceinline__ uint64_t sdbm_dword(uint64_t h, uint32_t x) {
    const int32_t c0 = (int8_t)(x & 0xFFu), c1 = (int8_t)((x >> 8) & 0xFFu);
    const int32_t c2 = (int8_t)((x >> 16) & 0xFFu), c3 = (int8_t)(x >> 24);
    const int32_t t = c0 * (int32_t)K + c1;
    const int32_t u = c2 * (int32_t)K + c3;
    const uint64_t d = (uint64_t)((int64_t)t * kK2lo) + (uint64_t)(int64_t)u + ((uint64_t)(uint32_t)t << 32);
    return h * kK4 + d;
}

// Signed-byte pair products by SDWA (byte select + sign extension folded into the VALU op):
// c0 * K + c1 and c2 * K + c3 for the bytes c0..c3 of x, two instructions each.
__device__ __forceinline__ int32_t pair_lo(uint32_t x) {
    int32_t t;
    asm("v_mul_i32_i24_sdwa %0, sext(%1), %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD\n\t"
        "v_add_u32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
        : "=&v"(t)
        : "v"(x), "v"((int32_t)K));
    return t;
}
__device__ __forceinline__ int32_t pair_hi(uint32_t x) {
    int32_t t;
    asm("v_mul_i32_i24_sdwa %0, sext(%1), %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD\n\t"
        "v_add_u32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
        : "=&v"(t)
        : "v"(x), "v"((int32_t)K));
    return t;
}

// sdbm_dword with the pair products from SDWA: 11 VALU per dword.
__device__ __forceinline__ uint64_t sdbm_dword_fast(uint64_t h, uint32_t x) {
    const int32_t t = pair_lo(x);
    const int32_t u = pair_hi(x);
    const uint64_t d = (uint64_t)((int64_t)t * kK2lo + (int64_t)u) + ((uint64_t)(uint32_t)t << 32);
    return h * kK4 + d;
}

// A 64-bit constant C as C_lo + 2^32 C_hi with C_lo a signed 32-bit value, so that for a signed
// 32-bit t, t * C = t * C_lo (one v_mad_i64_i32) + 2^32 (t * C_hi) (mod 2^64).
struct SplitK {
    int32_t lo;
    uint32_t hi;
};
constexpr SplitK split_k(uint64_t c) {
    const uint32_t lo = (uint32_t)c;
    return lo >= 0x80000000u ? SplitK{(int32_t)(lo - 0x80000000u) - (int32_t)0x7FFFFFFF - 1, (uint32_t)(c >> 32) + 1u}
                             : SplitK{(int32_t)lo, (uint32_t)(c >> 32)};
}
constexpr SplitK kS4 = split_k(ipow(K, 4)), kS6 = split_k(ipow(K, 6));
constexpr uint64_t kK8 = ipow(K, 8);

// Eight Horner steps (the bytes of x0 then x1): h K^8 + t1 K^6 + u1 K^4 + t2 K^2 + u2, with t, u the
// SDWA pair products of x0 and x1. The pair terms go straight onto the accumulator by
// v_mad_i64_i32 (low constant word) plus a 32-bit product into the high word, so the eight bytes
// cost one 64x64 product (h K^8) instead of two: 18-19 VALU per 8 bytes against 22.
__device__ __forceinline__ uint64_t sdbm_qword_fast(uint64_t h, uint32_t x0, uint32_t x1) {
    const int32_t t1 = pair_lo(x0), u1 = pair_hi(x0), t2 = pair_lo(x1), u2 = pair_hi(x1);
    uint64_t acc = (uint64_t)((int64_t)t2 * kK2lo + (int64_t)u2);        // t2 K^2 - 2^32 t2 + u2
    acc = (uint64_t)((int64_t)u1 * kS4.lo + (int64_t)acc);
    acc = (uint64_t)((int64_t)t1 * kS6.lo + (int64_t)acc);
    acc += (uint64_t)(uint32_t)h * (uint32_t)kK8;
    const uint32_t hi = (uint32_t)(acc >> 32) + (uint32_t)t2 + (uint32_t)u1 * kS4.hi + (uint32_t)t1 * kS6.hi +
                        (uint32_t)h * (uint32_t)(kK8 >> 32) + (uint32_t)(h >> 32) * (uint32_t)kK8;
    return ((uint64_t)hi << 32) | (uint32_t)acc;
}

// keep the bytes of dword x whose index within it is >= lo and < hi (0..4)
__device__ __forceinline__ uint32_t byte_range(uint32_t x, int lo, int hi) {
    const uint32_t mlo = lo <= 0 ? 0xFFFFFFFFu : (lo >= 4 ? 0u : ~((1u << (8 * lo)) - 1u));
    const uint32_t mhi = hi >= 4 ? 0xFFFFFFFFu : (hi <= 0 ? 0u : ((1u << (8 * hi)) - 1u));
    return x & mlo & mhi;
}

// Horner of the bytes of a 16-byte piece whose piece index is in [lo, hi), others zeroed.
__device__ __forceinline__ uint64_t sdbm_piece(uint4 v, int lo, int hi) {
    uint64_t h = 0;
    h = sdbm_dword(h, byte_range(v.x, lo, hi));
    h = sdbm_dword(h, byte_range(v.y, lo - 4, hi - 4));
    h = sdbm_dword(h, byte_range(v.z, lo - 8, hi - 8));
    return sdbm_dword(h, byte_range(v.w, lo - 12, hi - 12));
}

// 4-bit mask of the bytes of x equal to the byte replicated in pat (exact SWAR test).
__device__ __forceinline__ uint32_t eq_mask4(uint32_t x, uint32_t pat) {
    const uint32_t t = x ^ pat;
    const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    return (((z >> 7) * 0x00204081u) >> 21) & 0xFu;
}

__device__ __forceinline__ uint32_t eq_mask16(uint4 v, uint32_t pat) {
    return eq_mask4(v.x, pat) | (eq_mask4(v.y, pat) << 4) | (eq_mask4(v.z, pat) << 8) |
           (eq_mask4(v.w, pat) << 12);
}

// 0x80 in every byte of x equal to the byte replicated in pat, 0 elsewhere (exact, 5 VALU ops)
__device__ __forceinline__ uint32_t eq_flags(uint32_t x, uint32_t pat) {
    const uint32_t t = x ^ pat;
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}

// 16-bit mask (bit i = byte i) of the bytes of a 16-byte piece equal to pat. The 0x80 flags of
// two dwords are packed by two v_dot4_u32_u8 with byte weights 1..128 (= 128 x the 8-bit mask).
__device__ __forceinline__ uint32_t eq_mask16_dot(uint4 v, uint32_t pat) {
    uint32_t lo = __builtin_amdgcn_udot4(eq_flags(v.x, pat), 0x08040201u, 0u, false);
    lo = __builtin_amdgcn_udot4(eq_flags(v.y, pat), 0x80402010u, lo, false);
    uint32_t hi = __builtin_amdgcn_udot4(eq_flags(v.z, pat), 0x08040201u, 0u, false);
    hi = __builtin_amdgcn_udot4(eq_flags(v.w, pat), 0x80402010u, hi, false);
    return (lo + (hi << 8)) >> 7;
}

// '\n' and ':' masks (bit i = byte i) of a 16-byte piece, 7 VALU per dword for both patterns.
// For a pattern P with bit 7 clear, byte b == P iff bit 7 of b is clear and ((b & 0x7F) ^ P) + 0x7F
// has bit 7 clear (the sum stays within the byte): the masked bytes and ~b's bit 7 are shared by
// both patterns, the xor-add is one v_xad_u32, and the flag one v_bfi_b32.
__device__ __forceinline__ uint32_t not_and(uint32_t a, uint32_t b) {   // ~a & b
    uint32_t r;
    asm("v_bfi_b32 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t xor_add(uint32_t a, uint32_t x, uint32_t y) {   // (a ^ x) + y
    uint32_t r;
    asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(x), "v"(y));
    return r;
}
// ~a & ~b & c in one gfx950 v_bitop3_b32 (truth-table index a*4 + b*2 + c: only index 1 is set)
__device__ __forceinline__ uint32_t nor_and(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x02" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t nl_colon_mask16(uint4 v) {   // '\n' mask | ':' mask << 16
    const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
    uint32_t an = 0, cn = 0, ah = 0, ch = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        // 7 VALU per dword for both patterns: the masked bytes are shared, and the "bit 7 of the
        // byte clear" term is folded into the flag's v_bitop3
        const uint32_t x = xs[d];
        const uint32_t x7 = x & 0x7F7F7F7Fu;
        const uint32_t fn = nor_and(xor_add(x7, 0x0A0A0A0Au, 0x7F7F7F7Fu), x, 0x80808080u);
        const uint32_t fc = nor_and(xor_add(x7, 0x3A3A3A3Au, 0x7F7F7F7Fu), x, 0x80808080u);
        const uint32_t w = (d & 1) ? 0x80402010u : 0x08040201u;
        if (d < 2) {
            an = __builtin_amdgcn_udot4(fn, w, an, false);
            cn = __builtin_amdgcn_udot4(fc, w, cn, false);
        } else {
            ah = __builtin_amdgcn_udot4(fn, w, ah, false);
            ch = __builtin_amdgcn_udot4(fc, w, ch, false);
        }
    }
    const uint32_t nl = (an + (ah << 8)) >> 7;
    const uint32_t cl = (cn + (ch << 8)) >> 7;
    return nl | (cl << 16);
}

// number of bytes equal to the replicated pattern
__device__ __forceinline__ uint32_t eq_count4(uint32_t x, uint32_t pat) {
    const uint32_t t = x ^ pat;
    const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    return __popc(z);
}

typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 as_uint4(v4u32 r) { return make_uint4(r[0], r[1], r[2], r[3]); }

// 16 bytes at `off`; bytes at or past `n` read as 0. Only the one piece that straddles the end
// of the batch takes the byte-wise path (buffer range checks are not byte-exact for dwordx4).
__device__ __forceinline__ uint4 load16(__amdgpu_buffer_rsrc_t rsrc, uint32_t off, uint32_t n) {
    if (off + 16u <= n) return as_uint4(__builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
    uint64_t lo = 0, hi = 0;
    for (uint32_t i = 0; i < 16u && off + i < n; ++i) {
        const uint64_t b = __builtin_amdgcn_raw_buffer_load_b8(rsrc, off + i, 0, 0);
        if (i < 8) lo |= b << (8 * i);
        else hi |= b << (8 * (i - 8));
    }
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

__device__ __forceinline__ uint64_t div_magic(uint64_t n, const Magic &mg) {
    if (mg.kind == 0) return n >> mg.shift;
    const uint64_t t = __umul64hi(mg.m, n);
    if (mg.kind == 1) return t >> mg.shift;
    return (((n - t) >> 1) + t) >> mg.shift;
}

__device__ __forceinline__ uint32_t mod_magic(uint64_t n, const Magic &mg, uint32_t d) {
    if (mg.kind == 0) return (uint32_t)n & (d - 1u);   // d a power of two (make_magic)
    return (uint32_t)(n - div_magic(n, mg) * (uint64_t)d);
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
    const uint32_t lo = __shfl_up((uint32_t)v, d, 64);
    const uint32_t hi = __shfl_up((uint32_t)(v >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int d) {
    const uint32_t lo = __shfl_xor((uint32_t)v, d, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += shfl_xor64(v, d);
    return v;
}

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
    return v;
}

// ---- DPP wave primitives (GFX9 row_shr / row_bcast / wave_shr; no LDS round trip) ----------
constexpr int kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114, kDppRowShr8 = 0x118;
constexpr int kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143, kDppWaveShr1 = 0x138;

template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp32(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW_MASK, 0xF, false);
}

template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint64_t dpp64(uint64_t old, uint64_t v) {
    const uint32_t lo = dpp32<CTRL, ROW_MASK>((uint32_t)old, (uint32_t)v);
    const uint32_t hi = dpp32<CTRL, ROW_MASK>((uint32_t)(old >> 32), (uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Inclusive wave64 scan with an associative combine f(left, right) and identity id.
template <class F>
__device__ __forceinline__ uint64_t wave_scan64(uint64_t v, uint64_t id, F f) {
    v = f(dpp64<kDppRowShr1>(id, v), v);
    v = f(dpp64<kDppRowShr2>(id, v), v);
    v = f(dpp64<kDppRowShr4>(id, v), v);
    v = f(dpp64<kDppRowShr8>(id, v), v);
    v = f(dpp64<kDppRowBcast15, 0xA>(id, v), v);
    v = f(dpp64<kDppRowBcast31, 0xC>(id, v), v);
    return v;
}

// value of the lane below (lane 0: id)
__device__ __forceinline__ uint64_t wave_shr1_64(uint64_t v, uint64_t id) { return dpp64<kDppWaveShr1>(id, v); }
__device__ __forceinline__ uint32_t wave_shr1_32(uint32_t v, uint32_t id) { return dpp32<kDppWaveShr1>(id, v); }

__device__ __forceinline__ uint32_t wave_add32(uint32_t v) {   // sum over the wave, in every lane
    v += dpp32<kDppRowShr1>(0u, v);
    v += dpp32<kDppRowShr2>(0u, v);
    v += dpp32<kDppRowShr4>(0u, v);
    v += dpp32<kDppRowShr8>(0u, v);
    v += dpp32<kDppRowBcast15, 0xA>(0u, v);
    v += dpp32<kDppRowBcast31, 0xC>(0u, v);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// inclusive wave scan of a u32 (DPP; no LDS)
__device__ __forceinline__ uint32_t wave_incl_add32(uint32_t v) {
    v += dpp32<kDppRowShr1>(0u, v);
    v += dpp32<kDppRowShr2>(0u, v);
    v += dpp32<kDppRowShr4>(0u, v);
    v += dpp32<kDppRowShr8>(0u, v);
    v += dpp32<kDppRowBcast15, 0xA>(0u, v);
    v += dpp32<kDppRowBcast31, 0xC>(0u, v);
    return v;
}

// inclusive wave64 max / min scans of a u32 (DPP)
__device__ __forceinline__ uint32_t wave_incl_max32(uint32_t v) {
    v = max(v, dpp32<kDppRowShr1>(0u, v));
    v = max(v, dpp32<kDppRowShr2>(0u, v));
    v = max(v, dpp32<kDppRowShr4>(0u, v));
    v = max(v, dpp32<kDppRowShr8>(0u, v));
    v = max(v, dpp32<kDppRowBcast15, 0xA>(0u, v));
    v = max(v, dpp32<kDppRowBcast31, 0xC>(0u, v));
    return v;
}
__device__ __forceinline__ uint32_t wave_incl_min32(uint32_t v) {
    v = min(v, dpp32<kDppRowShr1>(0xFFFFFFFFu, v));
    v = min(v, dpp32<kDppRowShr2>(0xFFFFFFFFu, v));
    v = min(v, dpp32<kDppRowShr4>(0xFFFFFFFFu, v));
    v = min(v, dpp32<kDppRowShr8>(0xFFFFFFFFu, v));
    v = min(v, dpp32<kDppRowBcast15, 0xA>(0xFFFFFFFFu, v));
    v = min(v, dpp32<kDppRowBcast31, 0xC>(0xFFFFFFFFu, v));
    return v;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

template <unsigned ABL>
__device__ __forceinline__ void stamp(const RouteParams &p, int tid, uint32_t t, int slot) {
    if ((ABL & ABL_STAMPS) && tid == 0) p.dbg[(size_t)t * 16 + slot] = __builtin_amdgcn_s_memrealtime();
}

// Segmented "line state" scan element: [63:32] newline count, [31] lane range holds a '\n',
// [16:0] first ':' of the line open at the right end of the range (tile position, kNone = none).
// combine(f, g) for f left of g: counts add; if g holds a '\n' its state wins, else the open
// line continues from f and its first colon is the earlier one.
__device__ __forceinline__ uint64_t seg_combine(uint64_t f, uint64_t g) {
    const uint64_t cnt = (f & 0xFFFFFFFF00000000ull) + (g & 0xFFFFFFFF00000000ull);
    uint32_t lo;
    if ((uint32_t)g & 0x80000000u) {
        lo = (uint32_t)g;
    } else {
        const uint32_t fc = (uint32_t)f & 0x1FFFFu, gc = (uint32_t)g & 0x1FFFFu;
        lo = ((uint32_t)f & 0x80000000u) | (fc < gc ? fc : gc);
    }
    return cnt | lo;
}

__device__ __forceinline__ uint64_t mk_status(uint32_t epoch, uint32_t flag, uint32_t value) {
    return ((uint64_t)(epoch & 0x3FFFFFFFu) << 34) | ((uint64_t)flag << 32) | value;
}

__device__ __forceinline__ bool alive_bit(const uint64_t *alive, uint32_t k) {
    return (alive[k >> 6] >> (k & 63)) & 1ull;
}

// Bit k of the batch's probed-dead bitmap: the reference zeroes the active buffer of every dead
// downstream it probes (sr-main.c:106). Read first, so that once a bit is set (after the first few
// lines) the line costs an L2 read and no same-address atomic.
__device__ __forceinline__ void note_dead(uint64_t *pd, uint32_t k) {
    uint64_t *w = pd + (k >> 6);
    const uint64_t bit = 1ull << (k & 63);
    if (!(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
        __hip_atomic_fetch_or(w, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every shard dead: each routed line probes all n positions of the permutation, i.e. every shard.
__device__ __noinline__ void note_all_dead(uint64_t *pd, uint32_t n) {
    for (uint32_t w = 0; w < (n + 63) / 64; ++w) {
        const uint64_t full = (w + 1) * 64 <= n ? ~0ull : ((1ull << (n & 63)) - 1ull);
        if ((__hip_atomic_load(pd + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & full) != full)
            __hip_atomic_fetch_or(pd + w, full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// find_downstream (sr-main.c:86-117) for one line. Returns the shard, SR_ROUTE_ALL_DEAD, or
// kRoutePending if more than kOverlay dead shards had to be probed (kRouteDefer: stopped after its
// first two picks, `defer`). The dead shards the probe visits (sr-main.c:106) go to mark_lds (the
// route kernel's per-tile LDS words), to mark / mark_wg (probe_defer_kernel and the replay), or
// nowhere: a global atomic per visit inside the route kernel's line loop cost 9 % at C2.
// The route kernel keeps the divisors' reciprocals its probes need first, N .. N - kMagicLds + 1,
// in the padding dword of LDS image rows (entry e, word w at row 4 e + w; the rows' padding is
// never read as bytes), so that a probe step waits on LDS rather than on a global load (a global
// load waited for inside the line loop also waits for every record store before it).
constexpr uint32_t kMagicLds = kOverlay + 1;
__device__ __forceinline__ Magic magic_from_pad(const uint32_t *img, uint32_t e) {
    Magic mg;
    const uint32_t lo = img[(4 * e) * 17 + 16], hi = img[(4 * e + 1) * 17 + 16];
    mg.m = ((uint64_t)hi << 32) | lo;
    mg.shift = img[(4 * e + 2) * 17 + 16];
    mg.kind = img[(4 * e + 3) * 17 + 16];
    return mg;
}

// The alive bitmap's first kAliveLds words sit in the pad dwords of image rows kAliveRow0 ..
// (word w: rows kAliveRow0 + 2w, + 1 for its high half), so that the probe's alive tests read LDS:
// a global load inside the line loop would also wait for every record store issued before it.
constexpr uint32_t kAliveRow0 = 4 * kMagicLds;
constexpr uint32_t kAliveLds = 16;   // words: up to 1024 downstreams
__device__ __forceinline__ uint32_t alive_pad_dword(const uint32_t *img, uint32_t k) {
    return img[(kAliveRow0 + (k >> 5)) * 17 + 16];
}

// MARK_LDS (RouteParams::mark): the tile's probed-dead bits (sr-main.c:106) in the pad dwords of
// rows kMarkRow0 .. (bit k in row kMarkRow0 + k / 32), stored in the tile's slot when it ends and
// ORed per batch by probe_defer_kernel, instead of a replay after the launch. Atomic ORs per tile
// serialise at the memory side: into the callers' words of 32 batches (two cache lines) +115 us per
// C2 launch; into a line per batch, each followed by a wait before the block's arrival, +6 us.
constexpr uint32_t kMarkRow0 = kAliveRow0 + 2 * kAliveLds;
__device__ __forceinline__ void note_dead_lds(uint32_t *img, uint32_t k) {
    atomicOr(&img[(kMarkRow0 + (k >> 5)) * 17 + 16], 1u << (k & 31));   // ds_or_b32, no return
}

// note_dead into a workgroup's LDS copy of the bitmap (shards below 64 * kReplayCheckWords); the
// workgroup ORs its copy into the global words once per stride. The global words are the hot
// addresses of a replay: same-address atomics, even one per workgroup and shard, serialise at the
// memory side (measured: 74 us for 16 dead shards over 32 batches of C5).
constexpr uint32_t kReplayCheckWords = 16;   // workgroup-local bitmap words (up to 1024 shards)
__device__ __forceinline__ void note_dead_wg(uint64_t *pd, unsigned long long *wg, uint32_t k) {
    if (wg && k < 64 * kReplayCheckWords) {   // the workgroup pushes its copy to pd (probed_dead_kernel)
        const unsigned long long bit = 1ull << (k & 63);
        if (!(wg[k >> 6] & bit)) atomicOr(&wg[k >> 6], bit);
        return;
    }
    note_dead(pd, k);
}

// DEFER (the route kernel, with dead shards): a line still unresolved after its first two picks
// returns kRouteDefer; probe_defer_kernel runs its whole probe later, one lane per line (a wave
// that runs the overlay loop below for one of its lines holds all its lanes for every step).
// What probe_shard reads of its parameters (RouteParams, or ProbeArgs in the packing's counting pass)
struct ProbeArgs {
    uint32_t nds, dead, picks, pad;
    Magic magic_n;
    const uint64_t *alive;
    const Magic *magic;
};

// OV: entries of the register overlay (at least the dead shards of the snapshot, or up to kOverlay: a probe
// that would need more returns kRoutePending for probe_wide_kernel); fewer entries, fewer registers
template <bool MARK = false, class P = RouteParams, int OV = kOverlay>
__device__ uint32_t probe_shard(uint64_t h, const P &p, uint64_t *mark = nullptr,
                                const uint32_t *pad_img = nullptr, unsigned long long *mark_wg = nullptr,
                                bool defer = false, uint32_t *mark_lds = nullptr) {
    const uint32_t n = p.nds;
    if (p.dead >= n) {                                    // includes N == 0
        if (MARK && n) note_all_dead(mark, n);
        return SR_ROUTE_ALL_DEAD;
    }
    if (p.dead == 0) return mod_magic(h, p.magic_n, n);   // every shard alive: j = h % N
    // up to 64 shards the alive bitmap is one word, read once per probe
    const bool lds_alive = pad_img && n <= 64 * kAliveLds;
    const uint64_t alive0 = n > 64 ? 0ull
                            : lds_alive ? ((uint64_t)alive_pad_dword(pad_img, 32) << 32) | alive_pad_dword(pad_img, 0)
                                        : p.alive[0];
    auto alive_k = [&](uint32_t k) {
        if (n <= 64) return ((alive0 >> k) & 1ull) != 0;
        if (lds_alive) return ((alive_pad_dword(pad_img, k) >> (k & 31)) & 1u) != 0;
        return alive_bit(p.alive, k);
    };
    auto magic_i = [&](uint32_t i) {
        return (pad_img && n - i < kMagicLds) ? magic_from_pad(pad_img, n - i) : p.magic[i];
    };
    // ds_index[] is the identity plus an overlay of (position -> value) writes, newest last. The
    // first two picks see at most one overlay entry (kept in one register, o0): with few dead
    // shards nearly every line ends there, without scanning the 16-entry overlay.
    uint32_t o0 = 0xFFFFFFFFu, o1 = 0xFFFFFFFFu;   // (pos << 16) | value
    uint32_t i = n;
    const int np = (defer && p.picks == 1) ? 1 : 2;
    for (int it = 0; it < np && i > 0; ++it, --i) {
        const uint32_t j = mod_magic(h, magic_i(i), i);                                  // :98
        const uint32_t k = (o0 >> 16) == j ? (o0 & 0xFFFFu) : j;                         // :99
        if (alive_k(k)) return k;                                                         // :101-104
        if (MARK) note_dead_wg(mark, mark_wg, k);                                         // :106
        if (mark_lds) note_dead_lds(mark_lds, k);
        if (j != i - 1) {                                                                 // :108-111
            const uint32_t v = (o0 >> 16) == i - 1 ? (o0 & 0xFFFFu) : i - 1;
            if (o0 == 0xFFFFFFFFu) o0 = (j << 16) | v;
            else o1 = (j << 16) | v;
        }
        h = (h * 7 + 5) / 3;                                                              // :113
    }
    if (defer && i > 0) return kRouteDefer;
    static_assert(OV >= 2 && OV <= kOverlay, "overlay entries");
    uint32_t ov[OV];
    int nov = (o0 != 0xFFFFFFFFu) + (o1 != 0xFFFFFFFFu);
#pragma unroll
    for (int e = 0; e < OV; ++e) ov[e] = e == 0 ? o0 : (e == 1 ? o1 : 0xFFFFFFFFu);
    for (; i > 0; --i) {
        const uint32_t j = mod_magic(h, magic_i(i), i);              // :98
        uint32_t k = j;                                              // :99
#pragma unroll
        for (int e = 0; e < OV; ++e)
            if ((ov[e] >> 16) == j) k = ov[e] & 0xFFFFu;
        if (alive_k(k)) return k;                                    // :101-104
        if (MARK) note_dead_wg(mark, mark_wg, k);                    // :106
        if (mark_lds) note_dead_lds(mark_lds, k);
        if (j != i - 1) {                                            // :108-111
            uint32_t v = i - 1;
#pragma unroll
            for (int e = 0; e < OV; ++e)
                if ((ov[e] >> 16) == i - 1) v = ov[e] & 0xFFFFu;
            if (nov == OV) return kRoutePending;
#pragma unroll
            for (int e = 0; e < OV; ++e)
                if (e == nov) ov[e] = (j << 16) | v;
            ++nov;
        }
        h = (h * 7 + 5) / 3;                                         // :113
    }
    return SR_ROUTE_ALL_DEAD;                                        // :115-116
}

// find_downstream's first picks (sr-main.c:86-117; probe_shard's first loop): all alive, h % N;
// one dead shard, at most two picks (the second pick never meets the dead shard); two or more
// dead, RouteParams::picks picks and then kRouteDefer (probe_defer_kernel finishes the probe; the
// host launches a kernel using it only when it can defer). Reciprocals and alive words from the LDS
// pads, the dead shards visited noted in the tile's LDS words (MARK_LDS). The probe of the chunk
// kernel and of the route kernel's KV_PICKS variants.
__device__ __forceinline__ uint32_t chunk_probe(uint64_t h, const RouteParams &p, uint32_t *img) {
    const uint32_t n = p.nds;
    if (p.dead >= n) return SR_ROUTE_ALL_DEAD;   // includes N == 0 (:115-116)
    if (p.dead == 0) return mod_magic(h, p.magic_n, n);
    const bool small = n <= 64;
    const uint64_t alive0 = small ? ((uint64_t)alive_pad_dword(img, 32) << 32) | alive_pad_dword(img, 0) : 0ull;
    const int np = p.dead >= 2 && p.picks == 1 ? 1 : 2;
    uint32_t o0 = 0xFFFFFFFFu;   // the permutation overlay after one pick: (position << 16) | value
    uint32_t i = n;
    for (int it = 0; it < np; ++it, --i) {
        // the first pick's reciprocal is the kernel argument (scalar registers, a scalar branch on
        // its kind), the second's an LDS pad
        const Magic mg = it == 0 ? p.magic_n : magic_from_pad(img, n - i);
        const uint32_t j = mod_magic(h, mg, i);                                           // :98
        const uint32_t k = (o0 >> 16) == j ? (o0 & 0xFFFFu) : j;                         // :99
        const bool al = small ? ((alive0 >> k) & 1ull) != 0
                              : (n <= 64 * kAliveLds ? ((alive_pad_dword(img, k) >> (k & 31)) & 1u) != 0
                                                     : alive_bit(p.alive, k));
        if (al) return k;                                                                 // :101-104
        if (p.mark_tiles) note_dead_lds(img, k);                                          // :106
        if (j != i - 1) o0 = (j << 16) | (i - 1);                                         // :108-111
        h = (h * 7 + 5) / 3;                                                              // :113
    }
    return kRouteDefer;
}

// KV_DEFER1's probe (find_downstream's first pick, sr-main.c:98-104): h % N when that shard is alive,
// else the deferral (probe_defer_kernel runs the whole probe, sr-main.c:86-117)
__device__ __forceinline__ uint32_t defer1_probe(uint64_t h, const RouteParams &p) {
    const uint32_t j = mod_magic(h, p.magic_n, p.nds);
    return ((p.alive_w0 >> j) & 1ull) ? j : kRouteDefer;
}

// KV_DEAD1's probe: find_downstream (sr-main.c:86-117) with one dead shard d. The first pick
// j = h % N (:98) is d only for lines that then zero d's buffer (:106) and swap ds_index[j] with
// ds_index[N - 1] (:108-111); the second pick h' % (N - 1), h' = (h * 7 + 5) / 3 (:113), lands on
// ds_index[j] = N - 1 or on an untouched position, and is never d: two picks end every probe.
__device__ __forceinline__ uint32_t dead1_probe(uint64_t h, const RouteParams &p, uint32_t *img) {
    const uint32_t n = p.nds, d = p.dead_k;
    const uint32_t j = mod_magic(h, p.magic_n, n);
    if (j != d) return j;
    if (p.mark_tiles) note_dead_lds(img, d);
    const uint32_t j2 = mod_magic((h * 7 + 5) / 3, p.magic_n1, n - 1);
    return j2 == j ? n - 1 : j2;
}

// The end of a tile's MARK_LDS (the dead shards its probes visited, sr-main.c:106): its words go to its
// slot (plain stores, nothing waits), ORed per batch after the launch by probe_defer_kernel or, in a
// route + pack launch with one dead shard, by the packing's mtu_scan_kernel.
template <unsigned ABL>
__device__ __forceinline__ void mark_tile_end(const RouteParams &p, const uint32_t *img, const BatchDesc &bd, uint32_t t,
                                              int tid);

// ---------------------------------------------------------------------------------------
// The route kernel
// ---------------------------------------------------------------------------------------
template <int BLOCK>
struct SmemT {
    static constexpr int kWaves = BLOCK / 64;
    static constexpr int kTileB = BLOCK * kLaneBytes;
    static constexpr int kHalo = 2048;                // bytes before the tile kept in LDS
    static constexpr int kWin = BLOCK;                // tile-local lines staged per round
    // LDS image of the batch bytes [T0 - kHalo, T0 + tile): 64-byte rows stored as 17 dwords (one
    // pad dword per row) so that lanes reading at 64-byte strides hit distinct banks.
    static constexpr int kRows = (kHalo + kTileB) / 64;
    static constexpr int kWords = kRows * 17 + 20;
    uint32_t img[kWords];
    int32_t lend[kWin + 1];          // per staged line: tile position of its '\n'; slot 0 = previous
    int32_t lcol[kWin + 1];          // per staged line: first ':' in the tile part (kNone if none)
    uint32_t wave_cnt[kWaves];
    // segment layout of a window (tiles of mixed lengths): lanes wanted per wave, line starts as a
    // lane bitmap, per 64-lane word the line covering its first lane ((start << 16) | line) and the
    // part of the line a word passes on to the next
    static constexpr int kSegWords = ((kTileB + kHalo) / 64 + kWin) / 64 + 4;
    uint32_t seg_w[kWaves][2];
    uint64_t seg_mask[kSegWords];
    uint32_t seg_first[kSegWords];
    uint64_t seg_carry[kSegWords];
    uint32_t wave_scan[kWaves][4];   // per wave, inclusive at its last lane: '\n' count, -, colon key; a chunk with two '\n'
    uint64_t kp_lo[kPowLo];          // K^i
    uint64_t kp_hi[kPowHi];          // K^(64 i)
    uint64_t kp_inv[kPowInv];        // K^-z (an LDS read rather than three 64-bit constants held in VGPRs)
    static constexpr int kPowWords = (kPowLo + kPowHi + kPowInv) * 2;   // u32 words of the three tables
    int32_t s_pre, c_pre;            // straddling line: tile-relative start / first colon before T0
    uint32_t hist[kHistKeys];        // RouteParams::hist: the tile's records per key
    uint32_t epoch, base;
    uint32_t scan_head, scan_pub, scan_total;   // scanner: bases computed / published, line total
};

// K^-z for z = 1, 2, 3 (undoing z bytes of zero padding)
__device__ __forceinline__ uint64_t kinv_small(int z) {
    constexpr uint64_t i1 = kKinv, i2 = kKinv * kKinv, i3 = kKinv * kKinv * kKinv;
    return z == 1 ? i1 : (z == 2 ? i2 : i3);
}

// K^n for 0 <= n < 1536 from the LDS tables
template <class S>
__device__ __forceinline__ uint64_t kpow_n(const S &sm, int n) {
    return sm.kp_hi[n >> 6] * sm.kp_lo[n & 63];
}

// dword index in the padded LDS image of image byte b (b % 4 == 0 for whole dwords)
__device__ __forceinline__ int img_dw(int b) { return (b >> 6) * 17 + ((b >> 2) & 15); }

// sdbm (Horner, no colon test) of the n <= 64 image bytes starting at image byte a.
// Aligned dword reads + v_alignbyte; whole dwords by sdbm_dword, the tail through the
// zero-padding identity Horner(x, 0^z) = Horner(x) * K^z.
template <class S>
__device__ __forceinline__ uint64_t sdbm_lds(const S &sm, int a, int n) {
    const int base = a & ~3, sh = a & 3;
    const int i0 = img_dw(base), r0 = base & 63;
    const int nfull = n >> 2, rem = n & 3;
    uint32_t w[17];
#pragma unroll
    for (int m = 0; m < 17; ++m) w[m] = sm.img[i0 + m + ((r0 + 4 * m) >> 6)];
    uint64_t h = 0;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        if (m < nfull) h = sdbm_dword(h, __builtin_amdgcn_alignbyte(w[m + 1], w[m], sh));
    }
    if (rem) {
        uint32_t x = 0;
#pragma unroll
        for (int m = 0; m < 16; ++m)
            if (m == nfull) x = __builtin_amdgcn_alignbyte(w[m + 1], w[m], sh);
        x &= (1u << (8 * rem)) - 1u;
        h = sdbm_dword(h, x) * kinv_small(4 - rem);
    }
    return h;
}

// sdbm of the 0 < n <= 64 image bytes starting at image byte a, from aligned dword reads: the
// bytes of the first dword before a are zeroed (leading zeros leave a Horner value unchanged), the
// last partial dword is zero-padded and the padding undone by K^-z. Dword m of the run is p[m]
// before the row's pad dword and p[m + 1] after it.
// slot != nullptr: also read that granule into st part-way through (after the dwords before
// the row's pad): the tile's record base, requested about a round trip before it is needed.
template <class S>
__device__ __forceinline__ uint64_t sdbm_img(const S &sm, int a, int n, const uint64_t *slot = nullptr,
                                             uint64_t *st = nullptr) {
    const int lead = a & 3, L = lead + n;
    const int F = L >> 2, rem = L & 3;
    const int dw = a >> 2, s16 = dw & 15, cross = 16 - s16;
    const uint32_t *const p = &sm.img[(dw >> 4) * 17 + s16];
    const uint32_t first = p[0] & (0xFFFFFFFFu << (8 * lead));
    // a partial last dword of rem bytes: shifted up so that they are its high bytes (the bytes
    // past the name drop out, and leading zero bytes leave a Horner value unchanged), then
    // h K^rem + Horner(x): no mask and no K^-z correction
    if (F == 0) return sdbm_dword_fast(0, first << (8 * (4 - rem)));
    uint64_t h = sdbm_dword_fast(0, first);
    int m = 1;
    // four dwords per iteration (a quarter of the loop control; adjacent reads pair into ds_read2)
    const int F1 = F < cross ? F : cross;   // dwords before the row's pad dword
    for (; m + 3 < F1; m += 4)
        h = sdbm_qword_fast(sdbm_qword_fast(h, p[m], p[m + 1]), p[m + 2], p[m + 3]);
    for (; m < F1; ++m) h = sdbm_dword_fast(h, p[m]);
    if (slot) *st = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (; m + 3 < F; m += 4)
        h = sdbm_qword_fast(sdbm_qword_fast(h, p[m + 1], p[m + 2]), p[m + 3], p[m + 4]);
    for (; m < F; ++m) h = sdbm_dword_fast(h, p[m + 1]);
    if (rem) h = h * sm.kp_lo[rem] + sdbm_dword_fast(0, p[m + (m >= cross ? 1 : 0)] << (8 * (4 - rem)));
    return h;
}

// 32-bit LDS address of a __shared__ object, and a two-dword LDS store at immediate dword offsets
// from one base register (the compiler rematerialises a base per store otherwise: 2 VALU each)
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
template <int O0, int O1>
__device__ __forceinline__ void ds_write2_at(uint32_t base, uint32_t a, uint32_t b) {
    asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4" ::"v"(base), "v"(a), "v"(b), "i"(O0), "i"(O1)
                 : "memory");
}

// store / load one 16-byte chunk at image byte b (b % 16 == 0: never crosses a row)
template <class S>
__device__ __forceinline__ void img_put16(S &sm, int b, uint4 v) {
    const int i = img_dw(b);
    sm.img[i] = v.x;
    sm.img[i + 1] = v.y;
    sm.img[i + 2] = v.z;
    sm.img[i + 3] = v.w;
}
template <class S>
__device__ __forceinline__ uint4 img_get16(const S &sm, int b) {
    const int i = img_dw(b);
    return make_uint4(sm.img[i], sm.img[i + 1], sm.img[i + 2], sm.img[i + 3]);
}

// Number of '\n' bytes in tile m, counted by one wave (only used when a predecessor has not
// published its count within the spin budget).
template <int BLOCK>
__device__ uint32_t count_tile_wave(uint32_t nbytes, __amdgpu_buffer_rsrc_t rsrc, uint32_t m, int lane) {
    constexpr uint32_t T = BLOCK * kLaneBytes;
    uint32_t c = 0;
    for (uint32_t off = lane * 16; off < T; off += 1024) {
        const uint4 v = load16(rsrc, m * T + off, nbytes);
        c += eq_count4(v.x, 0x0A0A0A0Au) + eq_count4(v.y, 0x0A0A0A0Au) + eq_count4(v.z, 0x0A0A0A0Au) +
             eq_count4(v.w, 0x0A0A0A0Au);
    }
    return (uint32_t)wave_sum64(c);
}

// ---- record numbering: one scanner wave per batch --------------------------------------------
// Blocks 0 .. nb-1 of a launch are scanners, one per batch; they are dispatched before every tile.
// A tile publishes its '\n' count straight after its loads (status granule, never waits for
// anything); the scanner of its batch walks the batch's tiles in order, 64 per round, and
// publishes each tile's first record index (bases granule) as soon as the counts of all its
// predecessors are in. A tile needs its base only when it writes its records, after hashing.
// A tile whose count has not appeared within the spin budget is counted by the scanner itself,
// so the scan completes whatever the dispatch order.
constexpr uint32_t kFlagBase = 2u;
constexpr uint32_t kFlagXcc = 3u;
// A tile's count granule carries (8 | its XCD) in bits 28..31 of the value above the count.
constexpr uint32_t kCountMask = 0x0FFFFFFFu;

// XCD of the executing workgroup. Placement is observed, never assumed: a granule whose producer
// and consumer share an XCD is stored plain (the line stays in that XCD's L2, where the consumer's
// sc1 poll finds it); any other granule is stored sc1 (written through, dropped from L2).
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x;
}

// 8-byte granule store: plain when the reader shares this XCD, else sc1 (agent scope)
__device__ __forceinline__ void granule_store(uint64_t *slot, uint64_t v, bool same_xcd) {
    if (same_xcd)
        __hip_atomic_store(slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else
        __hip_atomic_store(slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool granule_ok(uint64_t st, uint32_t ep, uint32_t flag) {
    return (uint32_t)(st >> 34) == ep && ((st >> 32) & 3u) == flag;
}

template <int BLOCK>
__device__ void scan_batch(const RouteParams &p, const BatchDesc &bd, uint32_t epoch, int lane) {
    constexpr int kGroups = 4;   // 64-tile groups polled per round
    const uint64_t *status = p.status + bd.sbase;
    uint64_t *bases = p.bases + bd.sbase;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)bd.bytes, (short)0, (int)bd.nbytes, 0x00020000);
    const uint32_t ep = epoch & 0x3FFFFFFFu;
    uint32_t run = 0;
    uint32_t c = 0;      // first tile whose base is not yet published
    int spin = 0;        // rounds without progress on group c
    while (c < bd.ntiles) {
        // one round trip: the counts of up to kGroups groups from c on
        uint32_t cnt[kGroups];
        bool have[kGroups];
#pragma unroll
        for (int k = 0; k < kGroups; ++k) {
            const uint32_t tt = c + 64 * k + lane;
            cnt[k] = 0;
            have[k] = tt >= bd.ntiles;
            if (!have[k]) {
                const uint64_t st = __hip_atomic_load(&status[tt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (granule_ok(st, ep, kFlagAgg)) {
                    cnt[k] = (uint32_t)st & kCountMask;
                    have[k] = true;
                }
            }
        }
        // head group still incomplete after the spin budget: count its silent tiles here
        if (spin >= kSpinBudget) {
            uint64_t missing = __ballot(!have[0]);
            while (missing) {
                const int L = __builtin_ctzll(missing);
                missing &= missing - 1;
                const uint32_t c2 = count_tile_wave<BLOCK>(bd.nbytes, rsrc, c + (uint32_t)L, lane);
                if (lane == L) {
                    cnt[0] = c2;
                    have[0] = true;
                }
            }
        }
        // publish the longest complete prefix (tile by tile, so a tile never waits for a later one)
        bool progress = false;
#pragma unroll
        for (int k = 0; k < kGroups; ++k) {
            const uint64_t missing = __ballot(!have[k]);
            const int nready = missing ? __builtin_ctzll(missing) : 64;
            if (nready == 0) break;
            const uint32_t tt = c + lane;   // c has advanced by 64 per fully published group
            const uint32_t v = lane < nready ? cnt[k] : 0u;
            const uint32_t incl = wave_incl_add32(v);
            if (lane < nready && tt < bd.ntiles)
                __hip_atomic_store(&bases[tt], mk_status(epoch, kFlagBase, run + incl - v), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            run += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            c += (uint32_t)nready;
            progress = true;
            if (nready < 64 || c >= bd.ntiles) break;
        }
        if (progress) {
            spin = 0;
        } else {
            ++spin;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (lane == 0) *bd.n_out = run;
}

// Scanner with its global stores split off (the product's): on gfx9 a wave's stores share vmcnt
// with its loads, so a scanner that also published would wait for its own stores before every
// poll. Wave 0 polls the tiles' counts and computes their bases into an LDS ring (head index
// released after the writes); wave 1 publishes the ring to the bases granules and the batch's
// line count. Flow control keeps the ring (the LDS image, 4096 entries) from overrunning.
// ABL_STAMPS: tile workgroup index (the dbg slot) of tile t of batch bd
__device__ __forceinline__ uint32_t stamp_block(const RouteParams &p, const BatchDesc &bd, uint32_t t) {
    return p.xcd_local ? (bd.tile0 + t) * 8u + bd.cls : bd.tile0 + t;
}

template <int BLOCK, unsigned ABL, class S>
__device__ void scan_batch_split(const RouteParams &p, const BatchDesc &bd, uint32_t epoch, S &sm,
                                 int wave, int lane) {
    constexpr uint32_t kRing = 4096;
    static_assert(S::kWords >= (int)kRing, "scanner ring in the LDS image");
    uint32_t *const ring = sm.img;
    if (wave == 0) {
        constexpr int kGroups = 4;
        const uint64_t *status = p.status + bd.sbase;
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc((void *)bd.bytes, (short)0, (int)bd.nbytes, 0x00020000);
        const uint32_t ep = epoch & 0x3FFFFFFFu;
        // tiles that share this XCD get their base by a plain store (ring entry bit 31)
        constexpr bool kAgentOnly = (ABL & ABL_AGENT_GRANULES) != 0;
        const uint32_t mine = kAgentOnly ? 0u : (8u | xcc_id()) << 28;
        if (lane == 0 && !kAgentOnly)
            __hip_atomic_store(&p.ctl->scan_xcc[blockIdx.x], mk_status(epoch, kFlagXcc, xcc_id()), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        uint32_t run = 0, c = 0, rounds = 0;
        int spin = 0;
        if (!(ABL & ABL_SCAN_SERIAL)) {
            // Pipelined polls of the 64 granules from c: the next poll is issued before the previous
            // one is consumed, so two are in flight and the scanner looks every half round trip
            // (a poll's round trip under the tiles' load is ~1.2 us). Unrolled by two with the
            // roles of the two poll registers swapped, so no copy waits for a poll in flight.
            const uint32_t last = bd.ntiles - 1u;
            auto poll = [&](uint32_t c0) -> uint64_t {   // unconditional load: clamped address
                const uint32_t tt = c0 + lane < last ? c0 + lane : last;
                return __hip_atomic_load(&status[tt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            };
            // consume poll `cur` (tiles [ccur, ccur + 64)) from c, with poll `nxt` issued first
            auto step = [&](uint64_t cur, uint32_t ccur, uint64_t &nxt, uint32_t &cnxt) {
                while (c + 64 > __hip_atomic_load(&sm.scan_pub, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) + kRing)
                    __builtin_amdgcn_s_sleep(1);
                cnxt = c;
                nxt = poll(c);
                const int sh = (int)(c - ccur);
                uint64_t st = cur;
                if (sh) {
                    const int src = (lane + sh) & 63;
                    st = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(cur >> 32), src) << 32) |
                         (uint32_t)__shfl((int)(uint32_t)cur, src);
                }
                const uint32_t tt = c + lane;
                uint32_t cnt = 0, loc = 0;
                bool have = tt >= bd.ntiles;
                if (!have && lane + sh < 64 && granule_ok(st, ep, kFlagAgg)) {
                    cnt = (uint32_t)st & kCountMask;
                    loc = ((uint32_t)st & ~kCountMask) == mine && mine ? 0x80000000u : 0u;
                    have = true;
                }
                if (spin >= kSpinBudget) {   // still incomplete: count the silent tiles here
                    uint64_t missing = __ballot(!have);
                    while (missing) {
                        const int L = __builtin_ctzll(missing);
                        missing &= missing - 1;
                        const uint32_t c2 = count_tile_wave<BLOCK>(bd.nbytes, rsrc, c + (uint32_t)L, lane);
                        if (lane == L) {
                            cnt = c2;
                            have = true;
                        }
                    }
                }
                const uint64_t missing = __ballot(!have);
                const int nready = missing ? __builtin_ctzll(missing) : 64;
                if (nready) {
                    const uint32_t v = lane < nready ? cnt : 0u;
                    const uint32_t incl = wave_incl_add32(v);
                    if (lane < nready && tt < bd.ntiles) {
                        ring[tt % kRing] = (run + incl - v) | loc;
                        if (ABL & ABL_STAMPS)
                            p.dbg[(size_t)stamp_block(p, bd, tt) * 16 + 13] = __builtin_amdgcn_s_memrealtime();
                    }
                    run += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                    c += (uint32_t)nready;
                    if (c > bd.ntiles) c = bd.ntiles;
                    spin = 0;
                    if (lane == 0) {
                        if (c >= bd.ntiles) sm.scan_total = run;
                        __hip_atomic_store(&sm.scan_head, c, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                } else {
                    ++spin;
                    __builtin_amdgcn_s_sleep(1);
                }
            };
            uint64_t pa = poll(0), pb = 0;
            uint32_t ca = 0, cb = 0;
            while (c < bd.ntiles) {
                step(pa, ca, pb, cb);
                if (c >= bd.ntiles) break;
                step(pb, cb, pa, ca);
            }
        }
        while (c < bd.ntiles) {
            // the publisher must have taken the ring slots this round may overwrite
            while (c + 64 * kGroups > __hip_atomic_load(&sm.scan_pub, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) +
                                          kRing)
                __builtin_amdgcn_s_sleep(1);
            uint32_t cnt[kGroups], loc[kGroups];
            bool have[kGroups];
            const uint64_t t_iss = (ABL & ABL_STAMPS) ? __builtin_amdgcn_s_memrealtime() : 0;
#pragma unroll
            for (int k = 0; k < kGroups; ++k) {
                const uint32_t tt = c + 64 * k + lane;
                cnt[k] = 0;
                loc[k] = 0;
                have[k] = tt >= bd.ntiles;
                if (!have[k]) {
                    const uint64_t st = __hip_atomic_load(&status[tt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (granule_ok(st, ep, kFlagAgg)) {
                        cnt[k] = (uint32_t)st & kCountMask;
                        loc[k] = ((uint32_t)st & ~kCountMask) == mine && mine ? 0x80000000u : 0u;
                        have[k] = true;
                    }
                }
            }
            if (ABL & ABL_STAMPS) {   // poll round trips: (issue, all returned) per round
                if (lane == 0) {
                    const size_t o = 300000u + blockIdx.x * 4096u + (rounds & 2047u) * 2u;
                    p.dbg[o] = t_iss;
                    p.dbg[o + 1] = __builtin_amdgcn_s_memrealtime();
                }
                ++rounds;
            }
            if (spin >= kSpinBudget) {   // head group still incomplete: count its silent tiles here
                uint64_t missing = __ballot(!have[0]);
                while (missing) {
                    const int L = __builtin_ctzll(missing);
                    missing &= missing - 1;
                    const uint32_t c2 = count_tile_wave<BLOCK>(bd.nbytes, rsrc, c + (uint32_t)L, lane);
                    if (lane == L) {
                        cnt[0] = c2;
                        have[0] = true;
                    }
                }
            }
            const uint32_t c_start = c;
#pragma unroll
            for (int k = 0; k < kGroups; ++k) {
                const uint64_t missing = __ballot(!have[k]);
                const int nready = missing ? __builtin_ctzll(missing) : 64;
                if (nready == 0) break;
                const uint32_t v = lane < nready ? cnt[k] : 0u;
                const uint32_t incl = wave_incl_add32(v);
                if (lane < nready && c + lane < bd.ntiles) {
                    ring[(c + lane) % kRing] = (run + incl - v) | loc[k];
                    if (ABL & ABL_STAMPS) p.dbg[(size_t)stamp_block(p, bd, c + lane) * 16 + 13] = __builtin_amdgcn_s_memrealtime();
                }
                run += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                c += (uint32_t)nready;
                if (nready < 64 || c >= bd.ntiles) break;
            }
            if (c > bd.ntiles) c = bd.ntiles;
            if (c != c_start) {
                spin = 0;
                if (lane == 0) {
                    if (c >= bd.ntiles) sm.scan_total = run;
                    __hip_atomic_store(&sm.scan_head, c, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            } else {
                ++spin;
                __builtin_amdgcn_s_sleep(1);
            }
        }
    } else if (wave == 1) {
        uint64_t *const bases = p.bases + bd.sbase;
        uint32_t pub = 0;
        while (pub < bd.ntiles) {
            const uint32_t h = __hip_atomic_load(&sm.scan_head, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (h == pub) {
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            for (uint32_t i = pub + lane; i < h; i += 64) {
                const uint32_t r = ring[i % kRing];
                granule_store(&bases[i], mk_status(epoch, kFlagBase, r & 0x7FFFFFFFu), (r >> 31) != 0u);
                if (ABL & ABL_STAMPS) p.dbg[(size_t)stamp_block(p, bd, i) * 16 + 12] = __builtin_amdgcn_s_memrealtime();
            }
            pub = h;
            if (lane == 0) __hip_atomic_store(&sm.scan_pub, pub, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (lane == 0) *bd.n_out = __hip_atomic_load(&sm.scan_total, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// a tile's first record index, from its scanner (per lane; the lanes of a wave read one address).
// Fallback after a long wait (never taken when blocks are dispatched in order): count the '\n'
// bytes before the tile directly.
__device__ uint32_t wait_base(const uint64_t *slot, uint32_t epoch, __amdgpu_buffer_rsrc_t rsrc, uint32_t T0) {
    const uint32_t ep = epoch & 0x3FFFFFFFu;
    for (uint32_t spin = 0; spin < (1u << 22); ++spin) {
        const uint64_t st = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (granule_ok(st, ep, kFlagBase)) return (uint32_t)st;
        __builtin_amdgcn_s_sleep(1);
    }
    uint32_t n = 0;
    for (uint32_t off = 0; off < T0; off += 4)
        n += eq_count4(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0), 0x0A0A0A0Au);
    return n;
}

// Arrivals: every block adds itself to a sharded counter (no return value, nothing waits); the
// last block waits until all have arrived, then resets the counters and advances the epoch.
// Every block read the epoch before arriving, so none of this launch can see the new one.
__device__ __forceinline__ void arrive_count(const RouteParams &p, uint32_t blk) {
    __hip_atomic_fetch_add(&p.ctl->done[blk & 7u][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ void arrive_last(const RouteParams &p, uint32_t blk, uint32_t epoch) {
    if (blk != p.total_blocks - 1) return;
    for (uint32_t spin = 0; spin < (1u << 26); ++spin) {
        uint32_t n = 0;
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8)
            n += __hip_atomic_load(&p.ctl->done[s8][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n >= p.total_blocks) break;
        __builtin_amdgcn_s_sleep(2);
    }
    uint32_t weighed = 0, segmented = 0;
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
        __hip_atomic_store(&p.ctl->done[s8][0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        weighed += __hip_atomic_exchange(&p.ctl->layout[s8][0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        segmented += __hip_atomic_exchange(&p.ctl->layout[s8][1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (weighed && p.layout_out) {   // the host's layout choice reads these (route_host.hpp)
        __hip_atomic_store(&p.layout_out[1], weighed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&p.layout_out[2], segmented, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&p.layout_out[0], epoch + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_store(&p.ctl->epoch, epoch + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ void arrive(const RouteParams &p, uint32_t blk, uint32_t epoch) {
    arrive_count(p, blk);
    arrive_last(p, blk, epoch);
}
// A tile's arrival right after it has read the epoch (the invariant above holds all the same), not
// at its end: the atomic's round trip then runs under the tile's loads instead of after its last
// store. Segment-layout launches keep the arrival at the end: their tiles add the layout statistics
// in their last window, which the last block reads once everyone has arrived.
template <unsigned ABL>
constexpr bool kEarlyArrive = (ABL & KV_SEGMENTS) == 0;

template <int BLOCK, unsigned ABL>
struct KernelTraits {
    // waves per SIMD to reserve registers for: 1024-thread tiles run one workgroup per CU,
    // smaller tiles several (LDS: 86 KB / 45 KB / 24 KB per workgroup)
    static constexpr int kMinWavesPerSimd = BLOCK >= 1024 ? 4 : (BLOCK >= 512 ? 6 : 7);
    static constexpr int kMaxWavesPerSimd = 8;
    static constexpr int kMaxVgpr = 512 / kMinWavesPerSimd / 8 * 8;   // 72 for 7 waves per SIMD
};

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, never for its
// outstanding global loads.
__device__ __forceinline__ void wg_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A tile workgroup's launch header {nb, total_blocks, xcd_local, nds} and batch, from two scalar
// loads issued together: the header, and the row of cls_tab for its block index B mod 8, which the
// host deals by block (route_host.hpp): entry k of row r = (the first B / 8 past batch j's tiles among
// the blocks B = r (mod 8)) << 6 | j, ascending, ~0u pads. The batch is the row's first entry past
// B / 8 (63: past the row, a padding block). The tile's class-local index then comes with the batch
// descriptor (tile0), so that two dependent scalar round trips precede the tile's own loads (the class
// row indexed by the class, from the header's batch count and mode, was three, and four with the
// entry re-read by index). The kernels' only argument is the RouteParams, at the kernarg segment's
// start. Scanner blocks (B < nb) get a batch too and ignore it.
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint32_t launch_header_batch(uint4 &hdr) {
    static_assert(offsetof(RouteParams, nb) == 0 && offsetof(RouteParams, xcd_local) == 8, "header layout");
    static_assert(sizeof(RouteParams::cls_tab[0]) == 32 && kPerClass == 8, "one s_load_dwordx8 per row");
    const auto ka = __builtin_amdgcn_kernarg_segment_ptr();
    const uint32_t roff = (blockIdx.x & 7u) * 32u;
    u32x8 row;
    asm volatile("s_load_dwordx4 %0, %2, 0x0\n\t"
                 "s_load_dwordx8 %1, %2, %3 offset:%4\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&s"(hdr), "=&s"(row)
                 : "s"(ka), "s"(roff), "i"((int)offsetof(RouteParams, cls_tab)));
    const uint32_t bx = blockIdx.x >> 3;
    uint32_t bi = 63u;
    bool found = false;
#pragma unroll
    for (int j = 0; j < kPerClass; ++j) {
        if (!found && bx < (row[j] >> 6)) {
            bi = row[j] & 63u;
            found = true;
        }
    }
    return bi;
}

// One tile's input as loaded into registers: thread tid holds the tile's bytes [64 tid, 64 tid + 64)
// in v[0..3] (its own chunk: every wave-instruction still reads one contiguous 4 KiB span), and
// threads below kHalo/16 hold 16 bytes of the 2 KiB before the tile.
struct TileIn {
    uint32_t bi, t;
    uint64_t sx;   // the batch scanner's kFlagXcc granule
    uint4 v[4];
    uint4 hv;
};

template <int BLOCK, unsigned ABL>
__device__ __forceinline__ void tile_issue(const RouteParams &p, uint32_t bi, uint32_t t, TileIn &in, int tid) {
    constexpr int kTileB = BLOCK * kLaneBytes;
    constexpr int kHalo = SmemT<BLOCK>::kHalo;
    const BatchDesc &bd = p.b[bi];
    const uint32_t T0 = t * (uint32_t)kTileB;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)bd.bytes, (short)0, (int)bd.nbytes, 0x00020000);
    in.bi = bi;
    in.t = t;
    in.hv = make_uint4(0, 0, 0, 0);
    if (tid < kHalo / 16 && t > 0 && !(ABL & ABL_NO_PROLOGUE))   // zeros before the batch start
        in.hv = as_uint4(__builtin_amdgcn_raw_buffer_load_b128(rsrc, T0 - kHalo + tid * 16, 0, 0));
    if (T0 + (uint32_t)kTileB <= bd.nbytes) {   // every tile but a batch's last: no per-piece bounds test
#pragma unroll
        for (int k = 0; k < 4; ++k)
            in.v[k] = as_uint4(__builtin_amdgcn_raw_buffer_load_b128(rsrc, T0 + tid * kLaneBytes + k * 16, 0, 0));
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) in.v[k] = load16(rsrc, T0 + tid * kLaneBytes + k * 16, bd.nbytes);
    }
}

// SR_KNOB_PREFETCH (route_chunk_kernel): one dword of every 128-byte line of tile t + p.prefetch of the
// batch (the tile this XCD class runs about that many tiles later), issued after the tile's own loads;
// the value is kept to the workgroup's end (prefetch_sink), so nothing waits for it before then.
// 64 tiles ahead: C5 169.5 -> 165.4 us per 32-batch launch, 96: 164.6 (16 of 64 dead 201.3-201.6
// against 203.1-203.7 at 64; profiles/r05/prefetch_distance_r5k.jsonl); 224 (a whole round of
// resident tiles) +3 %; in route_kernel the code alone cost C2 +4 us (prefetch_cost_ab_r5j.jsonl)
__device__ __forceinline__ uint32_t prefetch_tile(const RouteParams &p, const BatchDesc &bd, uint32_t t, int tid) {
    if (!p.prefetch || tid >= 128 || t + p.prefetch >= bd.ntiles) return 0u;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)bd.bytes, (short)0, (int)bd.nbytes, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b32(rsrc, (t + p.prefetch) * 16384u + (uint32_t)tid * 128u, 0, 0);
}
__device__ __forceinline__ void prefetch_sink(uint32_t v) { asm volatile("" ::"v"(v)); }

// Route one tile (reference: sr-main.c:175-189 + process_data_line + hash + find_downstream's
// choice, for every line that ends in the tile), in two halves. First half: the tile's bytes from
// the registers of `in` into the LDS image (thread tid's chunk = image row tid), the '\n' / ':'
// masks of the thread's 64 bytes (bit i = byte 64 tid + i) into nlm / clm, and the tile's '\n'
// count published for the scanner.
template <int BLOCK, unsigned ABL>
__device__ __forceinline__ void tile_load(const RouteParams &p, SmemT<BLOCK> &sm, const TileIn &in, uint32_t epoch,
                                          uint32_t g, uint64_t &nlm, uint64_t &clm, uint32_t &c_in) {
    using S = SmemT<BLOCK>;
    constexpr int kWaves = S::kWaves;
    constexpr int kHalo = S::kHalo;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    uint64_t *const status = p.status + p.b[in.bi].sbase;

    stamp<ABL>(p, tid, g, 0);
    if (tid < kHalo / 16) img_put16(sm, tid * 16, in.hv);
    {
        // 17-dword rows: conflict-free per-lane rows; eight two-dword stores from one base address
        const uint32_t rb = lds_addr(&sm.img[(kHalo / 64 + tid) * 17]);
        ds_write2_at<0, 1>(rb, in.v[0].x, in.v[0].y);
        ds_write2_at<2, 3>(rb, in.v[0].z, in.v[0].w);
        ds_write2_at<4, 5>(rb, in.v[1].x, in.v[1].y);
        ds_write2_at<6, 7>(rb, in.v[1].z, in.v[1].w);
        ds_write2_at<8, 9>(rb, in.v[2].x, in.v[2].y);
        ds_write2_at<10, 11>(rb, in.v[2].z, in.v[2].w);
        ds_write2_at<12, 13>(rb, in.v[3].x, in.v[3].y);
        ds_write2_at<14, 15>(rb, in.v[3].z, in.v[3].w);
        uint32_t m[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (ABL & ABL_OLD_MASKS)
                m[k] = eq_mask16_dot(in.v[k], 0x0A0A0A0Au) | (eq_mask16_dot(in.v[k], 0x3A3A3A3Au) << 16);
            else
                m[k] = nl_colon_mask16(in.v[k]);
        }
        nlm = ((uint64_t)__builtin_amdgcn_perm(m[3], m[2], 0x05040100u) << 32) |
              __builtin_amdgcn_perm(m[1], m[0], 0x05040100u);
        clm = ((uint64_t)__builtin_amdgcn_perm(m[3], m[2], 0x07060302u) << 32) |
              __builtin_amdgcn_perm(m[1], m[0], 0x07060302u);
        c_in = wave_incl_add32((uint32_t)__popcll(nlm));   // also the line scan's '\n' count
        if (lane == 63) sm.wave_cnt[wave] = c_in;
    }
    wg_barrier();
    stamp<ABL>(p, tid, g, 1);
    uint32_t tile_count = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) tile_count += sm.wave_cnt[w];
    if (tid == 0) {   // publish this tile's '\n' count for the scanner
        const uint32_t x = xcc_id();
        const bool same = !(ABL & ABL_AGENT_GRANULES) && granule_ok(in.sx, epoch & 0x3FFFFFFFu, kFlagXcc) &&
                          (uint32_t)in.sx == x;
        granule_store(&status[in.t], mk_status(epoch, kFlagAgg, tile_count | ((8u | x) << 28)), same);
    }
}

// Second half: lines, hashes, shards and records of the tile whose bytes tile_load left in the
// LDS image and whose chunk masks are in nlm / clm.
template <int BLOCK, unsigned ABL>
__device__ __forceinline__ void tile_lines(const RouteParams &p, SmemT<BLOCK> &sm, const TileIn &in, uint32_t epoch,
                                           uint32_t g, uint64_t nlm, uint64_t clm, uint32_t c_in) {
    stamp<ABL>(p, threadIdx.x, g, 1);
    using S = SmemT<BLOCK>;
    constexpr int kWaves = S::kWaves;
    constexpr int kTileB = S::kTileB;
    constexpr int kHalo = S::kHalo;
    constexpr int kWin = S::kWin;
    constexpr int kPreWave = kWaves - 1;   // the wave that locates the straddling line
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const uint32_t bi = in.bi, t = in.t;
    const BatchDesc &bd = p.b[bi];
    const uint32_t nbytes = bd.nbytes;
    const uint64_t *const base_slot = p.bases + bd.sbase + t;
    const int64_t T0 = (int64_t)t * kTileB;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)bd.bytes, (short)0, (int)nbytes, 0x00020000);
    uint32_t tile_count = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) tile_count += sm.wave_cnt[w];
    if (ABL & ABL_LOAD_ONLY) {
        wg_barrier();
    } else {
    // ---- per lane: '\n' / ':' masks of its 64 contiguous bytes, segmented line-state scan -------
    const int o = tid * kLaneBytes;   // tile position of the lane's first byte (nlm / clm bit i: byte o + i)
    // Line state before each lane's chunk, by two u32 wave scans (DPP) and a prefix over the
    // earlier waves: the number of '\n' before it, and the first ':' of the line open at its start.
    //  * the colon candidate of a chunk is its first ':' after its last '\n' (or its first ':' if it
    //    holds no '\n'): the first ':' of the line open at a chunk's end is the smallest candidate
    //    from the latest chunk with a '\n' on;
    //  * key = ((8191 - C) << 17) | candidate, C = the inclusive '\n' count of the wave up to here
    //    (the same for every lane after the latest '\n', smaller before it), so a min-scan of keys
    //    takes the smallest candidate of the latest segment.
    auto lane_cand = [&](uint64_t nl, uint64_t cl) -> uint32_t {
        uint64_t cm = cl;
        if (nl) {
            const int lastb = 63 - __clzll(nl);
            cm = lastb == 63 ? 0ull : (cl & (~0ull << (lastb + 1)));
        }
        return cm ? (uint32_t)(o + __builtin_ctzll(cm)) : (uint32_t)kNone;
    };
    // the lane's first line and the first ':' of the line open at its start, from the inclusive
    // wave scans and the earlier waves' totals (sm.wave_scan)
    auto lane_state = [&](uint32_t cin, uint32_t kin, int &lf, int &ofc) {
        uint32_t p_cnt = 0, p_col = (uint32_t)kNone;   // the earlier waves: '\n' count, open line's first ':'
#pragma unroll
        for (int w = 0; w < kWaves - 1; ++w) {
            if (w < wave) {
                const uint4 ws = *(const uint4 *)&sm.wave_scan[w][0];
                p_cnt += ws.x;
                const uint32_t wc = ws.z & 0x1FFFFu;
                p_col = ws.x ? wc : min(p_col, wc);
            }
        }
        // exclusive state of this lane: the inclusive state of the lane below, on top of the prefix
        const uint32_t c_ex = wave_shr1_32(cin, 0u);
        const uint32_t k_ex = wave_shr1_32(kin, 0xFFFFFFFFu) & 0x1FFFFu;
        lf = (int)(p_cnt + c_ex);                       // tile-local index of lane's 1st line
        ofc = (int)(c_ex ? k_ex : min(p_col, k_ex));    // first ':' (in the tile) of the open line
    };
    const uint32_t k_in = wave_incl_min32(((8191u - c_in) << 17) | lane_cand(nlm, clm));
    // one '\n' at most in every chunk of the wave (the one-line-per-lane path below)
    const uint32_t multi = __ballot(__popcll(nlm) > 1) != 0ull ? 1u : 0u;
    if (lane == 63) *(uint4 *)&sm.wave_scan[wave][0] = make_uint4(c_in, 0u, k_in, multi);
    wg_barrier();
    stamp<ABL>(p, tid, g, 2);
    int lane_first, open_fc;
    lane_state(c_in, k_in, lane_first, open_fc);
    uint32_t multi_any = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) multi_any |= sm.wave_scan[w][3];

    // ---- last wave: where the line that straddles into the tile starts, its first ':' ----------
    if (wave == kPreWave) {
        int64_t s_abs = 0;
        int32_t c_pre = kNone;
        // fast window: the last 512 bytes before the tile, 8 per lane (a line of up to 512 bytes)
        const int fb = kHalo - 512 + 8 * lane;
        const uint32_t y0 = sm.img[img_dw(fb)], y1 = sm.img[img_dw(fb + 4)];
        const uint32_t nl8 = eq_mask4(y0, 0x0A0A0A0Au) | (eq_mask4(y1, 0x0A0A0A0Au) << 4);
        const uint64_t fm = __ballot(nl8 != 0);
        if (t > 0 && !(ABL & ABL_NO_PROLOGUE) && fm) {
            const int L = 63 - __builtin_clzll(fm);
            const int pos = (int)__builtin_amdgcn_readlane(fb + 31 - __builtin_clz(nl8 | 1u), L);
            s_abs = T0 - kHalo + pos + 1;
            // the line's first ':' before T0 lies in the window too
            const int b0 = pos + 1 - fb;   // first byte of the line within my 8
            const uint32_t keep = b0 <= 0 ? 0xFFu : (b0 >= 8 ? 0u : (0xFFu & ~((1u << b0) - 1u)));
            const uint32_t cm8 = (eq_mask4(y0, 0x3A3A3A3Au) | (eq_mask4(y1, 0x3A3A3A3Au) << 4)) & keep;
            const uint64_t cb = __ballot(cm8 != 0);
            if (cb) {
                const int Lc = __builtin_ctzll(cb);
                c_pre = (int)__builtin_amdgcn_readlane(fb + __builtin_ctz(cm8 | 0x100u), Lc) - kHalo;
            }
        } else if (t > 0 && !(ABL & ABL_NO_PROLOGUE)) {
            // the halo: lane l looks at LDS bytes [32l, 32l + 32) = positions T0 - 2048 + 32l ...
            const uint4 a0 = img_get16(sm, 32 * lane), a1 = img_get16(sm, 32 * lane + 16);
            const uint32_t nl32 = eq_mask16(a0, 0x0A0A0A0Au) | (eq_mask16(a1, 0x0A0A0A0Au) << 16);
            const uint64_t m = __ballot(nl32 != 0);
            if (m) {
                const int L = 63 - __builtin_clzll(m);
                const int pos = (int)__builtin_amdgcn_readlane(32 * lane + 31 - __builtin_clz(nl32 | 1u), L);
                s_abs = T0 - kHalo + pos + 1;
            } else {   // a line longer than the halo (necessarily invalid): find its exact start
                int64_t hi = T0 - kHalo;
                uint64_t mm = 0;
                int64_t a = 0;
                uint32_t nl16 = 0;
                while (hi > 0 && !mm) {
                    const int64_t lo = hi - 1024 > 0 ? hi - 1024 : 0;
                    a = lo + lane * 16;
                    nl16 = 0;
                    if (a < hi) nl16 = eq_mask16(load16(rsrc, (uint32_t)a, nbytes), 0x0A0A0A0Au);
                    mm = __ballot(nl16 != 0);
                    hi = lo;
                }
                if (mm) {
                    const int L = 63 - __builtin_clzll(mm);
                    s_abs = (int64_t)readlane64((uint64_t)(a + 31 - __builtin_clz(nl16 | 1u)), L) + 1;
                }
            }
            const int s_rel = (int)(s_abs - T0);
            if (s_rel < 0 && -s_rel <= (int)SR_MAX_LINE_LENGTH - 1) {   // could be valid: first ':' before T0
                const int b0 = kHalo + s_rel - 32 * lane;   // first LDS byte of the line within my 32
                const uint32_t keep = b0 <= 0 ? 0xFFFFFFFFu : (b0 >= 32 ? 0u : ~((1u << b0) - 1u));
                const uint32_t cm = (eq_mask16(a0, 0x3A3A3A3Au) | (eq_mask16(a1, 0x3A3A3A3Au) << 16)) & keep;
                const uint64_t cb = __ballot(cm != 0);
                if (cb) {
                    const int L = __builtin_ctzll(cb);
                    const int pos = (int)__builtin_amdgcn_readlane(32 * lane + __builtin_ctz(cm | 0x80000000u), L);
                    c_pre = pos - kHalo;
                }
            }
        }
        if (lane == 0) {
            sm.s_pre = (int32_t)(s_abs - T0);
            sm.c_pre = c_pre;
        }
    }

    // ---- per line: windows of kWin tile-local lines ------------------------------------------
    // (e, c) of the lane's lines that fall into window [wbase, wbase + kWin) into sm.lend / lcol
    auto stage = [&](int wbase, uint64_t nl, uint64_t cl, int lf, int ofc) {
        const int nc = __popcll(nl);
        if (nl && lf + nc > wbase && lf < wbase + kWin) {
            uint64_t m = nl;
            int idx = lf;
            int prevb = -1;
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                int c;
                if (prevb < 0 && ofc != kNone) {
                    c = ofc;
                } else {
                    const uint64_t below = b == 0 ? 0ull : (~0ull >> (64 - b));
                    const uint64_t above = ~0ull << (prevb + 1);
                    const uint64_t cm = cl & below & above;
                    c = cm ? o + __builtin_ctzll(cm) : kNone;
                }
                if (idx >= wbase && idx < wbase + kWin) {
                    sm.lend[idx - wbase + 1] = o + b;
                    sm.lcol[idx - wbase + 1] = c;
                }
                ++idx;
                prevb = b;
            }
        }
    };
    if (tid == 0) sm.lend[0] = 0;
    uint32_t base = (ABL & ABL_FAKE_BASE) ? t * tile_count : 0u;   // first record index of the tile
    bool have_base = (ABL & (ABL_NO_LOOKBACK | ABL_NO_LINES | ABL_FAKE_BASE)) != 0;
    // Window 0 is staged from the masks in registers; later windows (tiles of more than kWin lines)
    // recompute them from the LDS image, so that no mask or line state stays live through the hash.
    // A tile whose chunks hold one '\n' at most and whose lines fit one window (C2's shape) stages
    // each line straight from its chunk: no loop over the chunk's '\n' bits.
    if (tile_count > 0) {
        if (!multi_any && (int)tile_count <= kWin) {
            if (nlm) {
                const int b = __builtin_ctzll(nlm);
                const uint64_t cm = clm & (b == 0 ? 0ull : (~0ull >> (64 - b)));
                sm.lend[lane_first + 1] = o + b;
                sm.lcol[lane_first + 1] = open_fc != kNone ? open_fc : (cm ? o + __builtin_ctzll(cm) : kNone);
            }
        } else {
            stage(0, nlm, clm, lane_first, open_fc);
        }
    }
    for (int wbase = 0; wbase < (int)tile_count;) {
        wg_barrier();
        if (wbase == 0) stamp<ABL>(p, tid, g, 4);
        // the tile's record base is read when the first record is written (ABL_EARLY_BASE: also
        // here); the pipelined scanner has normally published it well before
        uint64_t st_early = 0;
        if (!have_base && (ABL & ABL_EARLY_BASE))
            st_early = __hip_atomic_load(base_slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!(ABL & ABL_NO_LINES)) {
            const int s_pre = sm.s_pre;
            const int c_pre = sm.c_pre;
            const int nwin = min(kWin, (int)tile_count - wbase);
            // lanes per line from the mean line length: 64-byte hash segments per lane
            // (G * 64 < kTileB / tile_count, without the division)
            int G = 1;
            while (G < 32 && (G * 64 + 1) * (int)tile_count <= kTileB) G <<= 1;
            // the line's record: verdict, shard, record base (normally long published), write
            auto finish = [&](int j, int s, int len, bool len_ok, bool fmt_ok, uint64_t h) {
                uint32_t route;
                if (!len_ok) route = SR_ROUTE_INVALID_LENGTH;
                else if (!fmt_ok) route = SR_ROUTE_INVALID_FORMAT;
                else if (ABL & KV_ALIVE) route = p.nds ? mod_magic(h, p.magic_n, p.nds) : SR_ROUTE_ALL_DEAD;   // :145
                else if (ABL & KV_DEFER1) route = defer1_probe(h, p);                                // :145
                else if (ABL & KV_DEAD1) route = dead1_probe(h, p, sm.img);                          // :145
                else if (ABL & KV_PICKS) route = chunk_probe(h, p, sm.img);                          // :145
                else route = probe_shard(h, p, nullptr, sm.img, nullptr, p.defer != 0,
                                         p.mark_tiles ? sm.img : nullptr);                          // :145
                // a probe past its first two picks goes to probe_defer_kernel: the record is marked
                // pending and the hash kept by record index (no counter: same-address atomics from
                // every wave serialise at the memory side)
                const bool deferred = !(ABL & KV_ALIVE) && route == kRouteDefer;
                if (deferred) route = kRoutePending;
                sr_record r;
                r.offset = (uint32_t)(T0 + s);
                r.length = len > 0xFFFF ? (uint16_t)0xFFFF : (uint16_t)len;
                r.route = (uint16_t)route;
                if (!have_base) {
                    stamp<ABL>(p, tid, g, 3);
                    base = granule_ok(st_early, epoch & 0x3FFFFFFFu, kFlagBase)
                               ? (uint32_t)st_early
                               : wait_base(base_slot, epoch, rsrc, (uint32_t)T0);
                    stamp<ABL>(p, tid, g, 7);
                    have_base = true;
                }
                const uint32_t rec = base + (uint32_t)j;
                if (rec < bd.max_records) {
                    if constexpr (kCountsHist<ABL>)   // the packing's key histogram (ds_add, no return)
                        if (p.hist) atomicAdd(&sm.hist[route < p.nds ? route : p.nds], 1u);
                    if (deferred) bd.dhash[rec] = h;
                    if (!(ABL & (KV_ALIVE | KV_DEFER1 | KV_DEAD1)) && route == kRoutePending && !deferred) {
                        const uint32_t slot = atomicAdd(&p.ctl->pending, 1u);
                        if (slot < p.pending_cap) p.pending[slot] = PendingLine{rec, bi, h};
                    }
                    bd.recs[rec] = r;
                    if (bd.hashes) bd.hashes[rec] = h;
                }
            };
            // One line's work: bounds, verdict, sdbm (lane gi of the line's Gl lanes takes the
            // 64-byte segments gi, gi + Gl, ...), shard, record. Gw: the wave-uniform bound of
            // the lane groups (groups are aligned to their size, so xor partners below Gl stay
            // inside the group).
            auto line_at = [&](int j, int e, int c, int s, bool act, int gi, int Gl, int Gw) {
                const int len = e - s + 1;
                const bool len_ok = len >= (int)SR_MIN_LINE_LENGTH && len <= (int)SR_MAX_LINE_LENGTH;   // :180
                const bool fmt_ok = c != kNone && c < e;                                                // :140
                uint64_t h = 0;
                if (act && len_ok && fmt_ok && !(ABL & ABL_NO_HASH)) {
                    // sdbm of [s, c) = sum over 64-byte segments k of Horner(seg_k) * K^(c - end_k)
                    const int n = c - s, nseg = (n + 63) >> 6;
                    for (int k = gi; k < nseg; k += Gl) {
                        const int a = s + 64 * k, nn = min(64, n - 64 * k);
                        const bool mid = !(ABL & (ABL_NO_MID_BASE | ABL_EARLY_BASE)) && !have_base && k == gi;
                        uint64_t hs = (ABL & ABL_OLD_HASH) ? sdbm_lds(sm, a + kHalo, nn)
                                                           : sdbm_img(sm, a + kHalo, nn, mid ? base_slot : nullptr, &st_early);
                        if (k + 1 < nseg) hs *= kpow_n(sm, c - a - nn);   // the last segment ends at c
                        h += hs;
                    }
                }
                for (int d = Gw >> 1; d >= 1; d >>= 1) {
                    const uint64_t v = shfl_xor64(h, d);
                    if (d < Gl) h += v;
                }
                if (act && gi == 0) finish(j, s, len, len_ok, fmt_ok, h);
            };
            auto line = [&](int jj, bool act, int gi, int Gl, int Gw) {
                const int j = wbase + jj;
                const int e = act ? sm.lend[jj + 1] : 0;
                int c = act ? sm.lcol[jj + 1] : kNone;
                if (j == 0 && c_pre != kNone) c = c_pre;   // the straddling line's ':' lies before T0
                const int s = (j == 0) ? s_pre : (act ? sm.lend[jj] + 1 : 0);
                line_at(j, e, c, s, act, gi, Gl, Gw);
            };
            // Lanes per line. A tile whose longest name fits its G lanes in one pass (uniform
            // lengths: C2, C4) keeps one G-lane group per line (the KV_UNIFORM kernel always). A tile
            // of mixed lengths (C5: a 64-byte line next to 1024-byte ones) gets one lane per
            // 64-byte name segment instead, the lines packed back to back over the lanes: no idle
            // lanes, one segment per lane.
            bool segs = false;               // segment layout
            bool gain2 = false;              // the segment layout saves two or more rounds
            uint32_t TL = 0;                  // lanes the segment layout needs
            // (the segment variant decides in a tile's last window, after which the lane masks and
            // line states of later windows are dead)
            const bool last_win = wbase + kWin >= (int)tile_count;
            if ((ABL & KV_SEGMENTS) && last_win) {
                // per line: 64-byte name segments, one lane each (an empty name still takes one)
                uint32_t want = 0, nsg = 0;
                if (tid < nwin) {
                    const int jj = tid, j = wbase + jj;
                    const int e = sm.lend[jj + 1];
                    int c = sm.lcol[jj + 1];
                    if (j == 0 && c_pre != kNone) c = c_pre;
                    const int s = (j == 0) ? s_pre : sm.lend[jj] + 1;
                    const int len = e - s + 1;
                    if (len >= (int)SR_MIN_LINE_LENGTH && len <= (int)SR_MAX_LINE_LENGTH && c != kNone && c < e)
                        nsg = (uint32_t)(c - s + 63) >> 6;
                    want = max(1u, nsg);
                }
                const uint32_t incl = wave_incl_add32(want);
                const uint32_t wmx = wave_incl_max32(nsg);
                if (lane == 63) {
                    sm.seg_w[wave][0] = incl;
                    sm.seg_w[wave][1] = wmx;
                }
                if (tid < 2 * S::kSegWords) reinterpret_cast<uint32_t *>(sm.seg_mask)[tid] = 0u;
                wg_barrier();
                uint32_t pre = 0, mx = 0, tot = 0;
#pragma unroll
                for (int w = 0; w < kWaves; ++w) {
                    const uint32_t v = sm.seg_w[w][0];
                    tot += v;
                    pre += w < wave ? v : 0u;
                    mx = max(mx, sm.seg_w[w][1]);
                }
                TL = __builtin_amdgcn_readfirstlane(tot);
                // rounds of lanes times segments per lane, either way; the statistics for the
                // host's choice of kernel count only the tiles that gain two or more. (A tile's
                // segments exceed its 256 lanes by a few about half the time (C5): the second round
                // then runs on the one or two waves that hold those segments, the others only meet
                // its barriers; two-segment lanes everywhere cost 3 waves x 2 segments instead.)
                const uint32_t mxs = (uint32_t)__builtin_amdgcn_readfirstlane(mx);
                const int cost_u = ((nwin * G + BLOCK - 1) / BLOCK) * (int)((mxs + (uint32_t)G - 1) / (uint32_t)G);
                const int cost_s = ((int)TL + BLOCK - 1) / BLOCK;
                segs = cost_s < cost_u;
                gain2 = cost_s + 2 <= cost_u;
                if (segs) {
                    // line starts as bits of a lane bitmap; per 64-lane word, the line covering
                    // its first lane and where that line starts
                    if (tid < nwin) {
                        const uint32_t wn = want;
                        const uint32_t st = pre + incl - want;
                        atomicOr(&sm.seg_mask[st >> 6], 1ull << (st & 63));
                        const uint32_t m = (st + 63) & ~63u;
                        if (m < st + wn) sm.seg_first[m >> 6] = (st << 16) | (uint32_t)tid;
                    }
                    wg_barrier();
                }
            }
            if (wbase == 0) stamp<ABL>(p, tid, g, 14);   // after the segment pre-pass
            if ((ABL & KV_SEGMENTS) && last_win && tid == 0) {   // the layout statistics (arrive)
                __hip_atomic_fetch_add(&p.ctl->layout[g & 7u][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (gain2)
                    __hip_atomic_fetch_add(&p.ctl->layout[g & 7u][1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (!segs) {
                for (int r0 = 0; r0 < nwin * G; r0 += BLOCK) {
                    const uint32_t x = (uint32_t)(r0 + tid);
                    const int jj = (int)(x >> __builtin_ctz((unsigned)G));
                    line(jj, jj < nwin, (int)(x & (uint32_t)(G - 1)), G, G);
                }
            } else {
                for (int r0 = 0; r0 < (int)TL; r0 += BLOCK) {
                    const uint32_t x = (uint32_t)(r0 + tid);
                    const uint32_t k = x >> 6;   // the lane word: wave-uniform
                    const bool act = x < TL;
                    // a wave without a segment in this round only meets the barrier
                    const bool live = r0 + wave * 64 < (int)TL
#ifdef SR_SEG_ONE_ROUND   // timing bound only (wrong records): no segment work past a tile's first round
                                      && r0 == 0
#endif
                        ;
                    uint64_t below = 0, part = 0;
                    int sg = 0, glast = -1, j = 0, s = 0, len = 0;
                    bool len_ok = false, fmt_ok = false;
                    if (live) {
                        const uint64_t mask = readlane64(act ? sm.seg_mask[k] : 0ull, 0);
                        const uint32_t fst = (uint32_t)__builtin_amdgcn_readfirstlane(act ? sm.seg_first[k] : 0u);
                        below = mask & (~0ull >> (63 - lane));
                        const int hb = below ? 63 - __clzll(below) : -1;   // head lane of my line here
                        const int jj = (int)(fst & 0xFFFFu) + __popcll(below) - (int)(mask & 1ull);
                        sg = below ? lane - hb : (int)(x - (fst >> 16));   // my segment of the line
                        j = wbase + jj;
                        const int e = act ? sm.lend[jj + 1] : 0;
                        int c = act ? sm.lcol[jj + 1] : kNone;
                        if (j == 0 && c_pre != kNone) c = c_pre;
                        s = (j == 0) ? s_pre : (act ? sm.lend[jj] + 1 : 0);
                        len = e - s + 1;
                        len_ok = len >= (int)SR_MIN_LINE_LENGTH && len <= (int)SR_MAX_LINE_LENGTH;   // :180
                        fmt_ok = c != kNone && c < e;                                                // :140
                        const int n = c - s;
                        const int nseg = (act && len_ok && fmt_ok) ? (n + 63) >> 6 : 0;   // 0: an empty name
                        glast = act ? max(nseg, 1) - 1 : -1;                              // the line's last lane
                        uint64_t hs = 0;
                        if (sg < nseg) {
                            const int a = s + 64 * sg, nn = min(64, n - 64 * sg);
                            const bool mid = !have_base && sg == nseg - 1;
                            hs = sdbm_img(sm, a + kHalo, nn, mid ? base_slot : nullptr, &st_early);
                            if (sg + 1 < nseg) hs *= kpow_n(sm, c - a - nn);
                        }
                        // a line's sum from the inclusive wave scan: S(x) - S(head - 1), or S(x) plus
                        // the line's part in the previous word (a line spans at most 23 lanes)
                        const uint64_t S = wave_scan64(hs, 0ull, [](uint64_t l, uint64_t r) { return l + r; });
                        const int src = hb > 0 ? hb - 1 : 0;
                        const uint64_t Sb = ((uint64_t)(uint32_t)__shfl((int)(S >> 32), src, 64) << 32) |
                                            (uint32_t)__shfl((int)(uint32_t)S, src, 64);
                        part = hb > 0 ? S - Sb : S;
                        if (lane == 63 && act && sg < glast) sm.seg_carry[k] = part;   // continues in word k + 1
                    }
                    wg_barrier();
                    if (sg == glast) {
                        const uint64_t h = below ? part : part + sm.seg_carry[k - 1];
                        finish(j, s, len, len_ok, fmt_ok, h);
                    }
                }
            }
        }

        wg_barrier();
        if (wbase == 0) stamp<ABL>(p, tid, g, 5);
        if (wbase + kWin >= (int)tile_count) break;
        if (tid == 0) sm.lend[0] = sm.lend[kWin];
        wg_barrier();
        wbase += kWin;
        {   // the lane's masks and line state again, from the image and the wave totals in LDS
            const uint32_t *const row = &sm.img[(kHalo / 64 + tid) * 17];
            uint32_t m[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) m[k] = nl_colon_mask16(make_uint4(row[4 * k], row[4 * k + 1], row[4 * k + 2], row[4 * k + 3]));
            const uint64_t nl = ((uint64_t)__builtin_amdgcn_perm(m[3], m[2], 0x05040100u) << 32) |
                                __builtin_amdgcn_perm(m[1], m[0], 0x05040100u);
            const uint64_t cl = ((uint64_t)__builtin_amdgcn_perm(m[3], m[2], 0x07060302u) << 32) |
                                __builtin_amdgcn_perm(m[1], m[0], 0x07060302u);
            const uint32_t cin = wave_incl_add32((uint32_t)__popcll(nl));
            const uint32_t kin = wave_incl_min32(((8191u - cin) << 17) | lane_cand(nl, cl));
            int lf, ofc;
            lane_state(cin, kin, lf, ofc);
            stage(wbase, nl, cl, lf, ofc);
        }
    }
    }
    stamp<ABL>(p, tid, g, 6);
}

template <int BLOCK, unsigned ABL>
__global__ __launch_bounds__(BLOCK, (KernelTraits<BLOCK, ABL>::kMinWavesPerSimd))
__attribute__((amdgpu_waves_per_eu((KernelTraits<BLOCK, ABL>::kMinWavesPerSimd), (KernelTraits<BLOCK, ABL>::kMaxWavesPerSimd)))) void route_kernel(RouteParams p) {
    using S = SmemT<BLOCK>;
    __shared__ S sm;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    if (ABL & ABL_LDS_PAD) {   // occupancy experiment: 4 KiB more LDS per workgroup
        __shared__ uint32_t pad[1024];
        if (p.nb > 1000000u) pad[tid] = tid;   // never true: keeps the array
        if (p.nb > 1000000u) p.ctl->pad1 = pad[(tid + 1) & 1023];
    }
    uint4 hdr;
    const uint32_t bi = launch_header_batch(hdr);
    if (blockIdx.x < hdr.x) {   // scanner of batch blockIdx.x (wave 0; no barriers on this path)
        // the scanner is the latency-critical link of every tile's record base: its few
        // instructions go ahead of the co-resident tiles' VALU work
        __builtin_amdgcn_s_setprio(3);
        // the batch's probed-dead bitmap starts empty (set after this launch by probe_defer_kernel,
        // probe_wide_kernel or probed_dead_kernel, sr-main.c:106; with every shard alive it stays empty)
        if (uint64_t *pd = p.b[blockIdx.x].probed_dead)
            for (uint32_t w = tid; w < p.nwords; w += BLOCK) pd[w] = 0ull;
        const uint32_t ep0 = __hip_atomic_load(&p.ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ABL & ABL_OLD_SCANNER) {
            if (wave == 0) scan_batch<BLOCK>(p, p.b[blockIdx.x], ep0, lane);
            if (tid == 0) arrive(p, blockIdx.x, ep0);
        } else {
            if (tid == 0) {
                sm.scan_head = 0;
                sm.scan_pub = 0;
                sm.scan_total = 0;
            }
            wg_barrier();
            scan_batch_split<BLOCK, ABL>(p, p.b[blockIdx.x], ep0, sm, wave, lane);
            if (tid == 64) arrive(p, blockIdx.x, ep0);   // the publisher, after its last store
        }
        return;
    }
    const uint32_t g = blockIdx.x - hdr.x;   // tile workgroup index within the launch
    stamp<ABL>(p, tid, g, 8);
    if ((ABL & ABL_STAMPS) && tid == 0) {   // placement: HW_ID (CU / SH / SE) and XCC_ID
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        p.dbg[(size_t)g * 16 + 10] = hw;
        p.dbg[(size_t)g * 16 + 11] = xcc_id();
    }
    // Launches of 8+ batches keep every batch on one XCD class (blocks b and b + 8 share an XCD):
    // a tile's predecessors then start before it on the same dispatcher, and its scanner (block
    // b, same class) sits beside them.
    if (bi >= kMaxBatches) {   // padding block of an unbalanced class
        if (tid == 0) arrive(p, blockIdx.x, __hip_atomic_load(&p.ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        return;
    }
    // the tile's loads first; the epoch, the scanner's XCD and the power tables (needed only at
    // the count publish and the hash) queue behind them
    const uint32_t t = (hdr.z ? (g >> 3) : g) - p.b[bi].tile0;   // the tile's index in its batch
    TileIn in;
    tile_issue<BLOCK, ABL>(p, bi, t, in, tid);
    const uint32_t kp = tid < S::kPowWords ? ((const uint32_t *)p.kpow)[tid] : 0u;
    // the scanner granule's load before the epoch's: the epoch's value is wanted at once (a wait for
    // every load issued before it, vmcnt counts in order), and a granule load issued after that wait
    // is a whole round trip more before the tile can publish its count (+5 % per C2 launch measured)
    in.sx = (ABL & ABL_AGENT_GRANULES) ? 0ull
                                       : __hip_atomic_load(&p.ctl->scan_xcc[bi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t ep0 = __hip_atomic_load(&p.ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (kEarlyArrive<ABL> && tid == 0) arrive_count(p, blockIdx.x);
    if (tid < S::kPowWords) ((uint32_t *)&sm.kp_lo[0])[tid] = kp;   // kp_lo | kp_hi | kp_inv are contiguous
    if (!(ABL & (KV_ALIVE | KV_DEFER1 | KV_DEAD1)) && p.dead && p.dead < p.nds && tid < 4 * (int)kMagicLds) {   // the probe's first reciprocals (probe_shard)
        const uint32_t e = (uint32_t)tid >> 2;   // divisor nds - e >= 1: entries e < nds only
        if (e < p.nds) sm.img[(uint32_t)tid * 17 + 16] = ((const uint32_t *)&p.magic[p.nds - e])[tid & 3];
    }
    if (!(ABL & (KV_ALIVE | KV_DEFER1 | KV_DEAD1)) && p.dead && p.dead < p.nds && p.nds <= 64 * kAliveLds && tid >= (int)kAliveRow0 &&
        (uint32_t)tid < kAliveRow0 + 2 * ((p.nds + 63) / 64))   // the alive words (probe_shard)
        sm.img[(uint32_t)tid * 17 + 16] = ((const uint32_t *)p.alive)[tid - kAliveRow0];
    if (!(ABL & (KV_ALIVE | KV_DEFER1)) && p.mark_tiles && tid >= (int)kMarkRow0 && (uint32_t)tid < kMarkRow0 + 2 * p.nwords)   // MARK_LDS: none yet
        sm.img[(uint32_t)tid * 17 + 16] = 0u;
    if (tid < 20) sm.img[S::kRows * 17 + tid] = 0u;
    if (kCountsHist<ABL> && p.hist && tid < kHistKeys) sm.hist[tid] = 0u;
    uint64_t nlm, clm;
    uint32_t c_in;
    tile_load<BLOCK, ABL>(p, sm, in, ep0, g, nlm, clm, c_in);
    tile_lines<BLOCK, ABL>(p, sm, in, ep0, g, nlm, clm, c_in);
    mark_tile_end<ABL>(p, sm.img, p.b[bi], t, tid);   // MARK_LDS: the dead shards this tile's probes visited
    if (kCountsHist<ABL> && p.hist) {   // the tile's key histogram for the packing (sr_route_pack_many)
        wg_barrier();
        const BatchDesc &bd = p.b[bi];
        if ((uint32_t)tid <= p.nds)
            p.hist[(size_t)(p.nds + 1) * bd.sbase + (size_t)tid * bd.ntiles + t] = sm.hist[tid];
    }
    if (tid == 0) {
        if (kEarlyArrive<ABL>) arrive_last(p, blockIdx.x, ep0);
        else arrive(p, blockIdx.x, ep0);
    }
    stamp<ABL>(p, tid, g, 9);
}

template <unsigned ABL>
__device__ __forceinline__ void mark_tile_end(const RouteParams &p, const uint32_t *img, const BatchDesc &bd, uint32_t t,
                                              int tid) {
    if ((ABL & (KV_ALIVE | KV_DEFER1)) || !p.mark_tiles || !bd.probed_dead) return;
    wg_barrier();
    if ((uint32_t)tid < p.nwords) {   // the tile's slot (no atomics)
        const uint32_t lo = img[(kMarkRow0 + 2 * (uint32_t)tid) * 17 + 16];
        const uint32_t hi = img[(kMarkRow0 + 2 * (uint32_t)tid + 1) * 17 + 16];
        p.tile_pd[(size_t)(bd.sbase + t) * p.nwords + tid] = ((uint64_t)hi << 32) | lo;
    }
}

// After a route launch with dead shards. MARK_LDS: block 0 of each batch ORs the tiles' probed-dead
// slots into the batch's bitmap (with the dead shards of its own probes, one atomic per word).
// DEFER: the probes the route kernel deferred (past their first two picks; probe_shard):
// find_downstream (sr-main.c:86-117) from the line's hash with the 16-entry register overlay; a line
// needing more goes on to probe_wide_kernel. Writes the record's route. A few percent of the records
// are deferred, so each wave first gathers the deferred record indices of a chunk of
// kDeferChunk records into LDS (ballot + popcount, no atomics) and then probes them one per lane:
// a wave runs the probe loop once per 64 deferred lines, not once per 64 records.
// The reciprocals and alive words of probe_shard in the route kernel's pad-dword layout
// (magic_from_pad, alive_pad_dword), for the kernels after it: a probe step then waits on LDS, not
// on a dependent global load per step.
constexpr uint32_t kProbePads = (kAliveRow0 + 2 * kAliveLds) * 17;
template <class P>
__device__ __forceinline__ bool probe_pad_value(const P &p, uint32_t tid, uint32_t &v) {
    if (tid < 4 * kMagicLds && (tid >> 2) < p.nds) {
        v = ((const uint32_t *)&p.magic[p.nds - (tid >> 2)])[tid & 3];
        return true;
    }
    if (p.nds <= 64 * kAliveLds && tid >= kAliveRow0 && tid < kAliveRow0 + 2 * ((p.nds + 63) / 64)) {
        v = ((const uint32_t *)p.alive)[tid - kAliveRow0];
        return true;
    }
    return false;
}
__device__ __forceinline__ void load_probe_pads(const RouteParams &p, uint32_t *pads, uint32_t tid) {
    uint32_t v;
    if (probe_pad_value(p, tid, v)) pads[tid * 17 + 16] = v;
}

constexpr uint32_t kDeferChunk = 256;   // records per wave and chunk (4 per lane)
constexpr uint32_t kDeferOrBlocks = 16; // blocks per batch that OR the tiles' probed-dead slots (MARK_LDS)
// OV: probe_shard's overlay entries, at least the snapshot's dead shards (launch_route picks 4, 8 or 16:
// two of four shards dead need two entries, not sixteen registers' worth of unrolled overlay)
template <int OV>
__global__ __launch_bounds__(256) void probe_defer_kernel(RouteParams p) {
    __shared__ uint32_t pads[kProbePads];
    __shared__ uint32_t list[4][kDeferChunk];
    __shared__ unsigned long long wg[kReplayCheckWords];   // MARK: the block's probed-dead bits
    const uint32_t bi = blockIdx.y;   // grid y = batch
    if (bi >= p.nb) return;
    const BatchDesc &bd = p.b[bi];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    uint64_t *const mark = p.mark ? bd.probed_dead : nullptr;
    // The block's independent loads first, so that their latencies overlap: the probe's pads, the
    // record count, the routes of the wave's first chunk (bounded by the capacity; masked by the
    // count below) and, in the first kDeferOrBlocks blocks, a slice of the tiles' probed-dead slots
    // (word 0; MARK_LDS in the route kernel).
    const uint32_t n = (uint32_t)min(*bd.n_out, (uint64_t)bd.max_records);
    uint32_t pv = 0;
    const bool has_pv = probe_pad_value(p, tid, pv);
    const uint32_t nor = min(gridDim.x, kDeferOrBlocks);
    uint64_t v0 = 0;
    if (mark && p.mark_tiles && blockIdx.x < nor)
        for (uint32_t t = blockIdx.x * 256u + tid; t < bd.ntiles; t += nor * 256u)
            v0 |= p.tile_pd[(size_t)(bd.sbase + t) * p.nwords];
    if (blockIdx.x >= nor && blockIdx.x * 4u * kDeferChunk >= n) return;   // uniform over the block
    const uint32_t x0 = (blockIdx.x * 4u + w) * kDeferChunk + lane;
    uint16_t r0[kDeferChunk / 64];
#pragma unroll
    for (uint32_t it = 0; it < kDeferChunk / 64; ++it) {
        const uint32_t x = x0 + 64u * it;
        r0[it] = (p.defer && x < n) ? bd.recs[x].route : (uint16_t)0;
    }
    if (has_pv) pads[tid * 17 + 16] = pv;
    if (tid < kReplayCheckWords) wg[tid] = 0ull;
    __syncthreads();
    if (mark && p.mark_tiles && blockIdx.x < nor) {   // MARK_LDS: the OR of the batch's tile slots, into this block's copy
        if (v0) atomicOr(&wg[0], (unsigned long long)v0);
        for (uint32_t q = 1; q < p.nwords; ++q) {
            uint64_t v = 0;
            for (uint32_t t = blockIdx.x * 256u + tid; t < bd.ntiles; t += nor * 256u)
                v |= p.tile_pd[(size_t)(bd.sbase + t) * p.nwords + q];
            if (v) atomicOr(&wg[q], (unsigned long long)v);
        }
    }
    const uint64_t below = (1ull << lane) - 1ull;
    bool first = true;
    for (uint32_t c = blockIdx.x * 4u + w; p.defer && c * kDeferChunk < n; c += gridDim.x * 4u) {
        const uint32_t xc = c * kDeferChunk + lane;
        uint16_t r[kDeferChunk / 64];
#pragma unroll
        for (uint32_t it = 0; it < kDeferChunk / 64; ++it) {
            const uint32_t x = xc + 64u * it;
            r[it] = x < n ? (first ? r0[it] : bd.recs[x].route) : (uint16_t)0;
        }
        first = false;
        uint32_t cnt = 0;
#pragma unroll
        for (uint32_t it = 0; it < kDeferChunk / 64; ++it) {
            const uint64_t m = __ballot(r[it] == kRoutePending);
            if (r[it] == kRoutePending) list[w][cnt + __popcll(m & below)] = xc + 64u * it;
            cnt += __popcll(m);
        }
        __builtin_amdgcn_wave_barrier();
        // every hash of the chunk's list requested before the first probe (at most four per lane)
        uint32_t xs[kDeferChunk / 64];
        uint64_t hs[kDeferChunk / 64];
#pragma unroll
        for (uint32_t it = 0; it < kDeferChunk / 64; ++it) {
            const uint32_t i = lane + 64u * it;
            xs[it] = i < cnt ? list[w][i] : 0u;
            hs[it] = i < cnt ? bd.dhash[xs[it]] : 0ull;
        }
#pragma unroll
        for (uint32_t it = 0; it < kDeferChunk / 64; ++it) {
            if (lane + 64u * it >= cnt) break;
            const uint32_t x = xs[it];
            const uint64_t h = hs[it];
            const uint32_t route = mark ? probe_shard<true, RouteParams, OV>(h, p, mark, pads, wg)
                                        : probe_shard<false, RouteParams, OV>(h, p, nullptr, pads);
            if (route == kRoutePending) {   // more than kOverlay dead probes: probe_wide_kernel
                const uint32_t slot = atomicAdd(&p.ctl->pending, 1u);
                if (slot < p.pending_cap) p.pending[slot] = PendingLine{x, bi, h};
            }
            bd.recs[x].route = (uint16_t)route;
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (mark) {   // the block's bits (p.mark: at most kAliveLds words), one atomic per nonzero word
        __syncthreads();
        if (tid < p.nwords && wg[tid])
            __hip_atomic_fetch_or(mark + tid, (uint64_t)wg[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Lines whose probe met more than kOverlay dead shards: run find_downstream (sr-main.c:86-117)
// literally on a permutation array held in LDS (N <= 65533 -> <= 128 KiB), one line at a time
// per workgroup. After each line the touched entries are restored by replaying the probe.
__global__ __launch_bounds__(64) void probe_wide_kernel(RouteParams p) {
    extern __shared__ uint16_t ds_index[];
    const uint32_t n = p.nds;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) ds_index[i] = (uint16_t)i;
    __syncthreads();
    const uint32_t np = min(__hip_atomic_load(&p.ctl->pending, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                            p.pending_cap);
    if (threadIdx.x != 0) return;
    for (uint32_t x = blockIdx.x; x < np; x += gridDim.x) {
        const PendingLine pl = p.pending[x];
        uint64_t h = pl.hash;
        uint32_t route = SR_ROUTE_ALL_DEAD, steps = 0;
        for (uint32_t i = n; i > 0; --i) {
            const uint32_t j = mod_magic(h, p.magic[i], i);
            const uint32_t k = ds_index[j];
            ++steps;
            if (alive_bit(p.alive, k)) { route = k; break; }
            if (p.b[pl.batch].probed_dead) note_dead(p.b[pl.batch].probed_dead, k);   // :106
            if (j != i - 1) {
                ds_index[j] = ds_index[i - 1];
                ds_index[i - 1] = (uint16_t)k;
            }
            h = (h * 7 + 5) / 3;
        }
        p.b[pl.batch].recs[pl.rec].route = (uint16_t)route;
        // restore the identity on every touched position
        h = pl.hash;
        for (uint32_t i = n; i > 0 && steps > 0; --i, --steps) {
            const uint32_t j = mod_magic(h, p.magic[i], i);
            ds_index[j] = (uint16_t)j;
            ds_index[i - 1] = (uint16_t)(i - 1);
            h = (h * 7 + 5) / 3;
        }
    }
}

// The dead-downstream side effect (sr-main.c:106), replayed after a launch when some shards are
// dead and a batch asked for its probed-dead bitmap: per record, the name's sdbm recomputed from the
// batch bytes (aligned dword loads, the first ':' ends it), then the probe of find_downstream with
// every dead shard it visits set in the bitmap. Lines that needed more than kOverlay dead probes were
// resolved by probe_wide_kernel, which sets their bits itself.
// The bitmap can only ever hold the snapshot's dead shards, and in a large batch every one of them is
// some line's first pick within the first few thousand lines: kReplayBlocks workgroups per batch
// (grid y = batch) stride over its records and stop as soon as the bitmap holds every dead shard.
// Each workgroup keeps its own copy of the bitmap in LDS: a lane notes a dead shard in the global
// word only when it is new to the workgroup, and one lane per stride reads the global words for the
// completion test (N <= 1024; beyond that the replay runs over every record).
constexpr uint32_t kReplayBlocks = 32;

__global__ __launch_bounds__(256) void probed_dead_kernel(RouteParams p) {
    __shared__ unsigned long long wg[kReplayCheckWords];
    __shared__ unsigned long long pushed[kReplayCheckWords];
    __shared__ uint32_t complete;
    __shared__ uint32_t pads[kProbePads];
    const uint32_t bi = blockIdx.y;
    if (bi >= p.nb) return;
    const BatchDesc &bd = p.b[bi];
    if (!bd.probed_dead) return;
    const uint32_t nw = p.nwords_check;   // 0: no workgroup copy, no completion test
    if (threadIdx.x < kReplayCheckWords) wg[threadIdx.x] = pushed[threadIdx.x] = 0ull;
    load_probe_pads(p, pads, threadIdx.x);
    const uint32_t n = (uint32_t)min(*bd.n_out, (uint64_t)bd.max_records);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)bd.bytes, (short)0, (int)bd.nbytes, 0x00020000);
    // thread 0: OR the workgroup's new bits into the global words (one atomic per word that has
    // any), and from the words' old values decide whether every dead shard is noted
    auto push = [&]() {
        bool all = nw != 0;
        for (uint32_t w = 0; w < nw; ++w) {
            const uint32_t hi = p.nds - 64 * w;
            const uint64_t full = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
            const uint64_t add = wg[w] & ~pushed[w];
            uint64_t seen = wg[w] | p.alive[w];
            if (add) {
                pushed[w] |= add;
                seen |= atomicOr((unsigned long long *)bd.probed_dead + w, (unsigned long long)add);
            } else if ((seen & full) != full) {
                seen |= __hip_atomic_load(bd.probed_dead + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            all = all && (seen & full) == full;
        }
        return all;
    };
    for (uint32_t i0 = blockIdx.x * 256u; i0 < n; i0 += gridDim.x * 256u) {
        __syncthreads();
        if (threadIdx.x == 0) complete = push() ? 1u : 0u;
        __syncthreads();
        if (complete) return;
        const uint32_t i = i0 + threadIdx.x;
        if (i >= n) continue;
        const sr_record r = bd.recs[i];
        if (r.route == SR_ROUTE_INVALID_LENGTH || r.route == SR_ROUTE_INVALID_FORMAT) continue;
        if (r.route == SR_ROUTE_ALL_DEAD) {   // every shard dead: the probe visited all of them
            if (p.dead >= p.nds && p.nds) note_all_dead(bd.probed_dead, p.nds);
            continue;
        }
        // sdbm over the bytes before the first ':' (sr-main.c:120-134): the route kernel's own when it
        // wrote them, else recomputed (the record is valid, so a ':' lies within the line)
        uint64_t h = 0;
        const uint32_t a0 = r.offset & ~3u, end = r.offset + r.length;
        bool done = bd.hashes != nullptr;
        if (done) h = bd.hashes[i];
        for (uint32_t a = a0; a < end && !done; a += 4) {
            const uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(rsrc, a, 0, 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t pos = a + (uint32_t)q;
                const uint32_t c = (x >> (8 * q)) & 0xFFu;
                if (!done && pos >= r.offset && pos < end) {
                    if (c == (uint32_t)':') done = true;
                    else h = sdbm_step(h, c);
                }
            }
        }
        (void)probe_shard<true>(h, p, bd.probed_dead, pads, nw ? wg : nullptr);
    }
    __syncthreads();   // the last stride's bits
    if (threadIdx.x == 0) (void)push();
}

}  // namespace srk
