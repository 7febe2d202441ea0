// mtu_kernel.hpp — on-device per-downstream MTU packing of a routed batch.
//
// Reference (hulu/statsd-router, /root/reference): every valid line is pushed to its downstream
// in arrival order by push_to_downstream (sr-main.c:73-83): if the downstream's active buffer
// plus the line would exceed DOWNSTREAM_BUF_SIZE (1450 B) the buffer is flushed first
// (ds_schedule_flush, sr-main.c:49-71), then the line is appended. Per downstream that is a greedy
// "next fit" over the line lengths, starting from the bytes already pending (the fill).
//
// Output (include/sr_route.h, sr_pack_packets):
//   sorted  : the batch's records regrouped stably by key: the valid lines of shard 0, 1, ...,
//             N-1 in arrival order, then every unrouted line (invalid length / format, all dead)
//             in input order (their WARN lines, sr-main.c:115,142,184, keep the input order);
//   packets : per shard with lines in the batch, its packets in order: every packet the batch
//             closes (flushed by a line that did not fit), then the shard's new pending buffer
//             (flag open). A packet is a run of consecutive `sorted` lines, led by `carry` bytes
//             of the buffer that was pending before the batch (a shard's first packet only).
//   fill_out: pending bytes per shard after the batch (0 for a shard the batch probed dead:
//             find_downstream drops its buffer, sr-main.c:106).
//
// Kernels (all on the context's stream; one wave per record tile for the sort):
//   mtu_count   per 1024-record tile, a histogram of keys (shard, or N = unrouted) in LDS;
//   mtu_scan    one workgroup: exclusive scan of the key-major histogram table = the first sorted
//               position of every (key, tile); shard line counts -> packing chunks;
//   mtu_scatter per tile, stable in-wave ranks (one ballot per distinct key) -> sorted records;
//   mtu_table   per chunk of <= 4096 lines of one shard: next-fit transfer table. From every
//               line i, next(i) = the first line that no longer fits a packet starting at i
//               (binary search over LDS prefix sums); pointer doubling gives each line's last
//               packet start in the chunk and the packets closed on the way. Then for every
//               possible incoming fill x in 0..1450: packets closed, last start, fill out;
//   mtu_chain   one workgroup: per shard, the chunks' tables composed in order from fill_in
//               (one table read per chunk), packet counts scanned into descriptor slots;
//   mtu_emit    per chunk: its packet chain from its incoming fill, by hops of 16 packets
//               (doubling) and then 16-packet walks in parallel, writing descriptors.
// Integer/byte work, latency-light: no MFMA.
#pragma once

#include "route_kernel.hpp"

namespace srk {

#ifndef SR_MTU_TILE
#define SR_MTU_TILE 1024
#endif
constexpr int kMtuTile = SR_MTU_TILE;            // records per sort tile (one wave; 1024: 16 loads in flight
                                                 // per lane, count + scatter 2-3 % faster than 512)
#ifndef SR_MTU_CHUNK
#define SR_MTU_CHUNK 4608
#endif
// sorted lines per packing chunk (the larger size): the most whose table kernel still runs eight
// workgroups per CU (18 KiB of prefix sums; 20 KiB of LDS per workgroup at most), so that a launch
// of up to 2048 x 4608 lines has every chunk resident at once
constexpr int kMtuChunk = SR_MTU_CHUNK;
constexpr int kMtuChunkSmall = 2048;             // ... the smaller: more chunks in flight, a longer chain
static_assert(kMtuChunk <= 8192 && kMtuChunk % 256 == 0 && kMtuChunkSmall % 256 == 0,
              "chunk entries hold line indices in 16 bits; whole rows of 256 threads");
constexpr int kMtuBlock = 256;                   // threads of the emit kernel (and the prefix helper's default)
#ifndef SR_MTU_TABLE_BLOCK
#define SR_MTU_TABLE_BLOCK 256
#endif
constexpr int kMtuTableBlock = SR_MTU_TABLE_BLOCK;   // threads of the table kernel
constexpr uint32_t kMtuMaxShards = 4096;
constexpr int kMtuCap = (int)SR_DOWNSTREAM_BUF_SIZE;   // 1450: sr-types.h:30
constexpr int kMtuWindow = kMtuCap / (int)SR_MIN_LINE_LENGTH + 1;   // a packet holds < 242 lines
constexpr int kMtuX = kMtuCap + 1;               // incoming fills 0..1450
constexpr uint32_t kMtuNone = 0xFFFFFFFFu;
constexpr uint16_t kMtuEnd = 0xFFFFu;
#ifndef SR_MTU_TAIL_HOPS
#define SR_MTU_TAIL_HOPS 16
#endif
constexpr int kMtuTailHops = SR_MTU_TAIL_HOPS;   // mtu_table: jumps each entry walks after the doubling
constexpr int kMtuP0 = 256;                      // prefix sums kept per chunk for the first line over the cap
static_assert(kMtuWindow <= kMtuP0, "the incoming packet closes within a chunk's first kMtuP0 lines");

constexpr int kMtuMaxBatches = 32;

// Developer ablation mask for timing the chunk kernels' phases (tools/ab_mtu.sh; results are wrong
// when set, never shipped): 1 doubling, 2 table fills, 4 emit walk, 8 next(), 16 prefix sums,
// 32 the table kernel's store of next() for emit.
#ifndef SR_MTU_SKIP
#define SR_MTU_SKIP 0
#endif

// One batch of a packing launch (user buffers). Batches are independent: each has its own pending
// bytes in and out (the downstream arrays of different data threads).
struct MtuBatchArg {
    const sr_record *recs;
    const uint64_t *n_records;
    const uint16_t *fill_in;       // [nds] pending bytes per shard before the batch (null = none)
    const uint64_t *probed_dead;   // null, or the batch's probed-dead bitmap (route kernel)
    sr_record *sorted;
    sr_packet *packets;
    uint64_t *counts;              // [0] packets, [1] valid lines, [2] lines
    uint16_t *fill_out;            // [nds]
    uint32_t max_records;
    uint32_t max_packets;
    uint32_t tile0;                // first record tile of the batch in the launch's scratch
    uint32_t chunk0;               // first chunk of the batch in the launch's scratch
    uint32_t grp0;                 // group mode: the batch's first scatter group in the launch
    const uint64_t *dhash;         // fused deferral: the route launch's deferred hashes, by record index
};

struct MtuLaunch {
    uint32_t nds, nb, tiles, chunks;   // shards; batches; record tiles and chunks of all batches
    uint32_t chunk_lines;              // lines per chunk of this launch (kMtuChunk or kMtuChunkSmall)
    uint32_t *tile_counts;             // batch b at (nds + 1) * tile0: [(nds + 1) * ntiles], key-major
    uint32_t *keys;                    // [nb][2 * nds + 4]: key starts (nds + 2) | chunk firsts (nds + 1)
    uint32_t *chunk_shard;             // [chunks]
    uint32_t *chunk_entry;             // [chunks] incoming fill
    uint32_t *chunk_open;              // [chunks] sorted position where the incoming packet began
    uint32_t *chunk_pk;                // [chunks] first descriptor the chunk writes
    uint32_t *closed;                  // [nb][nds] packets closed per shard
    uint64_t *table;                   // [chunks][kMtuX]
    uint8_t *nx;                       // [chunks][kMtuChunk] next(i) - i per line (mtu_table -> mtu_emit)
    uint16_t *plen;                    // [chunks][kMtuChunk] bytes of the packet a line starts (mtu_table -> mtu_emit)
    uint32_t *gp0;                     // [chunks][kMtuP0 + 1] the first prefix sums and the chunk's bytes
    uint64_t *dbg;                     // SR_MTU_STAMPS developer builds only: 8 timestamps per chunk
    uint32_t xcd;                      // chunk kernels: every batch's chunks on one XCD (mtu_chunk_slot)
    // group mode (sr_route_pack_many): the sort's tiles are the route kernel's 16 KiB tiles, whose key
    // histograms it wrote (RouteParams::hist, = tile_counts); the scatter's wave takes `group` of
    // them (0: the classic 1024-record tiles of mtu_count)
    uint32_t group, groups;
    // fused deferral (sr_route_pack_many / sr_route_pack_*, two or more dead shards): the route launch
    // left its deferred probes pending (no probe_defer_kernel); mtu_count_kernel<true> runs them whole
    // (find_downstream, sr-main.c:86-117), writes their routes back and notes the dead shards they visit
    // in the batches' probed-dead bitmaps (fd_mark) before counting
    ProbeArgs probe;
    uint32_t fd_mark, nwords;
    // group mode after a route launch with one dead shard: the route tiles' probed-dead slots ([tile][pd_words],
    // tile = the batch's route tiles from b.tile0), ORed into each batch's bitmap by mtu_scan_kernel (no
    // probe_defer_kernel); null: the bitmaps are complete
    const uint64_t *tile_pd;
    uint32_t pd_words, pad_pd;
    MtuBatchArg b[kMtuMaxBatches];
};
static_assert(sizeof(MtuLaunch) < 3584, "kernel argument size");

// One batch's view of the launch (what the kernels below index).
struct MtuParams {
    const sr_record *recs;
    const uint64_t *n_records;
    uint32_t max_records;
    uint32_t nds;             // shards; key nds = unrouted lines
    uint32_t ntiles;          // record tiles of the batch
    uint32_t max_chunks;      // chunks of the batch
    uint32_t chunk_lines;     // lines per chunk
    const uint16_t *fill_in;
    const uint64_t *probed_dead;
    uint32_t *tile_counts;    // [(nds + 1) * ntiles], key-major; scanned in place
    uint32_t *key_start;      // [nds + 2]: first sorted position of each key, [nds + 1] = lines
    uint32_t *chunk_first;    // [nds + 1]: first chunk of each shard, [nds] = chunks
    uint32_t *chunk_shard;
    uint64_t *table;
    uint8_t *nx;
    uint16_t *plen;
    uint32_t *gp0;
    uint32_t *chunk_entry;    // incoming fill | first line over the cap from it << 16
    uint32_t *chunk_open;     // kMtuNone: the incoming packet began before the batch
    uint32_t *chunk_pk;
    uint32_t *closed;
    sr_record *sorted;
    sr_packet *packets;
    uint64_t max_packets;
    uint64_t *counts;
    uint16_t *fill_out;
};

__device__ __forceinline__ MtuParams mtu_view(const MtuLaunch &L, uint32_t bi) {
    const MtuBatchArg &a = L.b[bi];
    MtuParams p;
    p.recs = a.recs;
    p.n_records = a.n_records;
    p.max_records = a.max_records;
    p.nds = L.nds;
    p.ntiles = (bi + 1 < L.nb ? L.b[bi + 1].tile0 : L.tiles) - a.tile0;
    p.max_chunks = (bi + 1 < L.nb ? L.b[bi + 1].chunk0 : L.chunks) - a.chunk0;
    p.chunk_lines = L.chunk_lines;
    p.fill_in = a.fill_in;
    p.probed_dead = a.probed_dead;
    p.tile_counts = L.tile_counts + (size_t)(L.nds + 1) * a.tile0;
    p.key_start = L.keys + (size_t)bi * (2 * L.nds + 4);
    p.chunk_first = p.key_start + L.nds + 2;
    p.chunk_shard = L.chunk_shard + a.chunk0;
    p.table = L.table + (size_t)a.chunk0 * kMtuX;
    p.nx = L.nx + (size_t)a.chunk0 * kMtuChunk;
    p.plen = L.plen + (size_t)a.chunk0 * kMtuChunk;
    p.gp0 = L.gp0 + (size_t)a.chunk0 * (kMtuP0 + 1);
    p.chunk_entry = L.chunk_entry + a.chunk0;
    p.chunk_open = L.chunk_open + a.chunk0;
    p.chunk_pk = L.chunk_pk + a.chunk0;
    p.closed = L.closed + (size_t)bi * L.nds;
    p.sorted = a.sorted;
    p.packets = a.packets;
    p.max_packets = a.max_packets;
    p.counts = a.counts;
    p.fill_out = a.fill_out;
    return p;
}

// The chunk slot of a chunk-kernel workgroup. With L.xcd (eight batches or more), workgroup B runs on
// XCD B % 8 (the dispatcher deals workgroups to the XCDs in turn) and takes the (B / 8)-th slot of
// the batches b = B (mod 8): every chunk of a batch on one XCD, so that the tables, next() and packet
// lengths the table kernel writes are read from that XCD's L2 by the emit kernel (whose chain walk
// reads one table entry per hop). kMtuNone: past the slots.
// (B wave-uniform, the whole wave active: lane m looks at batch x + 8m, one scan and one ballot instead
// of a loop waiting on each batch's scalar loads in turn)
__device__ __forceinline__ uint32_t mtu_chunk_slot(const MtuLaunch &L, uint32_t B) {
    if (!L.xcd) return B < L.chunks ? B : kMtuNone;
    static_assert(kMtuMaxBatches <= 8 * 64, "one lane per batch of an XCD");
    const uint32_t x = B & 7u, k = B >> 3, lane = threadIdx.x & 63u;
    const uint32_t b = x + 8u * lane;
    uint32_t s0 = 0, cnt = 0;
    if (b < L.nb) {
        s0 = L.b[b].chunk0;
        cnt = (b + 1 < L.nb ? L.b[b + 1].chunk0 : L.chunks) - s0;
    }
    const uint32_t incl = wave_incl_add32(cnt);
    const uint64_t m = __ballot(b < L.nb && k < incl);
    if (!m) return kMtuNone;
    const uint32_t j = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    return __builtin_amdgcn_readlane(s0, j) + (k - __builtin_amdgcn_readlane(incl - cnt, j));
}

// the batch owning global index g of a per-batch sequence starting at field `first` (nb <= 32; g
// wave-uniform, the whole wave active): lane j compares with batch j, one ballot (a loop waited on one
// scalar load per batch)
template <class F>
__device__ __forceinline__ uint32_t mtu_batch_of(const MtuLaunch &L, uint32_t g, F first) {
    static_assert(kMtuMaxBatches <= 64, "one lane per batch");
    const uint32_t lane = threadIdx.x & 63u;
    const bool past = lane >= 1 && lane < L.nb && g >= first(L.b[lane < kMtuMaxBatches ? lane : 0]);
    return (uint32_t)__popcll(__ballot(past));
}

__device__ __forceinline__ uint32_t mtu_lines(const MtuParams &p) {
    return (uint32_t)min(*p.n_records, (uint64_t)p.max_records);
}

__device__ __forceinline__ uint32_t mtu_key(const sr_record &r, uint32_t nds) {
    return r.route < nds ? (uint32_t)r.route : nds;
}

__device__ __forceinline__ bool mtu_dropped(const MtuParams &p, uint32_t s) {
    return p.probed_dead && ((p.probed_dead[s >> 6] >> (s & 63)) & 1ull);
}

// developer timeline (SR_MTU_STAMPS builds): s_memrealtime (100 MHz) at phase boundaries per chunk
__device__ __forceinline__ void mtu_stamp(const MtuLaunch &L, uint32_t gc, int slot) {
#ifdef SR_MTU_STAMPS
    if (threadIdx.x == 0 && L.dbg) L.dbg[(size_t)gc * 8 + slot] = __builtin_amdgcn_s_memrealtime();
#else
    (void)L, (void)gc, (void)slot;
#endif
}

// ---- sort: histogram, scan, stable scatter ----------------------------------------------------
// The tile's records, loaded up front (kMtuTile / 64 independent loads in flight per lane rather
// than one round trip per 64 records; the caller ignores positions past the batch, n > r0 >= 0).
constexpr int kMtuPerLane = kMtuTile / 64;
__device__ __forceinline__ void mtu_load_tile(const MtuParams &p, uint32_t r0, uint32_t n, int lane,
                                              sr_record (&r)[kMtuPerLane]) {   // records [r0, n) (n > r0)
#pragma unroll
    for (int k = 0; k < kMtuPerLane; ++k) {   // clamped, unconditional: the eight loads in flight together
        const uint32_t i = r0 + (uint32_t)(64 * k + lane);
        r[k] = p.recs[min(i, n - 1)];
    }
}

// The sort kernels run one record tile per wave, kMtuSortWaves tiles per workgroup (fewer, larger
// workgroups: a launch of 64-thread workgroups was dispatch-bound). Each wave has its own (nds + 1)
// counters of dynamic LDS and syncs only with itself.
constexpr int kMtuSortWaves = 4;
__device__ __forceinline__ void mtu_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// FD: the fused deferral (MtuLaunch::probe). The wave lists its tile's pending records in LDS
// (ballots, as probe_defer_kernel), every lane probes list entries (pads of reciprocals and alive
// words in LDS, the dead shards visited in the wave's LDS words, ORed into the batch's bitmap at
// the end), writes the route back into the record and counts it; the other records are counted by
// their own lanes.
template <bool FD>
__global__ __launch_bounds__(64 * kMtuSortWaves) void mtu_count_kernel(MtuLaunch L) {
    extern __shared__ uint32_t lds_hist[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t g = blockIdx.x * kMtuSortWaves + (uint32_t)wave;   // the wave's tile in the launch
    if constexpr (FD) {
        __shared__ uint32_t pads[kProbePads];
        __shared__ uint32_t plist[kMtuSortWaves][kMtuTile];
        __shared__ unsigned long long wgm[kMtuSortWaves][kReplayCheckWords];
        uint32_t pv;
        if (probe_pad_value(L.probe, threadIdx.x, pv)) pads[threadIdx.x * 17 + 16] = pv;
        if (lane < (int)kReplayCheckWords) wgm[wave][lane] = 0ull;
        __syncthreads();
        if (g >= L.tiles) return;
        const uint32_t bi = mtu_batch_of(L, g, [](const MtuBatchArg &a) { return a.tile0; });
        const MtuParams p = mtu_view(L, bi);
        const uint32_t nk = p.nds + 1, t = g - L.b[bi].tile0;
        uint32_t *hist = lds_hist + (size_t)wave * nk;
        const uint32_t n = mtu_lines(p), r0 = t * kMtuTile;
        sr_record r[kMtuPerLane];
        if (r0 < n) mtu_load_tile(p, r0, n, lane, r);
        for (uint32_t k = lane; k < nk; k += 64) hist[k] = 0;
        mtu_wave_sync();
        if (r0 >= n) {
            for (uint32_t k = lane; k < nk; k += 64) p.tile_counts[(size_t)k * p.ntiles + t] = 0u;
            return;
        }
        const uint64_t below = (1ull << lane) - 1ull;
        uint32_t cnt = 0;
#pragma unroll
        for (int k = 0; k < kMtuPerLane; ++k) {
            const uint32_t i = r0 + (uint32_t)(64 * k + lane);
            const bool valid = i < n;
            const bool pend = valid && r[k].route == kRoutePending;
            const uint64_t m = __ballot(pend);
            if (pend) plist[wave][cnt + (uint32_t)__popcll(m & below)] = i;
            cnt += (uint32_t)__popcll(m);
            if (valid && !pend) atomicAdd(&hist[mtu_key(r[k], p.nds)], 1u);
        }
        mtu_wave_sync();
        uint64_t *const mark = L.fd_mark ? const_cast<uint64_t *>(p.probed_dead) : nullptr;
        sr_record *const recs = const_cast<sr_record *>(p.recs);
        const uint64_t *const dh = L.b[bi].dhash;
        for (uint32_t j = (uint32_t)lane; j < cnt; j += 64u) {
            const uint32_t x = plist[wave][j];
            const uint64_t h = dh[x];
            const uint32_t route = mark ? probe_shard<true>(h, L.probe, mark, pads, wgm[wave])
                                        : probe_shard(h, L.probe, nullptr, pads);
            recs[x].route = (uint16_t)route;
            atomicAdd(&hist[route < p.nds ? route : p.nds], 1u);
        }
        mtu_wave_sync();
        for (uint32_t k = lane; k < nk; k += 64) p.tile_counts[(size_t)k * p.ntiles + t] = hist[k];
        if (mark && (uint32_t)lane < L.nwords && wgm[wave][lane])
            __hip_atomic_fetch_or(mark + lane, (uint64_t)wgm[wave][lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (g >= L.tiles) return;
    const uint32_t bi = mtu_batch_of(L, g, [](const MtuBatchArg &a) { return a.tile0; });
    const MtuParams p = mtu_view(L, bi);
    const uint32_t nk = p.nds + 1, t = g - L.b[bi].tile0;
    uint32_t *hist = lds_hist + (size_t)wave * nk;
    const uint32_t n = mtu_lines(p), r0 = t * kMtuTile;
    sr_record r[kMtuPerLane];
    if (r0 < n) mtu_load_tile(p, r0, n, lane, r);
    for (uint32_t k = lane; k < nk; k += 64) hist[k] = 0;
    mtu_wave_sync();
    if (r0 < n) {
#pragma unroll
        for (int k = 0; k < kMtuPerLane; ++k)
            if (r0 + (uint32_t)(64 * k + lane) < n) atomicAdd(&hist[mtu_key(r[k], p.nds)], 1u);
    }
    mtu_wave_sync();
    for (uint32_t k = lane; k < nk; k += 64) p.tile_counts[(size_t)k * p.ntiles + t] = hist[k];
}

// One workgroup of 1024 threads: exclusive scan of the key-major table (position of (key, tile)
// = lines of smaller keys + lines of the same key in earlier tiles), key starts, packing chunks.
__global__ __launch_bounds__(1024) void mtu_scan_kernel(MtuLaunch L) {
    const MtuParams p = mtu_view(L, blockIdx.x);
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry_s;
    __shared__ unsigned long long pd_or[kReplayCheckWords];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t nk = p.nds + 1, ntiles = p.ntiles;
    const size_t total = (size_t)nk * ntiles;
    // L.tile_pd (one dead shard, sr-main.c:106): the batch's probed-dead bitmap = the OR of its route tiles'
    // slots (their probes' marks), issued first so that the loads overlap the scan
    const bool or_slots = L.tile_pd && p.probed_dead && L.pd_words <= kReplayCheckWords;
    const uint64_t *const slots = or_slots ? L.tile_pd + (size_t)L.b[blockIdx.x].tile0 * L.pd_words : nullptr;
    uint64_t v0 = 0;
    if (or_slots)
        for (uint32_t t = tid; t < ntiles; t += 1024) v0 |= slots[(size_t)t * L.pd_words];
    if (tid < (int)kReplayCheckWords) pd_or[tid] = 0ull;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    if (or_slots) {
        if (v0) atomicOr(&pd_or[0], (unsigned long long)v0);
        for (uint32_t w = 1; w < L.pd_words; ++w) {
            uint64_t v = 0;
            for (uint32_t t = tid; t < ntiles; t += 1024) v |= slots[(size_t)t * L.pd_words + w];
            if (v) atomicOr(&pd_or[w], (unsigned long long)v);
        }
    }
    // 16 rows of 64 consecutive entries per wave and round (coalesced loads and stores, each row scanned
    // in registers): the route kernel's tile histograms (group mode) are 1024 tiles per 16 MiB batch, so
    // a batch of 16 shards scans 17 k entries
    constexpr int kScanPer = 16;
    for (size_t b0 = 0; b0 < total; b0 += 1024 * kScanPer) {
        const size_t wb = b0 + (size_t)wave * 64 * kScanPer + lane;
        uint32_t v[kScanPer], s = 0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            const size_t i = wb + 64 * k;
            v[k] = i < total ? p.tile_counts[i] : 0u;
        }
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {   // v[k]: exclusive within the wave's rows; s: their total
            const uint32_t incl = wave_incl_add32(v[k]);
            const uint32_t x = v[k];
            v[k] = s + incl - x;
            s += __builtin_amdgcn_readlane(incl, 63);
        }
        if (lane == 0) wsum[wave] = s;
        __syncthreads();
        uint32_t before = carry_s;
        for (int w = 0; w < wave; ++w) before += wsum[w];
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            const size_t i = wb + 64 * k;
            if (i < total) p.tile_counts[i] = before + v[k];
        }
        __syncthreads();
        if (tid == 1023) carry_s = before + s;
        __syncthreads();
    }
    const uint32_t n = mtu_lines(p);
    if (or_slots && (uint32_t)tid < L.pd_words)   // (the scan's barriers ordered every OR before this)
        const_cast<uint64_t *>(p.probed_dead)[tid] = pd_or[tid];
    for (uint32_t k = tid; k < nk; k += 1024) p.key_start[k] = ntiles ? p.tile_counts[(size_t)k * ntiles] : 0u;
    if (tid == 0) {
        p.key_start[nk] = n;
        p.counts[2] = n;
    }
    __syncthreads();
    // chunks per shard, exclusive scan over shards (serial per thread slice, then across threads)
    const uint32_t per = (p.nds + 1023) / 1024;
    uint32_t loc = 0;
    for (uint32_t s = tid * per; s < (tid + 1) * per && s < p.nds; ++s) {
        const uint32_t c = p.key_start[s + 1] - p.key_start[s];
        loc += (c + p.chunk_lines - 1) / p.chunk_lines;
    }
    const uint32_t incl = wave_incl_add32(loc);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - loc;
    for (int w = 0; w < wave; ++w) run += wsum[w];
    for (uint32_t s = tid * per; s < (tid + 1) * per && s < p.nds; ++s) {
        p.chunk_first[s] = run;
        const uint32_t c = p.key_start[s + 1] - p.key_start[s];
        const uint32_t nc = (c + p.chunk_lines - 1) / p.chunk_lines;
        for (uint32_t j = 0; j < nc; ++j)
            if (run + j < p.max_chunks) p.chunk_shard[run + j] = s;
        run += nc;
    }
    if (tid == 1023) {
        p.chunk_first[p.nds] = run;
        p.counts[1] = p.key_start[p.nds];
        if (run == 0) p.counts[0] = 0;   // (mtu_emit<WALK> writes it otherwise)
    }
    // the pending bytes of shards without lines (mtu_emit<WALK> writes the others')
    for (uint32_t s = tid; s < p.nds; s += 1024)
        if (p.key_start[s + 1] == p.key_start[s]) {
            const uint32_t x = p.fill_in ? min((uint32_t)p.fill_in[s], (uint32_t)kMtuCap) : 0u;
            const bool dropped = or_slots ? ((pd_or[s >> 6] >> (s & 63)) & 1ull) != 0 : mtu_dropped(p, s);
            p.fill_out[s] = dropped ? 0 : (uint16_t)x;
        }
}

#ifndef SR_SCATTER_WPE
#define SR_SCATTER_WPE 1   // minimum waves per SIMD the scatter kernel is compiled for (developer A/B)
#endif
__global__ __launch_bounds__(64 * kMtuSortWaves) __attribute__((amdgpu_waves_per_eu(SR_SCATTER_WPE)))
void mtu_scatter_kernel(MtuLaunch L) {
    extern __shared__ uint32_t lds_pos[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t g = blockIdx.x * kMtuSortWaves + (uint32_t)wave;
    if (g >= L.tiles) return;
    const uint32_t bi = mtu_batch_of(L, g, [](const MtuBatchArg &a) { return a.tile0; });
    const MtuParams p = mtu_view(L, bi);
    const uint32_t nk = p.nds + 1, t = g - L.b[bi].tile0;
    uint32_t *pos = lds_pos + (size_t)wave * nk;   // (plain LDS accesses; the wave syncs below order them)
    const uint32_t n = mtu_lines(p), r0 = t * kMtuTile;
    if (r0 >= n) return;
    sr_record rr[kMtuPerLane];
    mtu_load_tile(p, r0, n, lane, rr);
    for (uint32_t k = lane; k < nk; k += 64) pos[k] = p.tile_counts[(size_t)k * p.ntiles + t];
    mtu_wave_sync();
    const uint64_t lt = (1ull << lane) - 1ull;
    // every key before the first store: the loads are waited for here, not inside the rank loops
    // (a loop that stores cannot count its own stores, so a load first used inside it costs a
    // wait for every store before it)
    uint32_t keys[kMtuPerLane];
#pragma unroll
    for (int ck = 0; ck < kMtuPerLane; ++ck) keys[ck] = mtu_key(rr[ck], p.nds);
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the tile's records are in registers
    const uint32_t kbits = nk > 1 ? 32u - (uint32_t)__clz(nk - 1u) : 0u;   // bits of the largest key
#pragma unroll
    for (int ck = 0; ck < kMtuPerLane; ++ck) {
        const uint32_t i = r0 + (uint32_t)(64 * ck + lane);
        const bool valid = i < n;
        const uint32_t key = keys[ck];
        // stable in-wave ranks: the lanes holding my key, one ballot per key bit (not per distinct key)
        uint64_t same = __ballot(valid);
        for (uint32_t b = 0; b < kbits; ++b) {
            const bool bit = ((key >> b) & 1u) != 0;
            const uint64_t bm = __ballot(bit);
            same &= bit ? bm : ~bm;
        }
        const uint32_t base = pos[key];
        mtu_wave_sync();   // every lane's read before a leader's write
        if (valid) {
            p.sorted[base + (uint32_t)__popcll(same & lt)] = rr[ck];
            if (!(same & lt)) pos[key] = base + (uint32_t)__popcll(same);   // the key's first lane
        }
        mtu_wave_sync();
    }
}

// Group mode (sr_route_pack_many): wave g sorts the records of route tiles [q G, q G + G) of its
// batch, whose per-key histograms the route kernel published and mtu_scan turned into positions
// (pos[k][t] = the sorted position of tile t's first key-k record). The tiles' records are one
// input range [R(t0), R(t1)) with R(t) = sum over keys of pos[k][t] - pos[k][0], and for every key
// the group's records follow each other in the sorted order from pos[k][t0]: the classic scatter over
// that range in rounds of kMtuTile records, no count pass over the records before it.
__global__ __launch_bounds__(64 * kMtuSortWaves) void mtu_scatter_groups_kernel(MtuLaunch L) {
    extern __shared__ uint32_t lds_pos[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t g = blockIdx.x * kMtuSortWaves + (uint32_t)wave;
    if (g >= L.groups) return;
    const uint32_t bi = mtu_batch_of(L, g, [](const MtuBatchArg &a) { return a.grp0; });
    const MtuParams p = mtu_view(L, bi);
    const uint32_t nk = p.nds + 1, q = g - L.b[bi].grp0, nt = p.ntiles;
    const uint32_t t0 = q * L.group, t1 = min(t0 + L.group, nt);
    uint32_t *pos = lds_pos + (size_t)wave * nk;
    const uint32_t n = mtu_lines(p);
    if (t0 >= nt) return;
    uint32_t a0 = 0, a1 = 0;
    for (uint32_t k = (uint32_t)lane; k < nk; k += 64) {
        const uint32_t *col = p.tile_counts + (size_t)k * nt;
        const uint32_t b0 = col[0], v0 = col[t0];
        pos[k] = v0;
        a0 += v0 - b0;
        a1 += (t1 < nt ? col[t1] : col[0]) - b0;
    }
    const uint32_t r0 = wave_add32(a0);
    const uint32_t r1 = t1 < nt ? wave_add32(a1) : n;
    mtu_wave_sync();
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t kbits = nk > 1 ? 32u - (uint32_t)__clz(nk - 1u) : 0u;
    for (uint32_t rb = r0; rb < r1; rb += kMtuTile) {
        const uint32_t re = min(rb + (uint32_t)kMtuTile, r1);
        const uint32_t rows = (re - rb + 63u) >> 6;   // wave-uniform: a group of long lines is short
        sr_record rr[kMtuPerLane];
#pragma unroll
        for (int k = 0; k < kMtuPerLane; ++k)
            if ((uint32_t)k < rows) rr[k] = p.recs[min(rb + (uint32_t)(64 * k + lane), re - 1)];
        uint32_t keys[kMtuPerLane];
#pragma unroll
        for (int ck = 0; ck < kMtuPerLane; ++ck) keys[ck] = (uint32_t)ck < rows ? mtu_key(rr[ck], p.nds) : 0u;
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the round's records are in registers
#pragma unroll
        for (int ck = 0; ck < kMtuPerLane; ++ck) {
            if ((uint32_t)ck >= rows) continue;   // wave-uniform
            const uint32_t i = rb + (uint32_t)(64 * ck + lane);
            const bool valid = i < re;
            const uint32_t key = keys[ck];
            uint64_t same = __ballot(valid);
            for (uint32_t b = 0; b < kbits; ++b) {
                const bool bit = ((key >> b) & 1u) != 0;
                const uint64_t bm = __ballot(bit);
                same &= bit ? bm : ~bm;
            }
            const uint32_t base = pos[key];
            mtu_wave_sync();   // every lane's read before a leader's write
            if (valid) {
                p.sorted[base + (uint32_t)__popcll(same & lt)] = rr[ck];
                if (!(same & lt)) pos[key] = base + (uint32_t)__popcll(same);
            }
            mtu_wave_sync();
        }
    }
}

// ---- packing: per-chunk next-fit tables -------------------------------------------------------
#ifndef SR_MTU_HOP
#define SR_MTU_HOP 16
#endif
constexpr int kMtuHop = SR_MTU_HOP;   // packets per anchor of the emit walk (a power of two)
template <int CH>
struct MtuEmitSmem {
    alignas(16) uint8_t nx[CH];   // next(i) - i (1 .. kMtuWindow - 1), 0 = none in the chunk
    uint16_t J[CH];               // kMtuHop packet starts ahead on the chain (kMtuEnd: it ends first)
    uint16_t anchor[CH / kMtuHop + 2];
    uint32_t nanchor;
    uint32_t bc[4];               // WALK: the chunk's incoming fill, first line over the cap, open, first slot
};

struct MtuChunk {
    uint32_t shard, pos0, cnt;
    bool last;
};

__device__ __forceinline__ bool mtu_chunk_of(const MtuParams &p, uint32_t c, MtuChunk &ck) {
    if (c >= min(p.chunk_first[p.nds], p.max_chunks)) return false;
    ck.shard = p.chunk_shard[c];
    const uint32_t s0 = p.key_start[ck.shard], s1 = p.key_start[ck.shard + 1];
    ck.pos0 = s0 + (c - p.chunk_first[ck.shard]) * p.chunk_lines;
    ck.cnt = min(p.chunk_lines, s1 - ck.pos0);
    ck.last = ck.pos0 + ck.cnt == s1;
    return true;
}

// first chunk-local j with x + P[j] > cap (P inclusive; the caller knows one exists below hi)
__device__ __forceinline__ uint32_t mtu_first_over(const uint32_t *P, uint32_t lo, uint32_t hi, uint32_t lim) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (P[mid] > lim) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// LDS prefix sums of the chunk's lengths. Wave w owns lines [1024 w, 1024 w + 1024), lane-
// interleaved (line 1024 w + 64 k + lane): coalesced record loads, conflict-free LDS stores, the
// running sum carried across the wave's 16 rows by DPP scans; one barrier for the wave offsets.
template <int CH, int NT = kMtuBlock>
__device__ __forceinline__ void mtu_chunk_prefix(const MtuParams &p, const MtuChunk &ck, uint32_t *P,
                                                 uint32_t *wsum, uint32_t &lmin, uint32_t &lmax) {
    constexpr int kMtuPer = CH / NT, kWaves = NT / 64;
    if (SR_MTU_SKIP & 16) {
        for (uint32_t i = threadIdx.x; i < (uint32_t)CH; i += NT) P[i] = 64u * (i + 1);
        lmin = lmax = 64u;
        __syncthreads();
        return;
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t base = (uint32_t)wave * (CH / (NT / 64)) + (uint32_t)lane;
    uint32_t v[kMtuPer];
#pragma unroll
    for (int k = 0; k < kMtuPer; ++k) {   // unconditional (clamped) loads: all 16 in flight together
        const uint32_t i = base + 64u * k;
        const uint32_t len = p.sorted[ck.pos0 + min(i, ck.cnt - 1)].length;
        v[k] = i < ck.cnt ? len : 0u;
    }
    uint32_t mn = 0xFFFFFFFFu, mx = 0;   // the chunk's shortest and longest line (bounds next())
#pragma unroll
    for (int k = 0; k < kMtuPer; ++k) {
        const bool in = base + 64u * k < ck.cnt;
        mn = min(mn, in ? v[k] : 0xFFFFFFFFu);
        mx = max(mx, v[k]);
    }
    mn = wave_incl_min32(mn);
    mx = wave_incl_max32(mx);
    uint32_t carry = 0;
#pragma unroll
    for (int k = 0; k < kMtuPer; ++k) {
        v[k] = wave_incl_add32(v[k]) + carry;
        carry = (uint32_t)__builtin_amdgcn_readlane((int)v[k], 63);
    }
    if (lane == 63) {
        wsum[wave] = carry;
        wsum[kWaves + wave] = mn;
        wsum[2 * kWaves + wave] = mx;
    }
    __syncthreads();
    uint32_t add = 0;
    for (int w = 0; w < wave; ++w) add += wsum[w];
    lmin = wsum[kWaves];
    lmax = wsum[2 * kWaves];
    for (int w = 1; w < kWaves; ++w) {
        lmin = min(lmin, wsum[kWaves + w]);
        lmax = max(lmax, wsum[2 * kWaves + w]);
    }
#pragma unroll
    for (int k = 0; k < kMtuPer; ++k) P[base + 64u * k] = v[k] + add;
    __syncthreads();
}

// table[c][x] = (first line over the cap << 48) | (packets closed << 32) | (last packet start << 16,
// 0xFFFF = none) | fill after (a chunk closes at most kMtuChunk + 1 packets: 16 bits).
// One array of LDS: the prefix sums, overwritten by the doubling words once next() is in registers
// (its searches done), plus the first kMtuP0 prefix sums (the incoming fill's first line over the cap
// is always among them) and one table entry per possible first line. 4096-line chunks: 19 KiB of
// LDS and at most 64 VGPRs, so that eight workgroups share a CU and every chunk of a C2 launch is
// resident at once (round 3's kernel held P and the doubling words apart: 32 KiB, five per CU).
// next() and the doubling run in halves of the thread's rows to stay within the registers. For
// mtu_emit: next(i) - i and the bytes of the packet line i would start (both per line), the first
// prefix sums and the chunk's bytes.
template <int CH>
struct MtuTableSmem {
    union {
        uint32_t P[CH];        // inclusive prefix of the chunk's line lengths, then the doubling words:
                               // last packet start reached from here << 16 | packets closed on the way
        uint64_t e[kMtuP0];    // at the end, per first line j: packets closed << 32 | last start << 16 | fill out
    };
    uint32_t P0[kMtuP0];   // P[0 .. kMtuP0 - 1]
    uint32_t wsum[48];     // the prefix scan's wave sums, then the waves' shortest and longest lines
};
static_assert(kMtuChunkSmall >= 2 * kMtuP0, "the entries fit over the doubling words");

template <int CH, int NT = kMtuTableBlock>
__global__ __launch_bounds__(NT, 8) void mtu_table_kernel(MtuLaunch L) {
    constexpr int kMtuPer = CH / NT;
    constexpr int kHalf = kMtuPer >= 16 ? kMtuPer / 2 : kMtuPer;   // rows per pass
    static_assert(NT >= kMtuP0, "one thread per kept prefix sum");
    __shared__ MtuTableSmem<CH> sm;
    MtuChunk ck;
    const uint32_t gs = mtu_chunk_slot(L, blockIdx.x);
    if (gs == kMtuNone) return;
    const uint32_t bi = mtu_batch_of(L, gs, [](const MtuBatchArg &a) { return a.chunk0; });
    const MtuParams p = mtu_view(L, bi);
    const uint32_t c = gs - L.b[bi].chunk0;
    if (!mtu_chunk_of(p, c, ck)) return;
    const uint32_t tid = threadIdx.x;
    mtu_stamp(L, gs, 0);
    uint32_t lmin, lmax;
    mtu_chunk_prefix<CH, NT>(p, ck, sm.P, sm.wsum, lmin, lmax);
    mtu_stamp(L, gs, 1);
    const uint32_t cnt = ck.cnt, total = sm.P[cnt - 1];
    uint32_t *gp0 = p.gp0 + (size_t)c * (kMtuP0 + 1);
    if (tid < (uint32_t)kMtuP0) {
        const uint32_t v = sm.P[min(tid, cnt - 1)];
        sm.P0[tid] = v;
        gp0[tid] = v;
    }
    if (tid == 0) gp0[kMtuP0] = total;
    // next(i) for rows k (lines tid + NT k), from the inclusive prefix P: the last line lo that still
    // fits a packet starting at i (P[lo] <= lim = P[i - 1] + cap), next = lo + 1 (kMtuEnd: the
    // chunk's end comes first), by a fixed 8-step search over the 256 lines after i (a packet holds
    // fewer than 242). Every LDS read is unconditional at a clamped index (a read under a per-lane
    // condition becomes a branch with its own wait); past the chunk the clamped read gives
    // P[cnt - 1] = total. kHalf rows at a time (registers), results packed two per register.
    // The chunk's line lengths bound the search (workgroup-uniform): a packet from i holds at least
    // cap / lmax lines and at most cap / lmin (a line over the cap is a packet alone), so lo lies in
    // [i + lo_a, i + lo_b], inside the span searched from i + lo_a; with one line length (C2-C4)
    // the span is 1 and no step runs.
    const uint32_t lo_a = lmax && lmax <= (uint32_t)kMtuCap ? (uint32_t)kMtuCap / lmax - 1u : 0u;
    const uint32_t lo_b = !lmin ? 255u : lmin <= (uint32_t)kMtuCap ? (uint32_t)kMtuCap / lmin - 1u : 0u;
    const uint32_t d = lo_b - lo_a;   // the smallest power of two span > d
    const uint32_t span = d >= 128u ? 256u : d ? 2u << (31 - __builtin_clz(d)) : 1u;
    uint32_t nxp[(kMtuPer + 1) / 2];
    uint8_t *gnx = p.nx + (size_t)c * kMtuChunk;
    uint16_t *gpl = p.plen + (size_t)c * kMtuChunk;
#pragma unroll
    for (int h = 0; h < kMtuPer; h += kHalf) {
        uint32_t lo[kHalf], lim[kHalf];
#pragma unroll
        for (int k = 0; k < kHalf; ++k) {
            const uint32_t i = tid + (uint32_t)(h + k) * NT;
            lo[k] = i + lo_a;   // P[i + lo_a] <= lim (or the chunk ends first: see end)
            const uint32_t pm = sm.P[min(i ? i - 1 : 0u, cnt - 1)];
            lim[k] = pm * (uint32_t)(i != 0) + (uint32_t)kMtuCap;
        }
        for (uint32_t step = span >> 1; step; step >>= 1) {   // 0-8 steps, a workgroup-uniform loop
#pragma unroll
            for (int k = 0; k < kHalf; ++k) {
                const uint32_t t = lo[k] + step;
                lo[k] = sm.P[min(t, cnt - 1)] <= lim[k] ? t : lo[k];
            }
        }
#pragma unroll
        for (int k = 0; k < kHalf; ++k) {
            const uint32_t i = tid + (uint32_t)(h + k) * NT;
            const bool end = total <= lim[k];
            const uint32_t nxt = (i >= cnt || end) ? (uint32_t)kMtuEnd : lo[k] + 1;
            // the packet from line i: up to next(i) (its last line lo), or to the chunk's end
            const uint32_t pe = end ? total : sm.P[min(lo[k], cnt - 1)];
            if (i < cnt) {
                gnx[i] = nxt == kMtuEnd ? 0 : (uint8_t)(nxt - i);
                gpl[i] = (uint16_t)(pe - (lim[k] - (uint32_t)kMtuCap));
            }
            const int r = h + k;
            if (r & 1) nxp[r >> 1] |= nxt << 16;
            else nxp[r >> 1] = nxt;
        }
    }
    __syncthreads();   // every search's reads of P done: the array becomes the doubling words
#pragma unroll
    for (int k = 0; k < kMtuPer; ++k) {
        const uint32_t i = tid + (uint32_t)k * NT;
        const uint32_t nxt = (nxp[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
        sm.P[i] = nxt == kMtuEnd ? i << 16 : (nxt << 16) | 1u;   // past the chunk: self loops
    }
    __syncthreads();
    mtu_stamp(L, gs, 2);
    // pointer doubling: ld -> the last packet start of the chain and the packets closed on it. A
    // chain closes at most 2 * total / (cap + 1) + 1 packets (two consecutive closed packets exceed
    // the cap together), and at most cnt / (lo_a + 1) (a closed packet holds lo_a + 1 lines or more),
    // so that many jumps suffice. In place, one barrier per round: a neighbour read mid-round has
    // jumped at least as far as at the round's start, so after r rounds every jump spans >= 2^r
    // starts (or ends the chain). Only the first hi lines' chains are read, so the rounds stop once
    // kMtuTailHops jumps finish every chain, and those lines walk the rest (each word is a valid
    // jump: (start reached << 16) | packets closed, 0 closed = the chain's last start).
    const uint32_t kb = min(min(cnt, 2u * total / (uint32_t)(kMtuCap + 1) + 2u), cnt / (lo_a + 1u) + 2u);
    for (uint32_t span = 1; span * (uint32_t)kMtuTailHops < kb; span <<= 1) {
#pragma unroll
        for (int h = 0; h < kMtuPer; h += kHalf) {
            uint32_t v[kHalf], w[kHalf];
#pragma unroll
            for (int k = 0; k < kHalf; ++k) v[k] = sm.P[tid + (uint32_t)(h + k) * NT];
#pragma unroll
            for (int k = 0; k < kHalf; ++k) w[k] = sm.P[v[k] >> 16];
#pragma unroll
            for (int k = 0; k < kHalf; ++k)
                sm.P[tid + (uint32_t)(h + k) * NT] = (w[k] & 0xFFFF0000u) | ((v[k] + w[k]) & 0xFFFFu);
        }
        __syncthreads();
    }
    mtu_stamp(L, gs, 3);
    // one entry per possible first line j (< 242 <= kMtuP0): the fill out is the bytes of the open
    // packet from the last start l, the packet length stored above for l (this workgroup's own
    // global writes, ordered before the barriers since)
    const uint32_t hi = min(cnt, (uint32_t)kMtuWindow);
    uint64_t ev = 0;
    if (tid < hi) {
        const uint32_t v = sm.P[tid];
        uint32_t l = v >> 16, closed = v & 0xFFFFu;
        for (uint32_t w = sm.P[l]; w & 0xFFFFu; w = sm.P[l]) {   // at most kMtuTailHops jumps
            closed += w & 0xFFFFu;
            l = w >> 16;
        }
        ev = ((uint64_t)(1u + closed) << 32) | ((uint64_t)l << 16) | gpl[l];
    }
    __syncthreads();   // every read of the doubling words before the entries overwrite them
    if (tid < hi) sm.e[tid] = ev;
    __syncthreads();
    // incoming fills x0 .. x0 + per - 1 per thread: the first line over the cap moves down with x
    constexpr uint32_t per = (kMtuX + NT - 1) / NT;
    uint64_t *row = p.table + (size_t)c * kMtuX;
    const uint32_t x0 = tid * per;
    uint32_t j = 0;
    bool first = true;
    for (uint32_t x = x0; x < x0 + per && x < (uint32_t)kMtuX; ++x) {
        uint64_t e;
        if (x + total <= (uint32_t)kMtuCap) {
            e = (0xFFFFull << 16) | (x + total);
        } else {
            const uint32_t lim = (uint32_t)kMtuCap - x;
            if (first) {
                j = mtu_first_over(sm.P0, 0, hi - 1, lim);
                first = false;
            } else {
                while (j > 0 && sm.P0[j - 1] > lim) --j;
            }
            e = ((uint64_t)j << 48) | sm.e[j];
        }
        row[x] = e;
    }
    mtu_stamp(L, gs, 4);
}

// One workgroup: the chunks of every shard composed in order, descriptor slots scanned.
__global__ __launch_bounds__(1024) void mtu_chain_kernel(MtuLaunch L) {
    const MtuParams p = mtu_view(L, blockIdx.x);
    __shared__ uint32_t wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t per = (p.nds + 1023) / 1024;
    uint32_t loc = 0;
    for (uint32_t s = tid * per; s < (tid + 1) * per && s < p.nds; ++s) {
        uint32_t x = p.fill_in ? p.fill_in[s] : 0u, open = kMtuNone, closed = 0;
        if (x > (uint32_t)kMtuCap) x = kMtuCap;
        const uint32_t c0 = p.chunk_first[s], c1 = min(p.chunk_first[s + 1], p.max_chunks);
        for (uint32_t c = c0; c < c1; ++c) {
            const uint64_t e = p.table[(size_t)c * kMtuX + x];
            p.chunk_entry[c] = x | ((uint32_t)(e >> 48) << 16);
            p.chunk_open[c] = open;
            p.chunk_pk[c] = closed;   // shard-relative until the scan below
            const uint32_t cl = (uint32_t)(e >> 32) & 0xFFFFu;
            if (cl) {
                closed += cl;
                open = p.key_start[s] + (c - c0) * p.chunk_lines + (uint32_t)((e >> 16) & 0xFFFFu);
            }
            x = (uint32_t)(e & 0xFFFFu);
        }
        p.fill_out[s] = mtu_dropped(p, s) ? 0 : (uint16_t)x;
        loc += closed + (c1 > c0 ? 1u : 0u);
        p.closed[s] = closed;
    }
    const uint32_t incl = wave_incl_add32(loc);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - loc;
    for (int w = 0; w < wave; ++w) run += wsum[w];
    for (uint32_t s = tid * per; s < (tid + 1) * per && s < p.nds; ++s) {
        const uint32_t c0 = p.chunk_first[s], c1 = min(p.chunk_first[s + 1], p.max_chunks);
        for (uint32_t c = c0; c < c1; ++c) p.chunk_pk[c] += run;
        run += p.closed[s] + (c1 > c0 ? 1u : 0u);
    }
    if (tid == 1023) p.counts[0] = run;
}

__device__ __forceinline__ void mtu_put(const MtuParams &p, uint32_t k, uint32_t first, uint32_t nlines,
                                        uint32_t shard, uint32_t length, uint32_t carry, uint32_t open) {
    if (k < p.max_packets) {
        sr_packet d;
        d.first = first;
        d.nlines = (uint16_t)nlines;
        d.shard = (uint16_t)shard;
        d.length = (uint16_t)length;
        d.carry = (uint16_t)carry;
        d.open = open;
        p.packets[k] = d;
    }
}

// The chunk's packet chain (the first line that does not fit the incoming packet, then next()):
// four rounds of pointer doubling give every line the start kMtuHop packets ahead (J); one thread
// walks the chain by those hops, leaving an anchor every kMtuHop packets; then every anchor's
// thread walks its kMtuHop packets by next() (LDS), loads their lengths (the table kernel's bytes per
// packet start, all loads in flight together) and writes their descriptors (rank = 16 q + step).
// The chain's first line j comes with the chunk's incoming fill (mtu_chain, from the table): no
// prefix sums in LDS, so that every chunk of a launch is resident at once.
//
// WALK (a batch of at most 64 shards): no mtu_chain kernel. Wave 0 of every chunk walks the tables
// itself, one lane per shard of the batch, all lanes at once: a lane before the chunk's shard its
// whole chain from the shard's fill_in (the shard's packet total), the chunk's own shard's lane up to
// the chunk (its incoming fill, where its open packet began, the packets closed before it). The
// chunk's first descriptor is the totals of the shards before it plus its own shard's closed
// packets. A shard's last chunk writes its fill out, the batch's last chunk the batch's packet count
// (shards without lines: mtu_scan).
template <int CH, bool WALK>
__global__ __launch_bounds__(kMtuBlock, 8) void mtu_emit_kernel(MtuLaunch L) {   // 8 waves per SIMD: every chunk resident
    constexpr int kMtuPer = CH / kMtuBlock;
    __shared__ MtuEmitSmem<CH> sm;
    MtuChunk ck;
    const uint32_t gs = mtu_chunk_slot(L, blockIdx.x);
    if (gs == kMtuNone) return;
    const uint32_t bi = mtu_batch_of(L, gs, [](const MtuBatchArg &a) { return a.chunk0; });
    const MtuParams p = mtu_view(L, bi);
    const uint32_t c = gs - L.b[bi].chunk0;
    if (!mtu_chunk_of(p, c, ck)) return;
    mtu_stamp(L, gs, 5);
    const int tid = threadIdx.x;
    const uint32_t *gp0 = p.gp0 + (size_t)c * (kMtuP0 + 1);
    const uint16_t *gpl = p.plen + (size_t)c * kMtuChunk;
    // next(i) - i as mtu_table stored it (16 bytes per thread), issued before the walk
    constexpr int kNxPer = (CH / 16 + kMtuBlock - 1) / kMtuBlock;
    uint4 nxv[kNxPer];
#pragma unroll
    for (int k = 0; k < kNxPer; ++k) {
        const uint32_t v = (uint32_t)tid + (uint32_t)k * kMtuBlock;
        nxv[k] = v * 16 < ck.cnt ? reinterpret_cast<const uint4 *>(p.nx + (size_t)c * kMtuChunk)[v] : make_uint4(0, 0, 0, 0);
    }
    uint32_t x, j, open, k0;
    if constexpr (WALK) {
        if (tid < 64) {
            const uint32_t s = (uint32_t)tid;
            uint32_t tot = 0, xs = 0, os = kMtuNone, cs = 0;
            uint64_t es = 0;
            if (s <= ck.shard) {
                xs = p.fill_in ? min((uint32_t)p.fill_in[s], (uint32_t)kMtuCap) : 0u;
                const uint32_t c0 = p.chunk_first[s];
                const uint32_t c1 = s == ck.shard ? c + 1 : min(p.chunk_first[s + 1], p.max_chunks);
                for (uint32_t cc = c0; cc < c1; ++cc) {
                    const uint64_t e = p.table[(size_t)cc * kMtuX + xs];
                    if (cc == c) {   // this chunk's own entry, at its incoming fill
                        es = e;
                        break;
                    }
                    const uint32_t cl = (uint32_t)(e >> 32) & 0xFFFFu;
                    if (cl) {
                        cs += cl;
                        os = p.key_start[s] + (cc - c0) * p.chunk_lines + (uint32_t)((e >> 16) & 0xFFFFu);
                    }
                    xs = (uint32_t)(e & 0xFFFFu);
                }
                if (s < ck.shard) tot = cs + (c1 > c0 ? 1u : 0u);
            }
            const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_add32(tot), 63);
            if (s == ck.shard) {
                sm.bc[0] = xs;
                sm.bc[1] = (uint32_t)(es >> 48);
                sm.bc[2] = os;
                sm.bc[3] = base + cs;
                const uint32_t cl = (uint32_t)(es >> 32) & 0xFFFFu;
                if (ck.last) p.fill_out[s] = mtu_dropped(p, s) ? 0 : (uint16_t)(es & 0xFFFFu);
                if (c + 1 == min(p.chunk_first[p.nds], p.max_chunks)) p.counts[0] = base + cs + cl + 1u;
            }
        }
        __syncthreads();
        x = sm.bc[0];
        j = sm.bc[1];
        open = sm.bc[2];
        k0 = sm.bc[3];
    } else {
        const uint32_t xe = p.chunk_entry[c];
        x = xe & 0xFFFFu;
        j = xe >> 16;
        open = p.chunk_open[c];
        k0 = p.chunk_pk[c];
    }
    const uint32_t total = gp0[kMtuP0];
    const uint32_t carry = open == kMtuNone ? x : 0u;        // pending bytes from before the batch
    const uint32_t start = open == kMtuNone ? p.key_start[ck.shard] : open;
    if (x + total <= (uint32_t)kMtuCap) {   // no line of the chunk closes a packet: the incoming one stays open
        if (ck.last && tid == 0)
            mtu_put(p, k0, start, ck.pos0 + ck.cnt - start, ck.shard, x - carry + total, carry, 1u);
        return;
    }
    if (tid == 0)   // the incoming packet closes before line j
        mtu_put(p, k0, start, ck.pos0 + j - start, ck.shard, x - carry + (j ? gp0[j - 1] : 0u), carry, 0u);
    // next(i) - i into LDS, then J: next(i), doubled four times (exact: all reads of a round before
    // its writes)
#pragma unroll
    for (int k = 0; k < kNxPer; ++k) {
        const uint32_t v = (uint32_t)tid + (uint32_t)k * kMtuBlock;
        if (v * 16 < (uint32_t)CH) reinterpret_cast<uint4 *>(sm.nx)[v] = nxv[k];
    }
    __syncthreads();
    mtu_stamp(L, gs, 6);
    uint16_t jv[kMtuPer];
#pragma unroll
    for (int k = 0; k < kMtuPer; ++k) {
        const uint32_t i = (uint32_t)tid + (uint32_t)k * kMtuBlock;
        const uint32_t d = sm.nx[i];
        jv[k] = (i < ck.cnt && d) ? (uint16_t)(i + d) : kMtuEnd;
        sm.J[i] = jv[k];
    }
    __syncthreads();
    for (int r = 0; !(SR_MTU_SKIP & 4) && (1 << r) < kMtuHop; ++r) {
#pragma unroll
        for (int k = 0; k < kMtuPer; ++k) {
            const uint16_t t = sm.J[jv[k] == kMtuEnd ? 0u : jv[k]];
            jv[k] = jv[k] == kMtuEnd ? kMtuEnd : t;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kMtuPer; ++k) sm.J[(uint32_t)tid + (uint32_t)k * kMtuBlock] = jv[k];
        __syncthreads();
    }
    if (tid == 0) {   // anchors every kMtuHop packet starts from j
        uint32_t n = 0;
        for (uint32_t a = j; !(SR_MTU_SKIP & 4);) {
            sm.anchor[n++] = (uint16_t)a;
            const uint32_t nxt = sm.J[a];
            if (nxt == kMtuEnd) break;
            a = nxt;
        }
        sm.nanchor = n;
    }
    __syncthreads();
    const uint32_t na = sm.nanchor;
    for (uint32_t q = (uint32_t)tid; q < na; q += kMtuBlock) {
        // the anchor's packets: starts and ends from next() in LDS, then every packet's length
        // loaded before the first descriptor store (a store waits for the loads issued before it)
        // (consecutive packets: each starts where the one before it ends)
        uint32_t bs[kMtuHop];
        int ns = 0;
        bool is_open = false;
        const uint32_t a0 = sm.anchor[q];
        uint32_t a = a0;
#pragma unroll
        for (int step = 0; step < kMtuHop; ++step) {
            bs[step] = 1u;
            if (ns == step && !is_open) {
                const uint32_t d = sm.nx[a];
                is_open = d == 0;            // the last packet start: the packet stays pending
                bs[step] = is_open ? ck.cnt : a + d;
                ns = step + ((!is_open || ck.last) ? 1 : 0);   // an open packet not in the last chunk continues
                a += d;
            }
        }
        uint32_t pl[kMtuHop];
#pragma unroll
        for (int step = 0; step < kMtuHop; ++step)   // unconditional (clamped) loads, all in flight together
            pl[step] = gpl[min(step ? bs[step - 1] : a0, ck.cnt - 1)];
        uint32_t s0 = a0;
#pragma unroll
        for (int step = 0; step < kMtuHop; ++step) {
            if (step < ns)
                mtu_put(p, k0 + 1 + q * kMtuHop + (uint32_t)step, ck.pos0 + s0, bs[step] - s0, ck.shard, pl[step], 0u,
                        (is_open && ck.last && step == ns - 1) ? 1u : 0u);   // the chain's open packet
            s0 = bs[step];
        }
    }
    mtu_stamp(L, gs, 7);
}

}  // namespace srk

namespace srk {

// The outputs of one routed + packed batch copied into page-locked host memory (device-mapped) by
// one kernel on the batch's stream, so that a host waits once per batch (sr_route_pack_result):
// the copy sizes are the device's own counts, which no host round trip has to fetch first.
struct PackOut {
    const sr_record *sorted;
    const sr_packet *packets;
    const uint16_t *fill;        // pending bytes after the batch (n_downstreams)
    const uint64_t *probed;      // null: no dead shard in the snapshot (zeros written)
    const uint64_t *counts;      // {descriptors, valid lines, lines}
    uint64_t rec_cap, pk_cap;
    uint32_t nds, nwords;
    sr_record *h_sorted;         // device-mapped host pointers
    sr_packet *h_packets;
    uint16_t *h_fill;
    uint64_t *h_probed;
    uint64_t *h_counts;
    const sr_record *recs;       // sr_set_trace (else null): the records in input order and the hashes
    const uint64_t *hashes;
    sr_record *h_recs;
    uint64_t *h_hashes;
};

__global__ __launch_bounds__(256) void pack_out_kernel(PackOut o) {
    const uint64_t np = min(o.counts[0], o.pk_cap), nr = min(o.counts[2], o.rec_cap);
    const uint64_t tid = (uint64_t)blockIdx.x * 256u + threadIdx.x, stride = (uint64_t)gridDim.x * 256u;
    // records as 16-byte pairs (the tail record alone), packets 16 bytes each
    const uint4 *rs = reinterpret_cast<const uint4 *>(o.sorted);
    uint4 *rd = reinterpret_cast<uint4 *>(o.h_sorted);
    for (uint64_t i = tid; i < nr / 2; i += stride) rd[i] = rs[i];
    if ((nr & 1) && tid == 0) o.h_sorted[nr - 1] = o.sorted[nr - 1];
    const uint4 *ps = reinterpret_cast<const uint4 *>(o.packets);
    uint4 *pd = reinterpret_cast<uint4 *>(o.h_packets);
    for (uint64_t i = tid; i < np; i += stride) pd[i] = ps[i];
    for (uint64_t i = tid; i < o.nds; i += stride) o.h_fill[i] = o.fill[i];
    for (uint64_t i = tid; i < o.nwords; i += stride) o.h_probed[i] = o.probed ? o.probed[i] : 0ull;
    if (tid < 3) o.h_counts[tid] = o.counts[tid];
    if (o.recs) {   // TRACE: input-order records and per-line hashes (sr_route_pack_trace)
        for (uint64_t i = tid; i < nr; i += stride) {
            o.h_recs[i] = o.recs[i];
            o.h_hashes[i] = o.hashes[i];
        }
    }
}

}  // namespace srk
