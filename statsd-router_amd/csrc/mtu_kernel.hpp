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
//   mtu_count   per 512-record tile, a histogram of keys (shard, or N = unrouted) in LDS;
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
//   mtu_emit    per chunk: walks its packet chain from its incoming fill and writes descriptors.
// Integer/byte work, latency-light: no MFMA.
#pragma once

#include "route_kernel.hpp"

namespace srk {

constexpr int kMtuTile = 512;                    // records per sort tile (one wave)
constexpr int kMtuChunk = 4096;                  // sorted lines per packing chunk
constexpr int kMtuBlock = 256;                   // threads of the chunk kernels
constexpr int kMtuPer = kMtuChunk / kMtuBlock;   // lines per thread in a chunk
constexpr uint32_t kMtuMaxShards = 4096;
constexpr int kMtuCap = (int)SR_DOWNSTREAM_BUF_SIZE;   // 1450: sr-types.h:30
constexpr int kMtuWindow = kMtuCap / (int)SR_MIN_LINE_LENGTH + 1;   // a packet holds < 242 lines
constexpr int kMtuX = kMtuCap + 1;               // incoming fills 0..1450
constexpr uint32_t kMtuNone = 0xFFFFFFFFu;
constexpr uint16_t kMtuEnd = 0xFFFFu;

constexpr int kMtuMaxBatches = 32;

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
};

struct MtuLaunch {
    uint32_t nds, nb, tiles, chunks;   // shards; batches; record tiles and chunks of all batches
    uint32_t *tile_counts;             // batch b at (nds + 1) * tile0: [(nds + 1) * ntiles], key-major
    uint32_t *keys;                    // [nb][2 * nds + 4]: key starts (nds + 2) | chunk firsts (nds + 1)
    uint32_t *chunk_shard;             // [chunks]
    uint32_t *chunk_entry;             // [chunks] incoming fill
    uint32_t *chunk_open;              // [chunks] sorted position where the incoming packet began
    uint32_t *chunk_pk;                // [chunks] first descriptor the chunk writes
    uint32_t *closed;                  // [nb][nds] packets closed per shard
    uint64_t *table;                   // [chunks][kMtuX]
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
    const uint16_t *fill_in;
    const uint64_t *probed_dead;
    uint32_t *tile_counts;    // [(nds + 1) * ntiles], key-major; scanned in place
    uint32_t *key_start;      // [nds + 2]: first sorted position of each key, [nds + 1] = lines
    uint32_t *chunk_first;    // [nds + 1]: first chunk of each shard, [nds] = chunks
    uint32_t *chunk_shard;
    uint64_t *table;
    uint32_t *chunk_entry;
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
    p.fill_in = a.fill_in;
    p.probed_dead = a.probed_dead;
    p.tile_counts = L.tile_counts + (size_t)(L.nds + 1) * a.tile0;
    p.key_start = L.keys + (size_t)bi * (2 * L.nds + 4);
    p.chunk_first = p.key_start + L.nds + 2;
    p.chunk_shard = L.chunk_shard + a.chunk0;
    p.table = L.table + (size_t)a.chunk0 * kMtuX;
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

// the batch owning global index g of a per-batch sequence starting at field `first` (nb <= 32)
template <class F>
__device__ __forceinline__ uint32_t mtu_batch_of(const MtuLaunch &L, uint32_t g, F first) {
    uint32_t k = 0;
    for (uint32_t j = 1; j < L.nb; ++j) k += g >= first(L.b[j]) ? 1u : 0u;
    return k;
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

// ---- sort: histogram, scan, stable scatter ----------------------------------------------------
__global__ __launch_bounds__(64) void mtu_count_kernel(MtuLaunch L) {
    __shared__ uint32_t hist[kMtuMaxShards + 1];
    const uint32_t bi = mtu_batch_of(L, blockIdx.x, [](const MtuBatchArg &a) { return a.tile0; });
    const MtuParams p = mtu_view(L, bi);
    const int lane = threadIdx.x;
    const uint32_t nk = p.nds + 1, t = blockIdx.x - L.b[bi].tile0;
    for (uint32_t k = lane; k < nk; k += 64) hist[k] = 0;
    __syncthreads();
    const uint32_t n = mtu_lines(p), r0 = t * kMtuTile;
    for (uint32_t i = r0 + lane; i < r0 + kMtuTile && i < n; i += 64) atomicAdd(&hist[mtu_key(p.recs[i], p.nds)], 1u);
    __syncthreads();
    for (uint32_t k = lane; k < nk; k += 64) p.tile_counts[(size_t)k * p.ntiles + t] = hist[k];
}

// One workgroup of 1024 threads: exclusive scan of the key-major table (position of (key, tile)
// = lines of smaller keys + lines of the same key in earlier tiles), key starts, packing chunks.
__global__ __launch_bounds__(1024) void mtu_scan_kernel(MtuLaunch L) {
    const MtuParams p = mtu_view(L, blockIdx.x);
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t nk = p.nds + 1, ntiles = p.ntiles;
    const size_t total = (size_t)nk * ntiles;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    for (size_t b0 = 0; b0 < total; b0 += 1024 * 4) {
        uint32_t v[4], s = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const size_t i = b0 + (size_t)tid * 4 + k;
            v[k] = i < total ? p.tile_counts[i] : 0u;
            s += v[k];
        }
        const uint32_t incl = wave_incl_add32(s);
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t before = carry_s;
        for (int w = 0; w < wave; ++w) before += wsum[w];
        uint32_t run = before + incl - s;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const size_t i = b0 + (size_t)tid * 4 + k;
            if (i < total) p.tile_counts[i] = run;
            run += v[k];
        }
        __syncthreads();
        if (tid == 1023) carry_s = run;
        __syncthreads();
    }
    const uint32_t n = mtu_lines(p);
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
        loc += (c + kMtuChunk - 1) / kMtuChunk;
    }
    const uint32_t incl = wave_incl_add32(loc);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - loc;
    for (int w = 0; w < wave; ++w) run += wsum[w];
    for (uint32_t s = tid * per; s < (tid + 1) * per && s < p.nds; ++s) {
        p.chunk_first[s] = run;
        const uint32_t c = p.key_start[s + 1] - p.key_start[s];
        const uint32_t nc = (c + kMtuChunk - 1) / kMtuChunk;
        for (uint32_t j = 0; j < nc; ++j)
            if (run + j < p.max_chunks) p.chunk_shard[run + j] = s;
        run += nc;
    }
    if (tid == 1023) {
        p.chunk_first[p.nds] = run;
        p.counts[1] = p.key_start[p.nds];
    }
}

__global__ __launch_bounds__(64) void mtu_scatter_kernel(MtuLaunch L) {
    __shared__ uint32_t pos[kMtuMaxShards + 1];
    volatile uint32_t *vpos = pos;
    const uint32_t bi = mtu_batch_of(L, blockIdx.x, [](const MtuBatchArg &a) { return a.tile0; });
    const MtuParams p = mtu_view(L, bi);
    const int lane = threadIdx.x;
    const uint32_t nk = p.nds + 1, t = blockIdx.x - L.b[bi].tile0;
    for (uint32_t k = lane; k < nk; k += 64) pos[k] = p.tile_counts[(size_t)k * p.ntiles + t];
    __syncthreads();
    const uint32_t n = mtu_lines(p), r0 = t * kMtuTile;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t c0 = r0; c0 < r0 + kMtuTile && c0 < n; c0 += 64) {
        const uint32_t i = c0 + lane;
        bool pend = i < n;
        sr_record r{0, 0, 0};
        uint32_t key = 0;
        if (pend) {
            r = p.recs[i];
            key = mtu_key(r, p.nds);
        }
        // stable in-wave ranks: one round per distinct key of the 64 records
        for (uint64_t pm = __ballot(pend); pm; pm = __ballot(pend)) {
            const int leader = __builtin_ctzll(pm);
            const uint32_t k0 = (uint32_t)__builtin_amdgcn_readlane((int)key, leader);
            const bool mine = pend && key == k0;
            const uint64_t m = __ballot(mine);
            const uint32_t base = vpos[k0];
            if (mine) {
                p.sorted[base + (uint32_t)__popcll(m & lt)] = r;
                pend = false;
            }
            if (lane == leader) vpos[k0] = base + (uint32_t)__popcll(m);
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// ---- packing: per-chunk next-fit tables -------------------------------------------------------
struct MtuChunkSmem {
    uint32_t P[kMtuChunk];      // inclusive prefix of the chunk's line lengths
    uint16_t nx[kMtuChunk];     // chunk-local start of the packet after one starting here, kMtuEnd
    uint16_t lst[kMtuChunk];    // last packet start reached from here
    uint16_t dep[kMtuChunk];    // packets closed on the way
    uint32_t wsum[kMtuBlock / 64];
    uint16_t walk[kMtuChunk + 1];
};

struct MtuChunk {
    uint32_t shard, pos0, cnt;
    bool last;
};

__device__ __forceinline__ bool mtu_chunk_of(const MtuParams &p, uint32_t c, MtuChunk &ck) {
    if (c >= min(p.chunk_first[p.nds], p.max_chunks)) return false;
    ck.shard = p.chunk_shard[c];
    const uint32_t s0 = p.key_start[ck.shard], s1 = p.key_start[ck.shard + 1];
    ck.pos0 = s0 + (c - p.chunk_first[ck.shard]) * kMtuChunk;
    ck.cnt = min((uint32_t)kMtuChunk, s1 - ck.pos0);
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

// LDS prefix sums of the chunk's lengths and next(i) for every line
__device__ void mtu_chunk_build(const MtuParams &p, const MtuChunk &ck, MtuChunkSmem &sm, bool doubling) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t v[kMtuPer], s = 0;
#pragma unroll
    for (int k = 0; k < kMtuPer; ++k) {
        const uint32_t i = (uint32_t)tid * kMtuPer + k;
        v[k] = i < ck.cnt ? p.sorted[ck.pos0 + i].length : 0u;
        s += v[k];
    }
    const uint32_t incl = wave_incl_add32(s);
    if (lane == 63) sm.wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - s;
    for (int w = 0; w < wave; ++w) run += sm.wsum[w];
#pragma unroll
    for (int k = 0; k < kMtuPer; ++k) {
        run += v[k];
        sm.P[tid * kMtuPer + k] = run;
    }
    __syncthreads();
    for (uint32_t i = tid; i < ck.cnt; i += kMtuBlock) {
        const uint32_t pm = i ? sm.P[i - 1] : 0u;
        const uint32_t hi = min(ck.cnt, i + (uint32_t)kMtuWindow);
        uint16_t nxt = kMtuEnd;
        if (sm.P[hi - 1] - pm > (uint32_t)kMtuCap) nxt = (uint16_t)mtu_first_over(sm.P, i + 1, hi - 1, pm + kMtuCap);
        sm.nx[i] = nxt;
        sm.lst[i] = nxt == kMtuEnd ? (uint16_t)i : nxt;
        sm.dep[i] = nxt == kMtuEnd ? 0 : 1;
    }
    __syncthreads();
    if (!doubling) return;
    // pointer doubling: lst -> the last packet start of the chain, dep -> packets closed on it
    for (uint32_t span = 1; span < ck.cnt; span <<= 1) {
        uint16_t nl[kMtuPer], nd[kMtuPer];
#pragma unroll
        for (int k = 0; k < kMtuPer; ++k) {
            const uint32_t i = (uint32_t)tid + (uint32_t)k * kMtuBlock;
            if (i < ck.cnt) {
                const uint16_t l = sm.lst[i];
                nl[k] = sm.lst[l];
                nd[k] = (uint16_t)(sm.dep[i] + sm.dep[l]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kMtuPer; ++k) {
            const uint32_t i = (uint32_t)tid + (uint32_t)k * kMtuBlock;
            if (i < ck.cnt) {
                sm.lst[i] = nl[k];
                sm.dep[i] = nd[k];
            }
        }
        __syncthreads();
    }
}

// table[c][x] = (packets closed << 32) | (last packet start << 16, 0xFFFF = none) | fill after
__global__ __launch_bounds__(kMtuBlock) void mtu_table_kernel(MtuLaunch L) {
    __shared__ MtuChunkSmem sm;
    MtuChunk ck;
    const uint32_t bi = mtu_batch_of(L, blockIdx.x, [](const MtuBatchArg &a) { return a.chunk0; });
    const MtuParams p = mtu_view(L, bi);
    const uint32_t c = blockIdx.x - L.b[bi].chunk0;
    if (!mtu_chunk_of(p, c, ck)) return;
    mtu_chunk_build(p, ck, sm, true);
    const uint32_t total = sm.P[ck.cnt - 1];
    const uint32_t hi = min(ck.cnt, (uint32_t)kMtuWindow);
    uint64_t *row = p.table + (size_t)c * kMtuX;
    for (uint32_t x = threadIdx.x; x < (uint32_t)kMtuX; x += kMtuBlock) {
        uint64_t e;
        if (x + total <= (uint32_t)kMtuCap) {
            e = (0xFFFFull << 16) | (x + total);
        } else {
            const uint32_t j = mtu_first_over(sm.P, 0, hi - 1, (uint32_t)kMtuCap - x);
            const uint32_t l = sm.lst[j];
            e = ((uint64_t)(1u + sm.dep[j]) << 32) | ((uint64_t)l << 16) | (total - (l ? sm.P[l - 1] : 0u));
        }
        row[x] = e;
    }
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
            p.chunk_entry[c] = x;
            p.chunk_open[c] = open;
            p.chunk_pk[c] = closed;   // shard-relative until the scan below
            const uint64_t e = p.table[(size_t)c * kMtuX + x];
            const uint32_t cl = (uint32_t)(e >> 32);
            if (cl) {
                closed += cl;
                open = p.key_start[s] + (c - c0) * kMtuChunk + (uint32_t)((e >> 16) & 0xFFFFu);
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

__global__ __launch_bounds__(kMtuBlock) void mtu_emit_kernel(MtuLaunch L) {
    __shared__ MtuChunkSmem sm;
    __shared__ uint32_t nwalk, jfirst;
    MtuChunk ck;
    const uint32_t bi = mtu_batch_of(L, blockIdx.x, [](const MtuBatchArg &a) { return a.chunk0; });
    const MtuParams p = mtu_view(L, bi);
    const uint32_t c = blockIdx.x - L.b[bi].chunk0;
    if (!mtu_chunk_of(p, c, ck)) return;
    mtu_chunk_build(p, ck, sm, false);
    const int tid = threadIdx.x;
    const uint32_t x = p.chunk_entry[c], open = p.chunk_open[c], k0 = p.chunk_pk[c];
    const uint32_t total = sm.P[ck.cnt - 1];
    const uint32_t carry = open == kMtuNone ? x : 0u;        // pending bytes from before the batch
    const uint32_t start = open == kMtuNone ? p.key_start[ck.shard] : open;
    if (tid == 0) {
        // the chain of packet starts: the first line that does not fit the incoming packet, then next()
        uint32_t nw = 0;
        uint32_t j = kMtuEnd;
        if (x + total > (uint32_t)kMtuCap) {
            j = mtu_first_over(sm.P, 0, min(ck.cnt, (uint32_t)kMtuWindow) - 1, (uint32_t)kMtuCap - x);
            for (uint32_t cur = j;; cur = sm.nx[cur]) {
                sm.walk[nw++] = (uint16_t)cur;
                if (sm.nx[cur] == kMtuEnd) break;
            }
        }
        nwalk = nw;
        jfirst = j;
    }
    __syncthreads();
    const uint32_t nw = nwalk;
    if (nw == 0) {   // no line of the chunk closes a packet: the incoming one stays open
        if (ck.last && tid == 0)
            mtu_put(p, k0, start, ck.pos0 + ck.cnt - start, ck.shard, x - carry + total, carry, 1u);
        return;
    }
    if (tid == 0) {   // the incoming packet closes before line jfirst
        const uint32_t j = jfirst;
        mtu_put(p, k0, start, ck.pos0 + j - start, ck.shard, x - carry + (j ? sm.P[j - 1] : 0u), carry, 0u);
    }
    for (uint32_t w = tid; w < nw; w += kMtuBlock) {
        const uint32_t a = sm.walk[w];
        const bool is_open = w + 1 == nw;
        if (is_open && !ck.last) continue;   // continues into the next chunk
        const uint32_t b = is_open ? ck.cnt : sm.walk[w + 1];
        mtu_put(p, k0 + 1 + w, ck.pos0 + a, b - a, ck.shard, sm.P[b - 1] - (a ? sm.P[a - 1] : 0u), 0u,
                is_open ? 1u : 0u);
    }
}

}  // namespace srk
