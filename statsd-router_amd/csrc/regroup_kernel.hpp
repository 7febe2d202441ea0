// regroup_kernel.hpp — pack routed lines by owner GPU before the all-to-all regroup
// (DESIGN.md §7).
//
// On a node of G GPUs every GPU routes its own datagram batches; shard s is then OWNED by GPU
// s mod G, which sends it on to downstream s (the reference's push_to_downstream,
// sr-main.c:73-83, runs on the owner). Before the exchange each GPU packs its valid lines by owner:
//   out bytes : for owner 0, 1, ..., G-1 in turn, its lines in input order, each line starting at
//               a 4-byte aligned position (zero fill after the line), so the copy is dword-wide;
//   out recs  : one sr_record per packed line, same order; offset = position of the line
//               relative to the start of its owner's chunk, length and route unchanged;
//   counts    : per owner {lines, bytes} (u64 pairs) = the all-to-all split sizes.
// Lines routed to no shard (invalid length / format, all dead) are not packed: the GPU that
// received them reports them (the WARN lines of sr-main.c:115,142,184 stay with the receiver).
//
// Three launches over tiles of 256 x CH records (the tiles of all packed batches in sequence):
// per-tile counts, one workgroup scanning them, then the stable scatter (in-tile ranks recomputed
// with ballots and DPP scans).
#pragma once

#include "route_kernel.hpp"

namespace srk {

constexpr int kPackBlock = 256;
// 256-record chunks per tile, chosen per pack (pack_chunks_for in sr_route.hip): two for short lines,
// one when the lines are long, so that a launch of long lines has enough workgroups to balance the
// scatter's copy (C5 one workgroup generation of 512-record tiles: 256-record tiles +3-4 %; C2 -2 %)
constexpr int kPackMaxChunks = 2;
constexpr int kMaxOwners = 64;

// One routed batch of a pack (up to kPackMaxBatches per pack: a route launch's batches are packed
// and exchanged together, owner chunks holding batch 0's lines, then batch 1's, ...).
constexpr int kPackMaxBatches = 32;
#ifndef SR_PACK_COPY_BATCH
#define SR_PACK_COPY_BATCH 4   // the owner scatter's copy passes whose loads are issued together
#endif
struct PackBatch {
    const uint8_t *bytes;
    const sr_record *recs;
    const uint64_t *n_records;   // device line count written by the route kernel
    uint32_t nbytes;
    uint32_t max_records;
    uint32_t tile0;              // first tile of the batch in the pack's tile sequence
    uint32_t pad;
};

struct PackParams {
    uint32_t nb;
    uint32_t n_owners;
    uint32_t ntiles;             // tiles of all batches
    uint32_t pad;
    uint2 *tile_counts;          // [ntiles][n_owners] {lines, bytes} within the tile
    uint2 *tile_base;            // [ntiles][n_owners] exclusive prefix over tiles within the owner
    uint64_t *owner_start;       // [n_owners][2] {first line, first byte} of the owner's chunk
    uint64_t *owner_counts;      // [n_owners][2] {lines, bytes} (output)
    uint8_t *out_bytes;
    uint64_t out_cap;
    sr_record *out_recs;
    // sr_pack_owner_scatter: owner `own`'s chunk goes to own_bytes / own_recs (its place in the
    // exchange's receive buffers; capacity: its own byte count) instead of out_*; -1: none
    int32_t own;
    uint32_t pad2;
    uint8_t *own_bytes;
    sr_record *own_recs;
    PackBatch b[kPackMaxBatches];
};

// the batch of pack tile `tile` and the tile's first record in it (nb <= 32: a scan over SGPRs)
// batch of a (wave-uniform) tile: lane j compares with batch j's first tile, one ballot (a loop over the
// batches waited on one scalar load per batch)
template <int CH>
__device__ __forceinline__ const PackBatch &pack_batch_of(const PackParams &p, uint32_t tile, uint32_t &r0) {
    static_assert(kPackMaxBatches <= 64, "one lane per batch");
    const uint32_t lane = threadIdx.x & 63u;
    const bool past = lane >= 1 && lane < p.nb && tile >= p.b[lane < kPackMaxBatches ? lane : 0].tile0;
    const uint32_t k = (uint32_t)__popcll(__ballot(past));
    r0 = (tile - p.b[k].tile0) * (uint32_t)(kPackBlock * CH);
    return p.b[k];
}

__device__ __forceinline__ uint32_t pack_len4(uint32_t len) { return (len + 3u) & ~3u; }

// owner of record r, or -1 when the line goes to no shard
__device__ __forceinline__ int pack_owner(const sr_record &r, uint32_t n_owners) {
    return r.route < SR_ROUTE_INVALID_LENGTH ? (int)(r.route % n_owners) : -1;
}

// kCountTiles tiles per workgroup. Every load is issued before any is waited on: the {length, route}
// words (the records' second halves) by index clamped to the batch's capacity, and the batches' line
// counts beside them; records past the line count are masked afterwards. Gating the loads on the line
// count serialised two memory round trips per tile.
#ifndef SR_COUNT_TILES
#define SR_COUNT_TILES 1
#endif
constexpr int kCountTiles = SR_COUNT_TILES;
static_assert(offsetof(sr_record, length) == 4 && offsetof(sr_record, route) == 6, "{length, route} word");
template <int CH>
__global__ __launch_bounds__(kPackBlock) void pack_count_kernel(PackParams p) {
    __shared__ uint32_t s_lines[kCountTiles][kMaxOwners], s_bytes[kCountTiles][kMaxOwners];
    const int tid = threadIdx.x, lane = tid & 63;
    const uint32_t G = p.n_owners;
    const uint32_t t0 = blockIdx.x * kCountTiles;
    for (uint32_t o = tid; o < kCountTiles * G; o += kPackBlock) s_lines[o / G][o % G] = s_bytes[o / G][o % G] = 0;
    uint32_t lr[kCountTiles][CH];
    uint64_t nr[kCountTiles];
    uint32_t r0s[kCountTiles], cap[kCountTiles];
#pragma unroll
    for (int tt = 0; tt < kCountTiles; ++tt) {
        const uint32_t t = min(t0 + tt, p.ntiles - 1);
        uint32_t r0;
        const PackBatch &bt = pack_batch_of<CH>(p, t, r0);
        r0s[tt] = r0;
        cap[tt] = bt.max_records;
        nr[tt] = *bt.n_records;
        const uint32_t *w = reinterpret_cast<const uint32_t *>(bt.recs) + 1;
#pragma unroll
        for (int c = 0; c < CH; ++c)
            lr[tt][c] = w[2 * (size_t)min(r0 + c * kPackBlock + tid, bt.max_records - 1)];
    }
    __syncthreads();
#pragma unroll
    for (int tt = 0; tt < kCountTiles; ++tt) {
        if (t0 + tt >= p.ntiles) break;
        const uint32_t n = (uint32_t)min(nr[tt], (uint64_t)cap[tt]);
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const uint32_t i = r0s[tt] + c * kPackBlock + tid;
            int ow = -1;
            uint32_t len4 = 0;
            if (i < n) {
                sr_record r;
                r.length = (uint16_t)(lr[tt][c] & 0xFFFFu);
                r.route = (uint16_t)(lr[tt][c] >> 16);
                ow = pack_owner(r, G);
                len4 = pack_len4(r.length);
            }
            for (uint32_t o = 0; o < G; ++o) {
                const uint64_t m = __ballot(ow == (int)o);
                if (!m) continue;
                const uint32_t b = wave_incl_add32(ow == (int)o ? len4 : 0u);
                if (lane == 63) {
                    atomicAdd(&s_lines[tt][o], (uint32_t)__popcll(m));
                    atomicAdd(&s_bytes[tt][o], b);
                }
            }
        }
    }
    __syncthreads();
    for (uint32_t o = tid; o < kCountTiles * G; o += kPackBlock) {
        const uint32_t tt = o / G, ow = o % G;
        if (t0 + tt < p.ntiles) p.tile_counts[(size_t)(t0 + tt) * G + ow] = make_uint2(s_lines[tt][ow], s_bytes[tt][ow]);
    }
}

// one workgroup: per owner, exclusive scan of the tile counts; owner totals and chunk starts
__global__ __launch_bounds__(1024) void pack_scan_kernel(PackParams p) {
    __shared__ uint64_t s_tot[kMaxOwners][2];
    __shared__ uint32_t s_carry[2];
    __shared__ uint32_t s_wave[16][2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t G = p.n_owners;
    // kScanPer rows of 64 consecutive tiles per wave and round (a C2 launch's 16,384 tiles in one round):
    // coalesced loads and stores, the row scans in registers. Sixteen consecutive tiles per thread made
    // every load touch 64 lines on the one CU (18 µs per C2 launch)
    constexpr uint32_t kScanPer = 16;
    for (uint32_t o = 0; o < G; ++o) {
        if (tid == 0) s_carry[0] = s_carry[1] = 0;
        __syncthreads();
        for (uint32_t t0 = 0; t0 < p.ntiles; t0 += 1024 * kScanPer) {
            const uint32_t wb = t0 + (uint32_t)wave * 64 * kScanPer + lane;
            uint2 v[kScanPer];
#pragma unroll
            for (uint32_t k = 0; k < kScanPer; ++k) {
                const uint32_t t = wb + k * 64;
                v[k] = t < p.ntiles ? p.tile_counts[(size_t)t * G + o] : make_uint2(0, 0);
            }
            uint32_t rl = 0, rb = 0;   // the wave's running totals (uniform)
#pragma unroll
            for (uint32_t k = 0; k < kScanPer; ++k) {
                const uint32_t il = wave_incl_add32(v[k].x), ib = wave_incl_add32(v[k].y);
                v[k] = make_uint2(rl + il - v[k].x, rb + ib - v[k].y);   // exclusive within the wave's rows
                rl += __builtin_amdgcn_readlane(il, 63);
                rb += __builtin_amdgcn_readlane(ib, 63);
            }
            if (lane == 0) {
                s_wave[wave][0] = rl;
                s_wave[wave][1] = rb;
            }
            __syncthreads();
            uint32_t pl = s_carry[0], pb = s_carry[1];
            for (int w = 0; w < wave; ++w) {
                pl += s_wave[w][0];
                pb += s_wave[w][1];
            }
#pragma unroll
            for (uint32_t k = 0; k < kScanPer; ++k) {
                const uint32_t t = wb + k * 64;
                if (t < p.ntiles) p.tile_base[(size_t)t * G + o] = make_uint2(pl + v[k].x, pb + v[k].y);
            }
            __syncthreads();
            if (tid == 1023) {
                s_carry[0] = pl + rl;
                s_carry[1] = pb + rb;
            }
            __syncthreads();
        }
        if (tid == 0) {
            s_tot[o][0] = s_carry[0];
            s_tot[o][1] = s_carry[1];
        }
        __syncthreads();
    }
    if (tid == 0) {
        uint64_t line = 0, byte = 0;
        for (uint32_t o = 0; o < G; ++o) {
            p.owner_start[2 * o] = line;
            p.owner_start[2 * o + 1] = byte;
            p.owner_counts[2 * o] = s_tot[o][0];
            p.owner_counts[2 * o + 1] = s_tot[o][1];
            line += s_tot[o][0];
            byte += s_tot[o][1];
        }
    }
}

__device__ __forceinline__ void pack_wave_sync() {   // LDS hand-off between the lanes of one wave
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// The scatter's copy works in windows of kPackWin 16-byte pieces per wave (16 per lane).
constexpr uint32_t kPackWin = 1024;

template <int CH>
__global__ __launch_bounds__(kPackBlock) void pack_scatter_kernel(PackParams p) {
    __shared__ uint32_t s_run_l[kMaxOwners], s_run_b[kMaxOwners];   // running in-tile position per owner
    __shared__ uint32_t s_wl[4][kMaxOwners], s_wb[4][kMaxOwners];   // per-wave chunk totals
    // per wave, its owned lines in order (compacted): {source offset, destination, length | own << 31,
    // first piece}; and per window a bitmap of the pieces where a line starts, with per-dword prefix counts
    __shared__ uint4 s_info[4][64];
    __shared__ uint32_t s_bm[4][kPackWin / 32], s_bp[4][kPackWin / 32];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t r0;
    const PackBatch &bt = pack_batch_of<CH>(p, blockIdx.x, r0);
    const uint32_t n = (uint32_t)min(*bt.n_records, (uint64_t)bt.max_records);
    const uint32_t G = p.n_owners;
    for (uint32_t o = tid; o < G; o += kPackBlock) s_run_l[o] = s_run_b[o] = 0;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)bt.bytes, (short)0, (int)bt.nbytes, 0x00020000);
    const uint64_t lt = (1ull << lane) - 1ull;
    __syncthreads();
    for (int c = 0; c < CH; ++c) {
        const uint32_t i = r0 + c * kPackBlock + tid;
        int ow = -1;
        sr_record r{0, 0, 0};
        if (i < n) {
            r = bt.recs[i];
            ow = pack_owner(r, G);
        }
        const uint32_t len4 = pack_len4(r.length);
        uint32_t my_l = 0, my_b = 0;   // exclusive rank / byte position among the wave's lines of my owner
        for (uint32_t o = 0; o < G; ++o) {
            const uint64_t m = __ballot(ow == (int)o);
            if (!m) {
                if (lane == 0) s_wl[wave][o] = s_wb[wave][o] = 0;
                continue;
            }
            const uint32_t v = ow == (int)o ? len4 : 0u;
            const uint32_t incl = wave_incl_add32(v);
            if (ow == (int)o) {
                my_l = __popcll(m & lt);
                my_b = incl - v;
            }
            if (lane == 63) {
                s_wl[wave][o] = (uint32_t)__popcll(m);
                s_wb[wave][o] = incl;
            }
        }
        __syncthreads();
        uint32_t dst = 0;
        if (ow >= 0) {
            uint32_t pl = s_run_l[ow], pb = s_run_b[ow];
            for (int w = 0; w < wave; ++w) {
                pl += s_wl[w][ow];
                pb += s_wb[w][ow];
            }
            const uint2 tb = p.tile_base[(size_t)blockIdx.x * G + ow];
            const uint32_t rel = tb.y + pb + my_b;   // byte position within the owner's chunk
            sr_record o = r;
            o.offset = rel;
            if (ow == p.own) {   // straight into its place in the receive buffers
                dst = rel;
                p.own_recs[tb.x + pl + my_l] = o;
            } else {
                dst = (uint32_t)(p.owner_start[2 * ow + 1] + rel);
                p.out_recs[p.owner_start[2 * ow] + tb.x + pl + my_l] = o;
            }
        }
        // the wave's owned lines compacted (k = rank among them), with their first piece
        const uint32_t npc = ow >= 0 ? ((uint32_t)r.length + 15u) >> 4 : 0u;
        const uint64_t owned = __ballot(npc != 0);
        const uint32_t pinc = wave_incl_add32(npc);
        const uint32_t pre = pinc - npc;
        const uint32_t T = __builtin_amdgcn_readlane(pinc, 63);
        if (npc) s_info[wave][__popcll(owned & lt)] =
            make_uint4(r.offset, dst, r.length | (ow == p.own ? 0x80000000u : 0u), pre);
        __syncthreads();
        if (tid < (int)G) {
            uint32_t al = 0, ab = 0;
            for (int w = 0; w < 4; ++w) {
                al += s_wl[w][tid];
                ab += s_wb[w][tid];
            }
            s_run_l[tid] += al;
            s_run_b[tid] += ab;
        }
        constexpr int kCopyBatch = SR_PACK_COPY_BATCH;
        const uint64_t own_cap = p.own >= 0 ? p.owner_counts[2 * p.own + 1] : 0ull;
        // Copy the wave's lines as one list of 16-byte pieces (a line of L bytes has ceil(L / 16)), every
        // lane moving 16 bytes per pass whatever the mix of lengths. Per window of kPackWin pieces: a bitmap
        // of the pieces where an owned line starts, and its per-dword prefix counts; the line of piece sp
        // is then (lines started before the window) + (starts at or before sp in it) - 1: two independent
        // LDS reads, then the line's record (a binary search over the wave's piece prefix took six
        // dependent LDS reads per piece). Per piece one dwordx4 buffer load at the source's byte offset
        // (unaligned buffer access; byte loads for the one piece that crosses the batch's end), then a
        // dwordx4 store, the line's last piece zero-filled to its 4-byte padding; the loads of kCopyBatch
        // passes issued before their stores
        uint32_t *const bm = s_bm[wave], *const bp = s_bp[wave];
        const uint4 *const info = s_info[wave];
        for (uint32_t w0 = 0; w0 < T; w0 += kPackWin) {
            if (lane < (int)(kPackWin / 32)) bm[lane] = 0u;
            pack_wave_sync();
            if (npc && pre >= w0 && pre < w0 + kPackWin) atomicOr(&bm[(pre - w0) >> 5], 1u << ((pre - w0) & 31u));
            const uint32_t kb = (uint32_t)__popcll(__ballot(npc != 0 && pre < w0));   // lines started before w0
            pack_wave_sync();
            const uint32_t cnt = lane < (int)(kPackWin / 32) ? (uint32_t)__popc(bm[lane]) : 0u;
            const uint32_t cin = wave_incl_add32(cnt);
            if (lane < (int)(kPackWin / 32)) bp[lane] = cin - cnt + kb;
            pack_wave_sync();
            const uint32_t wn = min(T - w0, kPackWin);
            for (uint32_t l0 = lane; l0 < wn; l0 += 64u * kCopyBatch) {
                uint4 v[kCopyBatch];
                uint32_t kq[kCopyBatch];   // line (6 bits) | byte within it << 6; ~0 past the window
#pragma unroll
                for (int u = 0; u < kCopyBatch; ++u) {
                    const uint32_t lc = l0 + 64u * u;
                    v[u] = make_uint4(0, 0, 0, 0);
                    kq[u] = ~0u;
                    if (lc < wn) {
                        const uint32_t d = lc >> 5;
                        const uint32_t k = bp[d] + (uint32_t)__popc(bm[d] & (0xFFFFFFFFu >> (31u - (lc & 31u)))) - 1u;
                        const uint4 in = info[k];
                        const uint32_t q = (w0 + lc - in.w) << 4;
                        kq[u] = k | (q << 6);
                        v[u] = load16(rsrc, in.x + q, bt.nbytes);
                    }
                }
#pragma unroll
                for (int u = 0; u < kCopyBatch; ++u) {
                    if (kq[u] == ~0u) break;
                    const uint32_t q = kq[u] >> 6;
                    const uint4 in = info[kq[u] & 63u];
                    const bool mine = (in.z >> 31) != 0;
                    const uint32_t L = in.z & 0x7FFFFFFFu, d = in.y;
                    uint8_t *const out = mine ? p.own_bytes : p.out_bytes;
                    const uint64_t cap = mine ? own_cap : p.out_cap;
                    uint8_t *o = out + d + q;
                    if (q + 16u <= L && (uint64_t)d + q + 16u <= cap) {   // a whole piece of the line
                        *(uint4 *)o = v[u];
                    } else {   // the line's last piece: zero fill up to its 4-byte padding
                        const uint32_t L4 = pack_len4(L);
                        uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) {
                            const uint32_t qj = q + 4u * jj;
                            if (qj >= L) w[jj] = 0;
                            else if (qj + 4u > L) w[jj] &= (1u << (8u * (L - qj))) - 1u;
                        }
                        if (q + 16u <= L4 && (uint64_t)d + q + 16u <= cap) {
                            *(uint4 *)o = make_uint4(w[0], w[1], w[2], w[3]);
                        } else {
#pragma unroll
                            for (int jj = 0; jj < 4; ++jj)
                                if (q + 4u * jj < L4 && (uint64_t)d + q + 4u * jj + 4u <= cap) ((uint32_t *)o)[jj] = w[jj];
                        }
                    }
                }
            }
            pack_wave_sync();   // the window's bitmap is read to the end before the next is built
        }
        __syncthreads();
    }
}

}  // namespace srk
