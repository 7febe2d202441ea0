// chunk_kernel.hpp — the route kernel in the CHUNK layout (SR_LAYOUT_CHUNKS): every lane hashes
// exactly the 64 bytes it loaded, whatever the line lengths. Same inputs, outputs and side
// outputs as route_kernel (records, hashes, deferred probes, probed-dead marks, line count) and
// the same per-batch scanners, arrivals and epochs (route_kernel.hpp); identical records.
//
// Reference path (hulu/statsd-router, /root/reference):
//   udp_read_cb        sr-main.c:149-191  '\n' tokeniser + length gate 5 < L < 1450
//   process_data_line  sr-main.c:137-147  ':' presence -> INVALID_FORMAT
//   hash               sr-main.c:120-134  sdbm over the name (signed char, u64 wrap)
//   find_downstream    sr-main.c:86-117   shard pick (probe_shard, route_kernel.hpp)
//
// The sdbm hash of a name [s, c) is a polynomial in K = 65599 over its bytes (mod 2^64), so it
// splits at the 64-byte chunk boundaries of a 16 KiB tile:
//   * U(l): Horner of chunk l's 64 bytes, straight from the load registers (8 steps of 8 bytes);
//   * Suf_l(q): Horner of bytes [q, 64) of chunk l (the shorter side of q is read from the chunk's
//     own LDS row: <= 32 bytes; the other side follows from U);
//   * Y(l): Horner of every tile byte up to the end of chunk l, from one 64-bit block scan of
//     U(l) K^(64 (255 - l)) and one multiply by K^-(64 (255 - l)) (per-lane constants);
//   * H(q) = Y(l) - Suf_l(q) for a position q in chunk l, and the name [s, c) of a line is
//       h = K^(c' - 64) (H(c) - K^(64 (lc - ls)) H(s))          (c' = c mod 64, lc / ls the chunks)
//     Positions q that start or end a line spanning chunks are few; their H go to LDS slots
//     indexed by the line's start chunk, and the lane holding the line's '\n' combines them.
// A tile none of whose chunks a line crosses (every chunk ends in '\n': 64-byte aligned lines)
// needs neither the scan nor the slots: Y cancels from H(c) - H(s) when both lie in one chunk.
// The line that straddles into a tile is finished from its predecessor's TAIL granules (the
// open line's start, whether its colon was seen, and its partial or final hash: a decoupled
// look-back on hashes), so no tile reads or hashes bytes outside its own 16 KiB.
#pragma once

#include "route_kernel.hpp"

namespace srk {

constexpr unsigned KV_CHUNKS = 8388608u;       // the chunk-layout kernel (route_chunk_kernel)
// developer ablations of route_chunk_kernel (timing / counter attribution only, wrong records; built
// with -DSR_CHUNK_ABL=<mask> into tools/ab, never shipped)
enum : unsigned { CH_ABL_NO_U = 1u << 24, CH_ABL_NO_SUF = 1u << 25, CH_ABL_NO_EMIT = 1u << 26 };
constexpr int kCinv = 65;                      // K^-z, z = 0 .. 64
constexpr int kCpowEntries = kCinv + 2 * 256;  // + K^(64 (255 - l)), K^-(64 (255 - l)) per lane l
constexpr uint32_t kFlagTail = 1u;             // tail granules (flag field of mk_status)
// tail meta: bits 0..14 the open line's start in the tile (1 .. 16383), and
constexpr uint32_t kTailNoNl = 1u << 15;       // the tile holds no '\n' (the line is > 16 KiB)
constexpr uint32_t kTailColon = 1u << 16;      // its first ':' lies in the tile: the hash is final
constexpr uint32_t kTailLong = 1u << 17;       // already longer than SR_MAX_LINE_LENGTH: no hash
constexpr uint32_t kSlotBefore = 256;          // slot of a line that starts before the tile

struct ChunkSmem {
    static constexpr int kRows = 256;
    static constexpr int kWords = kRows * 17 + 4;   // 17-dword rows (pad dword 16: probe_shard's)
    alignas(16) uint32_t wsc[4][4];   // per wave (lane 63): '\n' count, last '\n' + 1, colon key, flags
    uint64_t wv[4];            // per wave: inclusive sum of U(l) K^(64 (255 - l))
    uint32_t img[kWords];
    uint64_t hs[257];          // H(start) of the line that starts in chunk l and leaves it
    uint64_t hc[257];          // H(first ':') of that line, when the ':' lies in another chunk
    uint64_t kp_lo[kPowLo];    // K^i (i < 64)      } contiguous: one copy from RouteParams::kpow
    uint64_t kp_hi[kPowHi];    // K^(64 i) (i < 24) }
    uint64_t kinv[kCinv];      // K^-z
    uint32_t head_nl;          // the byte before the tile is '\n' (or the tile starts the batch)
    uint32_t scan_head, scan_pub, scan_total;   // scanner blocks
};
static_assert(sizeof(ChunkSmem) <= 23040, "7 workgroups per CU (LDS granules of 512 bytes)");

// Horner of the n bytes [a, a + n) of one 64-byte image row (a + n <= 64; 0 for n == 0): the
// bytes of the first dword before a are masked off (leading zeros leave a Horner value unchanged),
// a partial last dword is shifted up so that its bytes past the run drop out (h K^rem + Horner).
__device__ __forceinline__ uint64_t row_horner(const uint32_t *row, const uint64_t *kp_lo, int a, int n) {
    if (n <= 0) return 0;
    const int lead = a & 3, L = lead + n, F = L >> 2, rem = L & 3;
    const uint32_t *const q = row + (a >> 2);
    const uint32_t first = q[0] & (0xFFFFFFFFu << (8 * lead));
    if (F == 0) return sdbm_dword_fast(0, first << (8 * (4 - rem)));
    uint64_t h = sdbm_dword_fast(0, first);
    int m = 1;
    for (; m + 1 < F; m += 2) h = sdbm_qword_fast(h, q[m], q[m + 1]);
    if (m < F) h = sdbm_dword_fast(h, q[m++]);
    if (rem) h = h * kp_lo[rem] + sdbm_dword_fast(0, q[m] << (8 * (4 - rem)));
    return h;
}

// 16 bytes at `a` by byte loads: bytes past the buffer's range read as 0, exactly
__device__ __forceinline__ uint4 load16_bytes(__amdgpu_buffer_rsrc_t rsrc, uint32_t a) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, a + i, 0, 0) << (8 * (i & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Wave-cooperative helpers of the look-back fallback (a predecessor that never published, or a
// line longer than a tile): the start of the line holding byte `before` - 1, and the sdbm of
// [a, b) (b - a <= SR_MAX_LINE_LENGTH) with its first ':' if any, from global memory.
__device__ uint32_t wave_line_start(__amdgpu_buffer_rsrc_t rsrc, uint32_t nbytes, uint32_t before, int lane) {
    int64_t hi = before;
    while (hi > 0) {
        const int64_t lo = hi - 1024 > 0 ? hi - 1024 : 0;
        const int64_t a = lo + lane * 16;
        uint32_t nl16 = 0;
        if (a < hi) {
            nl16 = eq_mask16(load16(rsrc, (uint32_t)a, nbytes), 0x0A0A0A0Au);
            const int keep = (int)(hi - a) < 16 ? (int)(hi - a) : 16;
            nl16 &= (1u << keep) - 1u;
        }
        const uint64_t mm = __ballot(nl16 != 0);
        if (mm) {
            const int L = 63 - __builtin_clzll(mm);
            return (uint32_t)readlane64((uint64_t)(a + 31 - __builtin_clz(nl16 | 1u)), L) + 1u;
        }
        hi = lo;
    }
    return 0;
}

// sdbm of the name part of [a, b): bytes up to the first ':' (returned in *colon, or ~0u).
// Lane l takes bytes [a + l z, a + (l + 1) z), z = ceil((b - a) / 64) <= 23.
template <class S>
__device__ uint64_t wave_name_hash(const S &sm, __amdgpu_buffer_rsrc_t rsrc, uint32_t nbytes, uint32_t a, uint32_t b,
                                   uint32_t *colon, int lane) {
    const uint32_t n = b > a ? b - a : 0u;
    const uint32_t z = (n + 63u) / 64u;
    const uint32_t x0 = a + (uint32_t)lane * z, x1 = min(x0 + z, b);
    uint32_t first = ~0u;
    for (uint32_t x = x0; x < x1 && first == ~0u; ++x)
        if (__builtin_amdgcn_raw_buffer_load_b8(rsrc, x, 0, 0) == ':') first = x;
    uint32_t c = first;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c = min(c, (uint32_t)__shfl_xor((int)c, d, 64));
    *colon = c;
    const uint32_t end = c < b ? c : b;   // the name ends at the first ':' or at b
    uint64_t h = 0;
    for (uint32_t x = x0; x < x1 && x < end; ++x)
        h = sdbm_step(h, x < nbytes ? __builtin_amdgcn_raw_buffer_load_b8(rsrc, x, 0, 0) : 0u);
    const uint32_t seg_end = min(x1, end);
    if (x0 < seg_end && end > seg_end) h *= kpow_n(sm, (int)(end - seg_end));
    if (x0 >= seg_end) h = 0;
    return wave_sum64(h);
}

// keep a value's computation where it is written (an empty volatile asm that "modifies" it):
// LLVM otherwise sinks long chains to their last uses and holds their inputs live instead
__device__ __forceinline__ void pin64(uint64_t &x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    asm volatile("" : "+v"(lo), "+v"(hi));
    x = ((uint64_t)hi << 32) | lo;
}

template <unsigned ABL>
__global__ __launch_bounds__(256, 7) __attribute__((amdgpu_waves_per_eu(7, 8))) void route_chunk_kernel(RouteParams p) {
    __shared__ ChunkSmem sm;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    uint4 hdr;
    const uint32_t bi = launch_header_batch(hdr);
    if (blockIdx.x < hdr.x) {   // scanner of batch blockIdx.x, as in route_kernel
        __builtin_amdgcn_s_setprio(3);
        if (uint64_t *pd = p.b[blockIdx.x].probed_dead)
            for (uint32_t w = tid; w < p.nwords; w += 256) pd[w] = 0ull;
        const uint32_t ep0 = __hip_atomic_load(&p.ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tid == 0) {
            sm.scan_head = 0;
            sm.scan_pub = 0;
            sm.scan_total = 0;
        }
        wg_barrier();
        scan_batch_split<256, ABL>(p, p.b[blockIdx.x], ep0, sm, wave, lane);
        if (tid == 64) arrive(p, blockIdx.x, ep0);
        return;
    }
    const uint32_t g = blockIdx.x - hdr.x;
    stamp<ABL>(p, tid, g, 8);
    if (bi >= kMaxBatches) {
        if (tid == 0) arrive(p, blockIdx.x, __hip_atomic_load(&p.ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        return;
    }
    const BatchDesc &bd = p.b[bi];
    const uint32_t nbytes = bd.nbytes;
    const uint32_t t = (hdr.z ? (g >> 3) : g) - bd.tile0;   // the tile's index in its batch
    const uint32_t T0 = t * 16384u;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)bd.bytes, (short)0, (int)nbytes, 0x00020000);
    const int o = tid * 64;   // the lane's chunk: tile bytes [o, o + 64)

    // ---- entry: the chunk's loads first, then the tables and granules that queue behind them ----
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        v[k] = as_uint4(__builtin_amdgcn_raw_buffer_load_b128(rsrc, T0 + (uint32_t)o + 16u * k, 0, 0));
    // unconditional loads (clamped addresses): a load under a lane condition becomes a branch and a
    // wait of its own
    constexpr int kKpWords = 2 * (kPowLo + kPowHi);
    const uint32_t kw = ((const uint32_t *)p.kpow)[tid < kKpWords ? tid : kKpWords - 1];
    const uint32_t iw = ((const uint32_t *)p.cpow)[tid < 2 * kCinv ? tid : 2 * kCinv - 1];
    // the block scan's per-lane constants K^(64 (255 - l)) and K^-(64 (255 - l)), queued behind the
    // tile's loads: in a tile that some line crosses a chunk boundary of (most C5 tiles), asked for
    // only after the first barrier they were a dependent round trip of their own
    const uint64_t R = p.cpow[kCinv + tid], RI = p.cpow[kCinv + 256 + tid];
    // the dword before the tile (its last byte: does the tile start a line?), after the tables and at a
    // clamped address: loaded under `t > 0` it was a branch whose value the compiler waited for at once,
    // i.e. for every tile load, before the tables' loads were even issued (a round trip more per tile)
    const uint32_t pw = __builtin_amdgcn_raw_buffer_load_b32(rsrc, T0 ? T0 - 4u : 0u, 0, 0);
    if (T0 + 16384u > nbytes) {
        // the batch's last tile: a piece past the end reads as zeros, but the range check of a 16-byte
        // load that straddles the end is not byte-exact (its bytes before the end can read as zero
        // too): that one piece is read again byte by byte (byte loads are range-checked exactly)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t a = T0 + (uint32_t)o + 16u * k;
            if (a < nbytes && a + 16u > nbytes) v[k] = load16_bytes(rsrc, a);
        }
    }
    const uint32_t ep0 = __hip_atomic_load(&p.ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t sx = __hip_atomic_load(&p.ctl->scan_xcc[bi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) arrive_count(p, blockIdx.x);   // as route_kernel's tiles (kEarlyArrive)
    if (!(ABL & (KV_ALIVE | KV_DEFER1 | KV_DEAD1)) && p.dead && p.dead < p.nds && tid < 4 * (int)kMagicLds) {   // probe_shard's first reciprocals
        const uint32_t e = (uint32_t)tid >> 2;
        if (e < p.nds) sm.img[(uint32_t)tid * 17 + 16] = ((const uint32_t *)&p.magic[p.nds - e])[tid & 3];
    }
    if (!(ABL & (KV_ALIVE | KV_DEFER1 | KV_DEAD1)) && p.dead && p.dead < p.nds && p.nds <= 64 * kAliveLds && tid >= (int)kAliveRow0 &&
        (uint32_t)tid < kAliveRow0 + 2 * ((p.nds + 63) / 64))   // the alive words (probe_shard)
        sm.img[(uint32_t)tid * 17 + 16] = ((const uint32_t *)p.alive)[tid - kAliveRow0];
    if (!(ABL & (KV_ALIVE | KV_DEFER1)) && p.mark_tiles && tid >= (int)kMarkRow0 && (uint32_t)tid < kMarkRow0 + 2 * p.nwords)   // MARK_LDS: none yet
        sm.img[(uint32_t)tid * 17 + 16] = 0u;
    if (tid == 0) sm.hs[kSlotBefore] = 0ull;
    const uint32_t pf = prefetch_tile(p, bd, t, tid);

    // ---- the chunk: LDS row, '\n' / ':' masks ------------------------------------------------
    uint64_t nlm, clm;
    {
        const uint32_t rb = lds_addr(&sm.img[tid * 17]);
        ds_write2_at<0, 1>(rb, v[0].x, v[0].y);
        ds_write2_at<2, 3>(rb, v[0].z, v[0].w);
        ds_write2_at<4, 5>(rb, v[1].x, v[1].y);
        ds_write2_at<6, 7>(rb, v[1].z, v[1].w);
        ds_write2_at<8, 9>(rb, v[2].x, v[2].y);
        ds_write2_at<10, 11>(rb, v[2].z, v[2].w);
        ds_write2_at<12, 13>(rb, v[3].x, v[3].y);
        ds_write2_at<14, 15>(rb, v[3].z, v[3].w);
        stamp<ABL>(p, tid, g, 0);   // (the row's stores need the loads: they have arrived)
        uint32_t m[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] = nl_colon_mask16(v[k]);
        nlm = ((uint64_t)__builtin_amdgcn_perm(m[3], m[2], 0x05040100u) << 32) | __builtin_amdgcn_perm(m[1], m[0], 0x05040100u);
        clm = ((uint64_t)__builtin_amdgcn_perm(m[3], m[2], 0x07060302u) << 32) | __builtin_amdgcn_perm(m[1], m[0], 0x07060302u);
        pin64(nlm);
        pin64(clm);
    }
    if (tid < kKpWords) ((uint32_t *)&sm.kp_lo[0])[tid] = kw;   // kp_lo | kp_hi are contiguous
    if (tid < 2 * kCinv) ((uint32_t *)&sm.kinv[0])[tid] = iw;
    if (tid == 0) sm.head_nl = t == 0 || (pw >> 24) == 0x0Au ? 1u : 0u;

    // ---- line state: three u32 wave scans, the wave totals in LDS ------------------------------
    const uint32_t nrel = nbytes - T0;             // batch bytes from the tile start (> 0)
    const bool valid = (uint32_t)o < nrel;         // the chunk holds batch bytes
    const int lastnl = nlm ? 63 - __clzll(nlm) : -1;
    // first ':' after the chunk's last '\n' (all of the chunk without one): the colon candidate of
    // the line open at the chunk's end (route_kernel's lane_cand)
    const uint64_t cafter = lastnl >= 63 ? 0ull : (clm & (~0ull << (lastnl + 1)));
    const uint32_t cand = cafter ? (uint32_t)(o + __builtin_ctzll(cafter)) : (uint32_t)kNone;
    const uint32_t c_in = wave_incl_add32((uint32_t)__popcll(nlm));
    const uint32_t nl_in = wave_incl_max32(nlm ? (uint32_t)(o + lastnl + 1) : 0u);
    const uint32_t k_in = wave_incl_min32(((8191u - c_in) << 17) | cand);
    const uint32_t flags = (__ballot(__popcll(nlm) > 1) ? 1u : 0u) | (__ballot(valid && !(nlm >> 63)) ? 2u : 0u);
    if (lane == 63) *(uint4 *)&sm.wsc[wave][0] = make_uint4(c_in, nl_in, k_in, flags);
    wg_barrier();   // B1
    stamp<ABL>(p, tid, g, 1);
    uint32_t tile_count = 0, tflags = 0, tl = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint4 ws = *(const uint4 *)&sm.wsc[w][0];
        tile_count += ws.x;
        tflags |= ws.w;
        tl = max(tl, ws.y);
    }
    if (tid == 0) {   // the tile's '\n' count for the scanner (route_kernel's tile_load)
        const uint32_t x = xcc_id();
        const bool same = granule_ok(sx, ep0 & 0x3FFFFFFFu, kFlagXcc) && (uint32_t)sx == x;
        granule_store(&p.status[bd.sbase + t], mk_status(ep0, kFlagAgg, tile_count | ((8u | x) << 28)), same);
    }
    const uint64_t *const base_slot = p.bases + bd.sbase + t;
    const bool long_tile = (tflags & 2u) != 0;
    // the lane's exclusive state: lines before its chunk, the last '\n' before it (+ 1), and the
    // first ':' of the line open at its start (route_kernel's lane_state)
    uint32_t p_cnt = 0, p_col = (uint32_t)kNone, p_nl = 0;
#pragma unroll
    for (int w = 0; w < 3; ++w) {
        if (w < wave) {
            const uint4 ws = *(const uint4 *)&sm.wsc[w][0];
            p_cnt += ws.x;
            p_nl = max(p_nl, ws.y);
            const uint32_t wc = ws.z & 0x1FFFFu;
            p_col = ws.x ? wc : min(p_col, wc);
        }
    }
    const uint32_t c_ex = wave_shr1_32(c_in, 0u);
    const uint32_t k_ex = wave_shr1_32(k_in, 0xFFFFFFFFu) & 0x1FFFFu;
    const int lf = (int)(p_cnt + c_ex);                                   // tile-local index of my first line
    const int ofc = (int)(c_ex ? k_ex : min(p_col, k_ex));               // first ':' of the line open at o
    const int prevnl = (int)max(p_nl, wave_shr1_32(nl_in, 0u));         // its start (0: the tile's first line)
    const bool before = prevnl == 0 && !sm.head_nl;                      // ... which began in an earlier tile
    const uint32_t ih = before ? kSlotBefore : (uint32_t)prevnl >> 6;   // its slot

    // ---- U: Horner of the chunk's 64 bytes, from its LDS row. After the count is published: a
    // tile's record base follows its predecessors' counts through the scanner, so the earlier the
    // counts go out, the less the tiles wait for their bases when they write their records ----------
    const uint32_t *const row = &sm.img[tid * 17];
    uint64_t U;
    {
        uint32_t x[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = row[i];
        U = sdbm_qword_fast(0ull, x[0], x[1]);
#pragma unroll
        for (int i = 2; i < 16; i += 2) U = sdbm_qword_fast(U, x[i], x[i + 1]);
        if (ABL & CH_ABL_NO_U) U = x[0];
        pin64(U);   // materialised here: sunk to its late uses it would keep 32 pair products live
    }

    // ---- the positions that need H: the open line's first ':' in this chunk, the chunk's tail line
    // (after its last '\n') and that line's first ':' ----------------------------------------------
    const int firstnl = nlm ? __builtin_ctzll(nlm) : 64;
    const uint64_t c0m = clm & (firstnl == 64 ? ~0ull : ((1ull << firstnl) - 1ull));
    const bool ev1 = ofc == kNone && c0m != 0ull;                         // the open line's first ':'
    const bool has_tail = valid && nlm != 0ull && lastnl < 63;           // a line starts in the chunk and leaves it
    const bool ev3 = has_tail && cafter != 0ull;
    auto suf = [&](int q) -> uint64_t {   // Suf(q) = Horner of [q, 64), 0 <= q < 64
        const bool back = q >= 32;         // read the shorter side
        const uint64_t r = row_horner(row, sm.kp_lo, back ? q : 0, back ? 64 - q : q);
        return back ? r : U - r * sm.kp_lo[(64 - q) & 63];
    };
    uint64_t S1 = 0, S2 = 0, S3 = 0;
    if (!(ABL & CH_ABL_NO_SUF) && __ballot(ev1)) {
        if (ev1) S1 = suf(__builtin_ctzll(c0m));
    }
    if (!(ABL & CH_ABL_NO_SUF) && __ballot(has_tail)) {
        if (has_tail) S2 = suf(lastnl + 1);
        if (ev3) S3 = suf(__builtin_ctzll(cafter));
    }
    stamp<ABL>(p, tid, g, 2);

    // ---- Y and the slots (only when some line crosses a chunk boundary) ------------------------
    uint64_t Y = tid == 0 ? U : 0ull;   // exact for chunk 0; elsewhere it cancels when s, c share a chunk
    if (long_tile) {
        const uint64_t Sw = wave_scan64(U * R, 0ull, [](uint64_t l, uint64_t r) { return l + r; });
        if (lane == 63) sm.wv[wave] = Sw;
        wg_barrier();   // B2
        uint64_t pre = 0;
#pragma unroll
        for (int w = 0; w < 3; ++w)
            if (w < wave) pre += sm.wv[w];
        Y = (Sw + pre) * RI;
        if (ev1 && nlm == 0ull) sm.hc[ih] = Y - S1;                    // its '\n' lies in a later chunk
        if (has_tail) {
            sm.hs[tid] = Y - S2;
            if (ev3) sm.hc[tid] = Y - S3;
        } else if (valid && nlm == 0ull && !before && prevnl == o) {
            sm.hs[tid] = Y - U;                                         // starts at o, ends later
        }
        wg_barrier();   // B3
        if (tid == 255 && valid && !(nlm >> 63)) {
            // the tile's open line, for the next tile: its start, its first ':' and hash so far
            const uint32_t cend = c_in ? (k_in & 0x1FFFFu) : min(p_col, k_in & 0x1FFFFu);   // ':' at the tile end
            uint32_t meta = 0;
            uint64_t q = 0;
            if (tl == 0) {
                meta = kTailNoNl;
            } else {
                const uint32_t ls = tl >> 6;
                meta = tl;
                if (16384u - tl > SR_MAX_LINE_LENGTH) {
                    meta |= kTailLong;
                } else if (cend != (uint32_t)kNone) {
                    meta |= kTailColon;
                    q = sm.kinv[64 - (cend & 63u)] * (sm.hc[ls] - sm.kp_hi[(cend >> 6) - ls] * sm.hs[ls]);
                } else {
                    q = Y - sm.kp_hi[255u - ls] * sm.hs[ls];
                }
            }
            uint64_t *const tg = p.tail + (size_t)(bd.sbase + t) * 4u;
            __hip_atomic_store(&tg[1], mk_status(ep0, kFlagTail, (uint32_t)q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&tg[2], mk_status(ep0, kFlagTail, (uint32_t)(q >> 32)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&tg[0], mk_status(ep0, kFlagTail, meta), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    stamp<ABL>(p, tid, g, 4);

    // ---- records ------------------------------------------------------------------------------
    // The tile's first record index: the freshest base the scanner has published among the 64 tiles
    // up to this one, plus the counts published since (each wave on its own, one round trip per try).
    // The scanner needs ~1.2 us to turn a count into a base; a chunk-layout tile publishes its count
    // only ~1.3 us before it writes its records, so waiting for the scanner's base of this very tile
    // cost 1.7 us per tile (stamps).
    uint32_t base = 0;
    if (t > 0) {
        const uint32_t ep = ep0 & 0x3FFFFFFFu;
        const int c = (int)t - lane;       // lane l: the scanner's base of tile t - l ...
        const int cc = c - 1;              // ... and the count of tile t - 1 - l
        bool done = false;
        for (uint32_t spin = 0; spin < (uint32_t)kSpinBudget && !done; ++spin) {
            const uint64_t bg = __hip_atomic_load(&p.bases[bd.sbase + (uint32_t)max(c, 0)], __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t cg = __hip_atomic_load(&p.status[bd.sbase + (uint32_t)max(cc, 0)], __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
            const bool bok = c == 0 || (c > 0 && granule_ok(bg, ep, kFlagBase));   // tile 0's base is 0
            const bool cok = cc >= 0 && granule_ok(cg, ep, kFlagAgg);
            const uint64_t okc = __ballot(cok);
            const int nc = ~okc ? __builtin_ctzll(~okc) : 64;   // counts of tiles t-1 .. t-nc are in
            const uint64_t cand = __ballot(bok && lane <= nc);
            if (cand) {
                const int l = __builtin_ctzll(cand);
                const uint32_t pre = wave_incl_add32(cok ? ((uint32_t)cg & kCountMask) : 0u);
                base = (uint32_t)__builtin_amdgcn_readlane((int)(c > 0 ? (uint32_t)bg : 0u), l) +
                       (l ? (uint32_t)__builtin_amdgcn_readlane((int)pre, l - 1) : 0u);
                done = true;
            } else {
                if (spin == 0) stamp<ABL>(p, tid, g, 3);
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (!done) base = wait_base(base_slot, ep0, rsrc, T0);
        stamp<ABL>(p, tid, g, 7);
        base = __builtin_amdgcn_readfirstlane(base);
    }
    auto emit = [&](int j, uint32_t off, int len, bool len_ok, bool fmt_ok, uint64_t h) {
        uint32_t route;
        if (!len_ok) route = SR_ROUTE_INVALID_LENGTH;
        else if (!fmt_ok) route = SR_ROUTE_INVALID_FORMAT;
        else if (ABL & KV_ALIVE) route = p.nds ? mod_magic(h, p.magic_n, p.nds) : SR_ROUTE_ALL_DEAD;   // :145
        else if (ABL & KV_DEFER1) route = defer1_probe(h, p);   // :145
        else if (ABL & KV_DEAD1) route = dead1_probe(h, p, sm.img);   // :145
        else route = chunk_probe(h, p, sm.img);   // :145
        const bool deferred = !(ABL & KV_ALIVE) && route == kRouteDefer;
        if (deferred) route = kRoutePending;
        const uint32_t rec = base + (uint32_t)j;
        if (rec < bd.max_records) {
            if (deferred) bd.dhash[rec] = h;
            if (!(ABL & (KV_ALIVE | KV_DEFER1 | KV_DEAD1)) && route == kRoutePending && !deferred) {
                const uint32_t slot = atomicAdd(&p.ctl->pending, 1u);
                if (slot < p.pending_cap) p.pending[slot] = PendingLine{rec, bi, h};
            }
            sr_record r;
            r.offset = off;
            r.length = len > 0xFFFF ? (uint16_t)0xFFFF : (uint16_t)len;
            r.route = (uint16_t)route;
            bd.recs[rec] = r;
            if (bd.hashes) bd.hashes[rec] = h;
        }
    };
    // The chunk's first line: its name hash within the tile, h = K^(c' - 64) (H(c) - K^(64 (lc - ls)) H(s))
    // (H(s) = 0 for a line that began in an earlier tile: its earlier part comes from the look-back).
    // A line within the chunk (C2: every line) is K^(c' - 64) (U - Suf(c')): no slots, no Y.
    const int c_first = ofc != kNone ? ofc : (c0m ? o + __builtin_ctzll(c0m) : kNone);
    const int e0 = o + firstnl;
    uint64_t hin0 = 0;
    if (nlm && c_first != kNone && c_first < e0) {
        if (prevnl == o && !before) {
            hin0 = sm.kinv[64 - (c_first & 63)] * (U - S1);
        } else {
            const uint64_t hcv = c_first >= o ? Y - S1 : sm.hc[ih];
            const uint64_t hsv = before ? 0ull : sm.hs[ih];
            const int d = before ? 0 : min((c_first >> 6) - (prevnl >> 6), kPowHi - 1);   // <= 23 for valid lines
            hin0 = sm.kinv[64 - (c_first & 63)] * (hcv - sm.kp_hi[d] * hsv);
        }
    }
    if (!(ABL & CH_ABL_NO_EMIT)) {
        if (nlm && !before) {   // the chunk's first line (one that began in an earlier tile: below)
            const int len = e0 - prevnl + 1;
            const bool len_ok = len >= (int)SR_MIN_LINE_LENGTH && len <= (int)SR_MAX_LINE_LENGTH;   // :180
            const bool fmt_ok = c_first != kNone && c_first < e0;                                  // :140
            emit(lf, T0 + (uint32_t)prevnl, len, len_ok, fmt_ok, len_ok && fmt_ok ? hin0 : 0ull);
        }
        // further lines of a chunk with several '\n' (lines under 64 bytes): within the chunk
        if (__ballot(__popcll(nlm) > 1)) {
            uint64_t rest = nlm & (nlm - 1ull);
            int prev = firstnl, j = lf + 1;
            while (rest) {
                const int eb = __builtin_ctzll(rest);
                rest &= rest - 1ull;
                const int len = eb - prev;
                const uint64_t cm = clm & ((1ull << eb) - 1ull) & (~0ull << (prev + 1));
                const bool len_ok = len >= (int)SR_MIN_LINE_LENGTH && len <= (int)SR_MAX_LINE_LENGTH;
                const bool fmt_ok = cm != 0ull;
                uint64_t h = 0;
                if (len_ok && fmt_ok) {
                    const int cq = __builtin_ctzll(cm);
                    h = sm.kinv[64 - cq] * (suf(prev + 1) - suf(cq));
                }
                emit(j, T0 + (uint32_t)(o + prev + 1), len, len_ok, fmt_ok, h);
                prev = eb;
                ++j;
            }
        }
    }
    stamp<ABL>(p, tid, g, 5);

    stamp<ABL>(p, tid, g, 6);
    // ---- the line that began in an earlier tile: its predecessor's tail granules ----------------
    const bool lb = nlm != 0ull && before;
    const uint64_t lbm = __ballot(lb);
    if (!(ABL & CH_ABL_NO_EMIT) && lbm) {
        const int L = __builtin_ctzll(lbm);
        const uint64_t *const tg = p.tail + (size_t)(bd.sbase + t - 1u) * 4u;
        const uint32_t ep = ep0 & 0x3FFFFFFFu;
        uint64_t gr = 0;
        bool ok = false;
        for (uint32_t spin = 0; spin < p.lb_spin; ++spin) {
            gr = lane < 3 ? __hip_atomic_load(&tg[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
            if (__ballot(lane < 3 && granule_ok(gr, ep, kFlagTail)) == 7ull) {
                ok = true;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        uint32_t meta = (uint32_t)__shfl((int)(uint32_t)gr, 0, 64);
        uint64_t q = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)gr, 2, 64) << 32) | (uint32_t)__shfl((int)(uint32_t)gr, 1, 64);
        uint32_t s_abs;
        if (ok && !(meta & kTailNoNl)) {
            s_abs = T0 - 16384u + (meta & 0x7FFFu);
        } else {   // never published (or no '\n' in it): find the line's start in global memory
            s_abs = wave_line_start(rsrc, nbytes, T0, lane);
            meta = 0;
            if (T0 - s_abs > SR_MAX_LINE_LENGTH) {
                meta = kTailLong;
            } else {
                uint32_t colon;
                q = wave_name_hash(sm, rsrc, nbytes, s_abs, T0, &colon, lane);
                if (colon < T0) meta = kTailColon;
            }
        }
        if (lane == L) {
            const int len = (int)(T0 + (uint32_t)e0 - s_abs + 1u);
            const bool len_ok = !(meta & kTailLong) && len >= (int)SR_MIN_LINE_LENGTH && len <= (int)SR_MAX_LINE_LENGTH;
            bool fmt_ok = true;
            uint64_t h = q;   // the name ended in the earlier tile (kTailColon)
            if (!(meta & kTailColon)) {
                fmt_ok = c_first != kNone && c_first < e0;
                h = (len_ok && fmt_ok) ? q * kpow_n(sm, c_first) + hin0 : 0ull;
            }
            if (!(len_ok && fmt_ok)) h = 0;
            emit(lf, s_abs, len, len_ok, fmt_ok, h);
        }
    }
    mark_tile_end<ABL>(p, sm.img, bd, t, tid);   // MARK_LDS: the dead shards this tile's probes visited
    if (tid == 0) arrive_last(p, blockIdx.x, ep0);
    prefetch_sink(pf);
    stamp<ABL>(p, tid, g, 9);
}

}  // namespace srk
