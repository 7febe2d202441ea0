// persist_kernel.hpp — the chunk-layout route kernel as PERSISTENT workgroups that keep the next
// tile's bytes in flight while they route the current one (launches whose every shard is alive).
//
// Reference path (hulu/statsd-router, /root/reference): as route_chunk_kernel (chunk_kernel.hpp):
//   udp_read_cb sr-main.c:149-191, process_data_line :137-147, hash :120-134, find_downstream's
//   all-alive pick h % N :86-117 (the first probe step with every shard alive).
//
// Why: the one-shot kernels give each 16 KiB tile one workgroup whose loads are in
// flight only during its first ~2.4 us of an ~8 us life, so 7 workgroups per CU keep ~34 KB in
// flight per CU: at the ~2.4 us latency of loaded HBM that is ~3.7 TB/s, the measured rate. Here a
// workgroup takes its XCD class's tiles in order from a counter (one atomic per tile, fetched a tile
// ahead; workgroups that start late take fewer) and issues tile k+1's bytes by LDS-DMA (buffer_load_dwordx4 ... lds: no VGPRs, counted by vmcnt,
// waited for with a counted s_waitcnt at the top of the next iteration) before it routes tile k, so
// every workgroup has a tile in flight all the time: two 16 KiB images per workgroup, 4 workgroups
// per CU, 64 KiB in flight per CU.
//
// LDS image: tile byte b at b (the DMA's lane-linear destination with coalesced 1 KiB reads per
// wave-instruction); lane l's chunk (bytes [64 l, 64 l + 64)) lies in its own wave's DMA region, so
// a wave reads only what its own loads wrote and needs no barrier for the image. The per-tile LDS
// words that waves exchange (wave scans, the byte before the tile) alternate by tile parity.
// Records, hashes, line counts, tail and count granules, look-backs, scanners and arrivals are
// route_chunk_kernel's, bit for bit (tests/test_gpu_layout.py, SR_LAYOUT_PERSIST).
#pragma once

#include "chunk_kernel.hpp"

namespace srk {

constexpr unsigned KV_PERSIST = 1u << 30;

struct PersistSmem {
    union {
        uint32_t img[8192];            // the scanner blocks' ring (scan_batch_split)
        uint32_t buf[2][4096];         // two tile images (tile parity)
    };
    alignas(16) uint32_t wsc[2][4][4];   // per parity, per wave (lane 63): '\n' count, last '\n' + 1, colon key, flags
    uint32_t pw[2][64];                // per parity: the dword before the tile (wave 0's LDS-DMA, every lane the same)
    uint64_t wv[4];                    // per wave: inclusive sum of U(l) K^(64 (255 - l))
    uint64_t hs[257];                  // H(start) of the line that starts in chunk l and leaves it
    uint64_t hc[257];                  // H(first ':') of that line, when the ':' lies in another chunk
    uint64_t kp_lo[kPowLo];            // K^i (i < 64)      } contiguous: one copy from RouteParams::kpow
    uint64_t kp_hi[kPowHi];            // K^(64 i) (i < 24) }
    uint64_t kinv[kCinv];              // K^-z
    uint32_t scan_head, scan_pub, scan_total;   // scanner blocks
    uint32_t take;                     // the tile the workgroup's last atomic took
    static constexpr int kWords = 8192;
};
static_assert(sizeof(PersistSmem) <= 40 * 1024, "4 workgroups per CU (160 KiB of LDS)");

// One tile's bytes by LDS-DMA: wave w's four 1 KiB pieces of tile ci of XCD class cls into image
// `par` (tile byte b at image byte b), and wave 0 also the dword before the tile into pw[par]. Bytes
// past the batch read as zeros (buffer range check). vm operations per wave: 4, wave 0: 5.
__device__ __forceinline__ void persist_issue(const RouteParams &p, PersistSmem &sm, uint32_t cls, uint32_t ci,
                                              uint32_t par, int wave, int lane) {
    uint32_t t = 0;
    const uint32_t bi = batch_of(p, cls, ci, t);
    const BatchDesc &bd = p.b[bi < kMaxBatches ? bi : 0];
    const uint32_t T0 = t * 16384u;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)bd.bytes, (short)0, (int)bd.nbytes, 0x00020000);
    typedef __attribute__((address_space(3))) void *lds_ptr;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr)&sm.buf[par][wave * 1024 + k * 256], 16,
                                                 T0 + (uint32_t)(wave * 4096 + k * 1024 + lane * 16), 0, 0, 0);
    if (wave == 0)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr)&sm.pw[par][0], 4, t ? T0 - 4u : 0u, 0, 0, 0);
}

template <unsigned ABL>
__global__ __launch_bounds__(256, 4) void route_persist_kernel(RouteParams p) {
    static_assert((ABL & KV_ALIVE) != 0, "the persistent kernel routes launches with every shard alive");
    __shared__ PersistSmem sm;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    if (blockIdx.x < p.nb) {   // scanner of batch blockIdx.x, as in route_kernel
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
    const uint32_t g = blockIdx.x - p.nb;
    const uint32_t cls = p.xcd_local ? (g & 7u) : 0u;
    const uint32_t w0 = p.xcd_local ? (g >> 3) : g;   // this workgroup's index among its class's
    uint32_t ntc = 0;                                 // tiles of the class
#pragma unroll
    for (int k = 0; k < kPerClass; ++k)
        if (p.cls_tab[cls][k] != ~0u) ntc = max(ntc, p.cls_tab[cls][k] >> 6);
    (void)w0;
    const uint32_t ep0 = __hip_atomic_load(&p.ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t *const ctr = &p.ctl->ptile[cls][0];
    // the class's tiles in order: one atomic per tile (lane 0 of wave 0), shared through LDS
    auto take = [&]() -> uint32_t {
        if (tid == 0) sm.take = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wg_barrier();
        const uint32_t v = __builtin_amdgcn_readfirstlane(sm.take);
        return v;
    };
    const uint32_t ci0 = take();
    if (ci0 >= ntc) {
        if (tid == 0) arrive(p, blockIdx.x, ep0);
        return;
    }
    // ---- once per workgroup: the first tile's bytes, then the power tables ----------------------
    persist_issue(p, sm, cls, ci0, 0, wave, lane);
    constexpr int kKpWords = 2 * (kPowLo + kPowHi);
    const uint32_t kw = ((const uint32_t *)p.kpow)[tid < kKpWords ? tid : kKpWords - 1];
    const uint32_t iw = ((const uint32_t *)p.cpow)[tid < 2 * kCinv ? tid : 2 * kCinv - 1];
    const uint64_t R = p.cpow[kCinv + tid], RI = p.cpow[kCinv + 256 + tid];   // K^(64 (255 - l)), its inverse
    if (tid < kKpWords) ((uint32_t *)&sm.kp_lo[0])[tid] = kw;   // (these waits drain the first tile too)
    if (tid < 2 * kCinv) ((uint32_t *)&sm.kinv[0])[tid] = iw;
    if (tid == 0) sm.hs[kSlotBefore] = 0ull;
    wg_barrier();
    const int o = tid * 64;   // the lane's chunk: tile bytes [o, o + 64)

    uint32_t nci = take();   // the next tile
    for (uint32_t it = 0, ci = ci0;; ++it) {
        const uint32_t par = it & 1u;
        const bool more = nci < ntc;
        // the next tile's bytes go out before anything of this one is waited for, then the atomic
        // that takes the tile after it (its value is first needed at this iteration's end)
        uint32_t after = ntc;
        if (more) {
            persist_issue(p, sm, cls, nci, par ^ 1u, wave, lane);
            if (tid == 0) after = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (wave == 0) __builtin_amdgcn_s_waitcnt(0x0F76);   // vmcnt(6): this tile's 5 are in
            else __builtin_amdgcn_s_waitcnt(0x0F74);             // vmcnt(4)
        } else {
            __builtin_amdgcn_s_waitcnt(0x0F70);                  // vmcnt(0)
        }
        asm volatile("" ::: "memory");   // no LDS read of this tile above the wait
        uint32_t t = 0;
        const uint32_t bi = batch_of(p, cls, ci, t);
        const BatchDesc &bd = p.b[bi];
        const uint32_t nbytes = bd.nbytes;
        const uint32_t T0 = t * 16384u;
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc((void *)bd.bytes, (short)0, (int)nbytes, 0x00020000);
        uint32_t *const row = &sm.buf[par][tid * 16];
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = *(const uint4 *)&row[4 * k];
        if (T0 + 16384u > nbytes) {
            // the batch's last tile: the 16-byte piece that straddles the end again byte by byte (the
            // range check of a 16-byte load is not byte-exact), into the registers and the image
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t a = T0 + (uint32_t)o + 16u * k;
                if (a < nbytes && a + 16u > nbytes) {
                    v[k] = load16_bytes(rsrc, a);
                    *(uint4 *)&row[4 * k] = v[k];
                }
            }
        }
        const uint64_t sx = __hip_atomic_load(&p.ctl->scan_xcc[bi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

        // ---- the chunk's '\n' / ':' masks and U (Horner of its 64 bytes) from the registers ------
        uint64_t nlm, clm, U;
        {
            uint32_t m[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) m[k] = nl_colon_mask16(v[k]);
            nlm = ((uint64_t)__builtin_amdgcn_perm(m[3], m[2], 0x05040100u) << 32) | __builtin_amdgcn_perm(m[1], m[0], 0x05040100u);
            clm = ((uint64_t)__builtin_amdgcn_perm(m[3], m[2], 0x07060302u) << 32) | __builtin_amdgcn_perm(m[1], m[0], 0x07060302u);
        }

        // ---- line state: three u32 wave scans, the wave totals in LDS ----------------------------
        const uint32_t nrel = nbytes - T0;
        const bool valid = (uint32_t)o < nrel;
        const int lastnl = nlm ? 63 - __clzll(nlm) : -1;
        const uint64_t cafter = lastnl >= 63 ? 0ull : (clm & (~0ull << (lastnl + 1)));
        const uint32_t cand = cafter ? (uint32_t)(o + __builtin_ctzll(cafter)) : (uint32_t)kNone;
        const uint32_t c_in = wave_incl_add32((uint32_t)__popcll(nlm));
        const uint32_t nl_in = wave_incl_max32(nlm ? (uint32_t)(o + lastnl + 1) : 0u);
        const uint32_t k_in = wave_incl_min32(((8191u - c_in) << 17) | cand);
        const uint32_t flags = (__ballot(__popcll(nlm) > 1) ? 1u : 0u) | (__ballot(valid && !(nlm >> 63)) ? 2u : 0u);
        if (lane == 63) *(uint4 *)&sm.wsc[par][wave][0] = make_uint4(c_in, nl_in, k_in, flags);
        wg_barrier();   // B1
        uint32_t tile_count = 0, tflags = 0, tl = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint4 ws = *(const uint4 *)&sm.wsc[par][w][0];
            tile_count += ws.x;
            tflags |= ws.w;
            tl = max(tl, ws.y);
        }
        if (tid == 0) {   // the tile's '\n' count for the scanner
            const uint32_t x = xcc_id();
            const bool same = granule_ok(sx, ep0 & 0x3FFFFFFFu, kFlagXcc) && (uint32_t)sx == x;
            granule_store(&p.status[bd.sbase + t], mk_status(ep0, kFlagAgg, tile_count | ((8u | x) << 28)), same);
        }
        {   // U after the count is out (the scanner's latency is every later tile's)
            U = sdbm_qword_fast(0ull, v[0].x, v[0].y);
            U = sdbm_qword_fast(U, v[0].z, v[0].w);
            U = sdbm_qword_fast(U, v[1].x, v[1].y);
            U = sdbm_qword_fast(U, v[1].z, v[1].w);
            U = sdbm_qword_fast(U, v[2].x, v[2].y);
            U = sdbm_qword_fast(U, v[2].z, v[2].w);
            U = sdbm_qword_fast(U, v[3].x, v[3].y);
            U = sdbm_qword_fast(U, v[3].z, v[3].w);
        }
        const uint64_t *const base_slot = p.bases + bd.sbase + t;
        const bool long_tile = (tflags & 2u) != 0;
        uint32_t p_cnt = 0, p_col = (uint32_t)kNone, p_nl = 0;
#pragma unroll
        for (int w = 0; w < 3; ++w) {
            if (w < wave) {
                const uint4 ws = *(const uint4 *)&sm.wsc[par][w][0];
                p_cnt += ws.x;
                p_nl = max(p_nl, ws.y);
                const uint32_t wc = ws.z & 0x1FFFFu;
                p_col = ws.x ? wc : min(p_col, wc);
            }
        }
        const uint32_t head_nl = t == 0 || (sm.pw[par][0] >> 24) == 0x0Au;   // the byte before the tile is '\n'
        const uint32_t c_ex = wave_shr1_32(c_in, 0u);
        const uint32_t k_ex = wave_shr1_32(k_in, 0xFFFFFFFFu) & 0x1FFFFu;
        const int lf = (int)(p_cnt + c_ex);
        const int ofc = (int)(c_ex ? k_ex : min(p_col, k_ex));
        const int prevnl = (int)max(p_nl, wave_shr1_32(nl_in, 0u));
        const bool before = prevnl == 0 && !head_nl;
        const uint32_t ih = before ? kSlotBefore : (uint32_t)prevnl >> 6;

        const int firstnl = nlm ? __builtin_ctzll(nlm) : 64;
        const uint64_t c0m = clm & (firstnl == 64 ? ~0ull : ((1ull << firstnl) - 1ull));
        const bool ev1 = ofc == kNone && c0m != 0ull;
        const bool has_tail = valid && nlm != 0ull && lastnl < 63;
        const bool ev3 = has_tail && cafter != 0ull;
        auto suf = [&](int q) -> uint64_t {   // Suf(q) = Horner of [q, 64), 0 <= q < 64
            const bool back = q >= 32;
            const uint64_t r = row_horner(row, sm.kp_lo, back ? q : 0, back ? 64 - q : q);
            return back ? r : U - r * sm.kp_lo[(64 - q) & 63];
        };
        uint64_t S1 = 0, S2 = 0, S3 = 0;
        if (__ballot(ev1)) {
            if (ev1) S1 = suf(__builtin_ctzll(c0m));
        }
        if (__ballot(has_tail)) {
            if (has_tail) S2 = suf(lastnl + 1);
            if (ev3) S3 = suf(__builtin_ctzll(cafter));
        }

        // ---- Y and the slots (only when some line crosses a chunk boundary) --------------------
        uint64_t Y = tid == 0 ? U : 0ull;
        if (long_tile) {
            const uint64_t Sw = wave_scan64(U * R, 0ull, [](uint64_t l, uint64_t r) { return l + r; });
            if (lane == 63) sm.wv[wave] = Sw;
            wg_barrier();   // B2
            uint64_t pre = 0;
#pragma unroll
            for (int w = 0; w < 3; ++w)
                if (w < wave) pre += sm.wv[w];
            Y = (Sw + pre) * RI;
            if (ev1 && nlm == 0ull) sm.hc[ih] = Y - S1;
            if (has_tail) {
                sm.hs[tid] = Y - S2;
                if (ev3) sm.hc[tid] = Y - S3;
            } else if (valid && nlm == 0ull && !before && prevnl == o) {
                sm.hs[tid] = Y - U;
            }
            wg_barrier();   // B3
            if (tid == 255 && valid && !(nlm >> 63)) {   // the tile's open line, for the next tile
                const uint32_t cend = c_in ? (k_in & 0x1FFFFu) : min(p_col, k_in & 0x1FFFFu);
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

        // ---- records: the base from the freshest published base + the counts since -------------
        uint32_t base = 0;
        if (t > 0) {
            const uint32_t ep = ep0 & 0x3FFFFFFFu;
            const int c = (int)t - lane;
            const int cc = c - 1;
            bool done = false;
            for (uint32_t spin = 0; spin < (uint32_t)kSpinBudget && !done; ++spin) {
                const uint64_t bg = __hip_atomic_load(&p.bases[bd.sbase + (uint32_t)max(c, 0)], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t cg = __hip_atomic_load(&p.status[bd.sbase + (uint32_t)max(cc, 0)], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
                const bool bok = c == 0 || (c > 0 && granule_ok(bg, ep, kFlagBase));
                const bool cok = cc >= 0 && granule_ok(cg, ep, kFlagAgg);
                const uint64_t okc = __ballot(cok);
                const int nc = ~okc ? __builtin_ctzll(~okc) : 64;
                const uint64_t cand2 = __ballot(bok && lane <= nc);
                if (cand2) {
                    const int l = __builtin_ctzll(cand2);
                    const uint32_t pre = wave_incl_add32(cok ? ((uint32_t)cg & kCountMask) : 0u);
                    base = (uint32_t)__builtin_amdgcn_readlane((int)(c > 0 ? (uint32_t)bg : 0u), l) +
                           (l ? (uint32_t)__builtin_amdgcn_readlane((int)pre, l - 1) : 0u);
                    done = true;
                } else {
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if (!done) base = wait_base(base_slot, ep0, rsrc, T0);
            base = __builtin_amdgcn_readfirstlane(base);
        }
        auto emit = [&](int j, uint32_t off, int len, bool len_ok, bool fmt_ok, uint64_t h) {
            uint32_t route;
            if (!len_ok) route = SR_ROUTE_INVALID_LENGTH;
            else if (!fmt_ok) route = SR_ROUTE_INVALID_FORMAT;
            else route = p.nds ? mod_magic(h, p.magic_n, p.nds) : SR_ROUTE_ALL_DEAD;   // :145, every shard alive
            const uint32_t rec = base + (uint32_t)j;
            if (rec < bd.max_records) {
                sr_record r;
                r.offset = off;
                r.length = len > 0xFFFF ? (uint16_t)0xFFFF : (uint16_t)len;
                r.route = (uint16_t)route;
                bd.recs[rec] = r;
                if (bd.hashes) bd.hashes[rec] = h;
            }
        };
        const int c_first = ofc != kNone ? ofc : (c0m ? o + __builtin_ctzll(c0m) : kNone);
        const int e0 = o + firstnl;
        uint64_t hin0 = 0;
        if (nlm && c_first != kNone && c_first < e0) {
            if (prevnl == o && !before) {
                hin0 = sm.kinv[64 - (c_first & 63)] * (U - S1);
            } else {
                const uint64_t hcv = c_first >= o ? Y - S1 : sm.hc[ih];
                const uint64_t hsv = before ? 0ull : sm.hs[ih];
                const int d = before ? 0 : min((c_first >> 6) - (prevnl >> 6), kPowHi - 1);
                hin0 = sm.kinv[64 - (c_first & 63)] * (hcv - sm.kp_hi[d] * hsv);
            }
        }
        if (nlm && !before) {   // the chunk's first line
            const int len = e0 - prevnl + 1;
            const bool len_ok = len >= (int)SR_MIN_LINE_LENGTH && len <= (int)SR_MAX_LINE_LENGTH;   // :180
            const bool fmt_ok = c_first != kNone && c_first < e0;                                  // :140
            emit(lf, T0 + (uint32_t)prevnl, len, len_ok, fmt_ok, len_ok && fmt_ok ? hin0 : 0ull);
        }
        if (__ballot(__popcll(nlm) > 1)) {   // further lines of a chunk with several '\n'
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
        // ---- the line that began in an earlier tile: its predecessor's tail granules ------------
        const bool lb = nlm != 0ull && before;
        const uint64_t lbm = __ballot(lb);
        if (lbm) {
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
            } else {
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
                uint64_t h = q;
                if (!(meta & kTailColon)) {
                    fmt_ok = c_first != kNone && c_first < e0;
                    h = (len_ok && fmt_ok) ? q * kpow_n(sm, c_first) + hin0 : 0ull;
                }
                if (!(len_ok && fmt_ok)) h = 0;
                emit(lf, s_abs, len, len_ok, fmt_ok, h);
            }
        }
        if (!more) break;
        if (tid == 0) sm.take = after;
        wg_barrier();
        ci = nci;
        nci = __builtin_amdgcn_readfirstlane(sm.take);
    }
    if (tid == 0) arrive(p, blockIdx.x, ep0);
}

}  // namespace srk
