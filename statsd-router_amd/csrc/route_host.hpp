// route_host.hpp — host-side helpers shared by the C ABI (sr_route.hip) and the ablation tool:
// divisor reciprocals, power tables, per-context device state and the launch sequence.
#pragma once

#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <utility>
#include <vector>

#include "chunk_kernel.hpp"

namespace srk {

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (device, kernel) of the process: data
// threads of one executable may run contexts on several devices at once.
inline void ensure_dyn_lds(const void *fn, int bytes) {
    static std::mutex mu;
    static std::vector<std::pair<int, const void *>> done;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    for (const auto &e : done)
        if (e.first == dev && e.second == fn) return;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    done.emplace_back(dev, fn);
}

inline Magic make_magic(uint64_t d) {
    Magic mg{0, 0, 0};
    if (d == 0) return mg;
    const int fl = 63 - __builtin_clzll(d);
    if ((d & (d - 1)) == 0) {
        mg.shift = (uint32_t)fl;
        return mg;
    }
    const unsigned __int128 num = (unsigned __int128)1 << (64 + fl);
    uint64_t pm = (uint64_t)(num / d);
    const uint64_t rem = (uint64_t)(num % d);
    const uint64_t e = d - rem;
    if (e < (1ull << fl)) {
        mg.kind = 1;
    } else {
        pm += pm;
        const uint64_t twice = rem + rem;
        if (twice >= d || twice < rem) pm += 1;
        mg.kind = 2;
    }
    mg.m = pm + 1;
    mg.shift = (uint32_t)fl;
    return mg;
}

inline uint64_t host_div(uint64_t n, const Magic &mg) {
    if (mg.kind == 0) return n >> mg.shift;
    const uint64_t t = (uint64_t)(((unsigned __int128)mg.m * n) >> 64);
    if (mg.kind == 1) return t >> mg.shift;
    return (((n - t) >> 1) + t) >> mg.shift;
}

// Device state owned by one context (one stream at a time).
struct DeviceState {
    uint32_t nds = 0, nwords = 0, dead = 0, max_tiles = 0, pending_cap = 0;
    size_t max_batch = 0;
    Magic magic_n{0, 0, 0};
    Magic magic_n1{0, 0, 0};             // KV_DEAD1: for h % (nds - 1)
    uint32_t dead_k = 0;                 // KV_DEAD1: the dead shard when exactly one is
    uint64_t *h_alive = nullptr;
    uint64_t *d_alive = nullptr;
    Magic *d_magic = nullptr;
    uint64_t *d_kpow = nullptr;
    uint64_t *d_cpow = nullptr;          // route_chunk_kernel's power tables (kCpowEntries)
    uint64_t *d_tail = nullptr;          // route_chunk_kernel's tail granules, 4 per tile
    uint32_t lb_spin = 1u << 16;         // its look-back polls before computing a line itself (SR_KNOB_LB_SPIN)
    uint32_t prefetch = 96;              // SR_KNOB_PREFETCH (RouteParams::prefetch, chunk layout)
    Control *d_ctl = nullptr;
    uint64_t *d_status = nullptr;
    uint64_t *d_bases = nullptr;
    PendingLine *d_pending = nullptr;
    uint64_t *d_tile_pd = nullptr;       // per tile, its probed-dead words (RouteParams::mark)
    uint64_t *d_defer = nullptr;         // hashes of deferred probes by record index, for batches
    size_t defer_cap = 0;                // routed without a hash array (two or more dead shards)
    // lane layout of the route kernel (SR_LAYOUT_*): AUTO follows the segment statistics that
    // KV_SEGMENTS launches publish into host-mapped memory (layout_out), probing now and then
    int layout_mode = 0;
    bool seg_on = false;             // AUTO: mixed-length traffic seen, KV_SEGMENTS launched
    int last_layout = 0;             // the variant of the last launch (SR_LAYOUT_UNIFORM / _SEGMENTS)
    uint32_t seen_seq = 0;
    uint64_t launches = 0;
    uint32_t *h_layout = nullptr;    // pinned, device-mapped: {sequence, tiles weighed, tiles segmented}
    uint32_t *d_layout = nullptr;
    // picks the route kernel makes before deferring a probe (RouteParams::picks) when the deferred
    // probes run anyway (two or more dead shards): 1 (measured: C4 / C5 with 25 % dead 1-2 % faster
    // than 2; with one dead shard nothing is deferred at 2 picks, and deferring a quarter of the
    // lines cost C2 +30 %); SR_KNOB_DEFER_PICKS = 2 overrides (sr_set_knob)
    uint32_t defer_picks = 1;
    uint32_t *d_hist = nullptr;      // RouteParams::hist (sr_route_pack_many), max_tiles x kHistKeys
    bool last_hist = false;          // the last launch wrote its tiles' key histograms
    // fused deferral (route + pack launches, SR_KNOB_FUSE_DEFER, off by default): asked for by the caller, and whether
    // the last launch left its deferred probes to the packing's counting pass (mtu_count_kernel<true>)
    bool fuse_defer = false, last_fused = false;
    // route + pack launches (sr_route_pack_many / _submit): the packing may OR the tiles' probed-dead slots
    // (asked for by the caller), and whether the last launch left them to it (mtu_scan_kernel)
    bool pack_ors_marks = false, last_marks_pending = false;
    uint32_t fd_mark = 0;
    const uint64_t *fd_dhash[kMaxBatches] = {};

    int init(size_t max_batch_bytes, uint32_t n_downstreams) {
        max_batch = max_batch_bytes;
        nds = n_downstreams;
        nwords = (n_downstreams + 63) / 64;
        // status granules for kMaxBatches batches of the smallest tile (256 threads, 16 KiB)
        max_tiles = (uint32_t)(kMaxBatches * ((max_batch_bytes + 16383) / 16384));
        h_alive = (uint64_t *)calloc(nwords ? nwords : 1, sizeof(uint64_t));
        if (!h_alive) return -ENOMEM;
        if (hipMalloc(&d_alive, (nwords ? nwords : 1) * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
        if (hipMalloc(&d_magic, (n_downstreams + 1) * sizeof(Magic)) != hipSuccess) return -ENOMEM;
        if (hipMalloc(&d_kpow, (kPowLo + kPowHi + kPowInv) * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
        if (hipMalloc(&d_cpow, kCpowEntries * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
        if (hipMalloc(&d_tail, (max_tiles ? max_tiles : 1) * 4 * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
        if (hipMemset(d_tail, 0, (max_tiles ? max_tiles : 1) * 4 * sizeof(uint64_t)) != hipSuccess) return -EIO;
        if (hipMalloc(&d_ctl, sizeof(Control)) != hipSuccess) return -ENOMEM;
        if (hipMalloc(&d_status, (max_tiles ? max_tiles : 1) * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
        if (hipMalloc(&d_bases, (max_tiles ? max_tiles : 1) * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
        if (hipMemset(d_bases, 0, (max_tiles ? max_tiles : 1) * sizeof(uint64_t)) != hipSuccess) return -EIO;
        if (hipMemset(d_ctl, 0, sizeof(Control)) != hipSuccess) return -EIO;
        if (hipHostMalloc((void **)&h_layout, 4 * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess) {
            h_layout = nullptr;
            return -ENOMEM;
        }
        memset(h_layout, 0, 4 * sizeof(uint32_t));
        if (hipHostGetDevicePointer((void **)&d_layout, h_layout, 0) != hipSuccess) return -EIO;

        if (hipMemset(d_status, 0, (max_tiles ? max_tiles : 1) * sizeof(uint64_t)) != hipSuccess) return -EIO;
        std::vector<Magic> mg(n_downstreams + 1);
        for (uint32_t d = 1; d <= n_downstreams; ++d) {
            mg[d] = make_magic(d);
            // self-check of the reciprocal against the hardware divide on awkward numerators
            const uint64_t probes[6] = {0ull, 1ull, d - 1ull, (uint64_t)d, ~0ull, 0x9E3779B97F4A7C15ull * d + 7};
            for (uint64_t nn : probes)
                if (host_div(nn, mg[d]) != nn / d) return -EIO;
        }
        magic_n = n_downstreams ? mg[n_downstreams] : Magic{0, 0, 0};
        magic_n1 = n_downstreams >= 2 ? mg[n_downstreams - 1] : Magic{0, 0, 0};
        if (hipMemcpy(d_magic, mg.data(), mg.size() * sizeof(Magic), hipMemcpyHostToDevice) != hipSuccess)
            return -EIO;
        std::vector<uint64_t> kp(kPowLo + kPowHi + kPowInv);
        for (int i = 0; i < kPowLo; ++i) kp[i] = ipow(K, (unsigned)i);
        for (int i = 0; i < kPowHi; ++i) kp[kPowLo + i] = ipow(K, 64u * (unsigned)i);
        for (int z = 0; z < kPowInv; ++z) kp[kPowLo + kPowHi + z] = ipow(kKinv, (unsigned)z);
        if (hipMemcpy(d_kpow, kp.data(), kp.size() * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess)
            return -EIO;
        std::vector<uint64_t> cp(kCpowEntries);
        for (int z = 0; z < kCinv; ++z) cp[z] = ipow(kKinv, (unsigned)z);
        for (int l = 0; l < 256; ++l) {
            cp[kCinv + l] = ipow(K, 64u * (255u - (unsigned)l));
            cp[kCinv + 256 + l] = ipow(kKinv, 64u * (255u - (unsigned)l));
        }
        if (hipMemcpy(d_cpow, cp.data(), cp.size() * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess)
            return -EIO;
        for (uint32_t i = 0; i < n_downstreams; ++i) h_alive[i >> 6] |= 1ull << (i & 63);
        if (hipMemcpy(d_alive, h_alive, (nwords ? nwords : 1) * sizeof(uint64_t), hipMemcpyHostToDevice) !=
            hipSuccess)
            return -EIO;
        dead = 0;
        return 0;
    }

    void release() {
        (void)hipFree(d_alive);
        (void)hipFree(d_magic);
        (void)hipFree(d_kpow);
        (void)hipFree(d_cpow);
        (void)hipFree(d_tail);
        d_cpow = nullptr;
        d_tail = nullptr;
        (void)hipFree(d_ctl);
        (void)hipFree(d_status);
        (void)hipFree(d_bases);
        (void)hipFree(d_pending);
        (void)hipFree(d_defer);
        (void)hipFree(d_tile_pd);
        (void)hipFree(d_hist);
        d_hist = nullptr;
        d_defer = nullptr;
        d_tile_pd = nullptr;
        defer_cap = 0;
        if (h_layout) (void)hipHostFree(h_layout);
        h_layout = nullptr;
        d_layout = nullptr;
        free(h_alive);
        d_alive = nullptr;
        d_magic = nullptr;
        d_kpow = nullptr;
        d_ctl = nullptr;
        d_status = nullptr;
        d_bases = nullptr;
        d_pending = nullptr;
        h_alive = nullptr;
    }

    int set_alive(const uint64_t *alive, hipStream_t stream) {
        // The snapshot's scratch first, so that a failure leaves the context's state as it was
        uint32_t live = 0;
        for (uint32_t w = 0; w < nwords; ++w) {
            uint64_t v = alive[w];
            if (w == nwords - 1 && (nds & 63)) v &= (1ull << (nds & 63)) - 1;
            live += (uint32_t)__builtin_popcountll(v);
        }
        const uint32_t ndead = nds - live;
        if (ndead > (uint32_t)kOverlay && !d_pending) {
            const uint32_t cap = (uint32_t)(max_batch / SR_MIN_LINE_LENGTH + 1);
            if (hipMalloc(&d_pending, (size_t)cap * sizeof(PendingLine)) != hipSuccess) {
                d_pending = nullptr;
                return -ENOMEM;
            }
            pending_cap = cap;
        }
        // two or more dead: the deferred probes keep hashes by record index; sized here for a batch
        // of max_batch bytes (the router's one-batch launches), so that a data thread's launches never
        // reallocate (hipFree / hipMalloc synchronise the device) in the middle of its stream
        if (ndead >= 2 && ndead < nds) {
            const int rc = reserve_defer(max_batch / SR_MIN_LINE_LENGTH + 1);
            if (rc) return rc;
        }
        if (ndead && ndead < nds && nds <= 64 * kAliveLds && !d_tile_pd &&
            hipMalloc(&d_tile_pd, (size_t)(max_tiles ? max_tiles : 1) * nwords * sizeof(uint64_t)) != hipSuccess) {
            d_tile_pd = nullptr;   // the launches replay the probes instead
        }
        for (uint32_t w = 0; w < nwords; ++w) {
            uint64_t v = alive[w];
            if (w == nwords - 1 && (nds & 63)) v &= (1ull << (nds & 63)) - 1;
            h_alive[w] = v;
        }
        dead = ndead;
        dead_k = 0;
        if (ndead == 1)
            for (uint32_t w = 0; w < nwords; ++w) {
                const uint64_t v = h_alive[w] | (w == nwords - 1 && (nds & 63) ? ~0ull << (nds & 63) : 0ull);
                if (~v) {
                    dead_k = 64 * w + (uint32_t)__builtin_ctzll(~v);
                    break;
                }
            }
        const bool copied = !nwords || hipMemcpyAsync(d_alive, h_alive, nwords * sizeof(uint64_t),
                                                      hipMemcpyHostToDevice, stream) == hipSuccess;
        // the copy reads h_alive: complete it before the snapshot can change again (also after a
        // failed enqueue, so that nothing can still be reading h_alive)
        const bool synced = hipStreamSynchronize(stream) == hipSuccess;
        return copied && synced ? 0 : -EIO;
    }

    int reserve_defer(size_t entries) {
        if (entries <= defer_cap) return 0;
        (void)hipFree(d_defer);
        d_defer = nullptr;
        defer_cap = 0;
        if (hipMalloc(&d_defer, entries * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
        defer_cap = entries;
        return 0;
    }

    // launch parameters without batches (add them with add_batch)
    RouteParams params() const {
        RouteParams p;
        memset(&p, 0, sizeof(p));
        p.nds = nds;
        p.dead = dead;
        p.pending_cap = pending_cap;
        p.magic_n = magic_n;
        p.alive = d_alive;
        p.magic = d_magic;
        p.kpow = d_kpow;
        p.ctl = d_ctl;
        p.status = d_status;
        p.bases = d_bases;
        p.pending = d_pending;
        p.tile_pd = d_tile_pd;
        p.dbg = nullptr;
        p.layout_out = d_layout;
        p.cpow = d_cpow;
        p.tail = d_tail;
        p.lb_spin = lb_spin;
        p.prefetch = prefetch;
        p.alive_w0 = h_alive ? h_alive[0] : 0ull;
        p.magic_n1 = magic_n1;
        p.dead_k = dead_k;
        return p;
    }

    // The route kernel variant for the next launch. AUTO: switch to the chunk layout when at least
    // a quarter of the tiles a KV_SEGMENTS launch weighed took the segment layout, back below a
    // tenth; every 32nd launch outside stream capture is a KV_SEGMENTS probe that weighs the
    // traffic (the first launch is one). Records are identical either way; only the time differs.
    bool choose_segments(hipStream_t stream) {
        bool seg;
        if (layout_mode == SR_LAYOUT_CHUNKS) {
            last_layout = SR_LAYOUT_CHUNKS;
            return false;
        }
        if (layout_mode == SR_LAYOUT_UNIFORM) {
            seg = false;
        } else if (layout_mode == SR_LAYOUT_SEGMENTS) {
            seg = true;
        } else {
            const uint32_t seq = __atomic_load_n(&h_layout[0], __ATOMIC_ACQUIRE);
            if (seq != seen_seq) {
                seen_seq = seq;
                const uint32_t weighed = __atomic_load_n(&h_layout[1], __ATOMIC_RELAXED);
                const uint32_t segmented = __atomic_load_n(&h_layout[2], __ATOMIC_RELAXED);
                if (!seg_on && 4ull * segmented >= weighed) seg_on = true;
                else if (seg_on && 10ull * segmented < weighed) seg_on = false;
            }
            hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
            const bool capturing = hipStreamIsCapturing(stream, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
            const bool probe = !capturing && launches % 32 == 0;
            if (!capturing) ++launches;
            // mixed traffic goes to the chunk layout; the probes keep weighing it with KV_SEGMENTS
            if (seg_on && !probe) {
                last_layout = SR_LAYOUT_CHUNKS;
                return false;
            }
            seg = probe;
        }
        last_layout = seg ? SR_LAYOUT_SEGMENTS : SR_LAYOUT_UNIFORM;
        return seg;
    }

    // one-batch launch parameters
    RouteParams params(const uint8_t *d_bytes, size_t nbytes, sr_record *d_out, size_t max_records,
                       uint64_t *d_hashes, uint64_t *d_n) const {
        RouteParams p = params();
        add_batch(p, d_bytes, nbytes, d_out, max_records, d_hashes, d_n);
        return p;
    }

    static bool add_batch(RouteParams &p, const uint8_t *d_bytes, size_t nbytes, sr_record *d_out,
                          size_t max_records, uint64_t *d_hashes, uint64_t *d_n, uint64_t *d_probed_dead = nullptr) {
        if (p.nb >= (uint32_t)kMaxBatches) return false;
        BatchDesc &b = p.b[p.nb++];
        b.bytes = d_bytes;
        b.nbytes = (uint32_t)nbytes;
        b.recs = d_out;
        b.hashes = d_hashes;
        b.n_out = d_n;
        b.max_records = (uint32_t)(max_records > 0xFFFFFFFFull ? 0xFFFFFFFFull : max_records);
        b.tile0 = b.ntiles = b.sbase = b.cls = b.pad = 0;
        b.probed_dead = d_probed_dead;
        b.dhash = nullptr;
        return true;
    }

    bool wide() const { return dead > (uint32_t)kOverlay && dead < nds; }
    // the probes note the dead shards they visit themselves (RouteParams::mark); otherwise a replay
    // after the launch does (probed_dead_kernel), from the route kernel's hashes when it wrote them
    bool marks_in_kernel() const { return dead && dead < nds && nds <= 64 * kAliveLds && d_tile_pd; }
    bool replay_wants_hashes() const { return dead && dead < nds && !marks_in_kernel(); }
};

// Launch the route kernel over the batches of p (tile ranges assigned here; empty batches get a
// zero line count without a kernel). With more than kOverlay dead shards every batch is launched
// on its own so that the deferred-probe list holds one batch at a time.
template <int BLOCK, unsigned ABL>
inline int launch_route(DeviceState &ds, const RouteParams &in, hipStream_t stream) {
    constexpr uint64_t T = (uint64_t)BLOCK * kLaneBytes;
    if (ds.wide() && in.nb > 1) {
        for (uint32_t i = 0; i < in.nb; ++i) {
            RouteParams one = in;
            one.nb = 1;
            one.b[0] = in.b[i];
            const int rc = launch_route<BLOCK, ABL>(ds, one, stream);
            if (rc) return rc;
        }
        return 0;
    }
    RouteParams p = in;
    p.nb = 0;
    bool replay = false;   // some batch asked for the probed-dead bitmap (probed_dead_kernel)
    p.nwords = ds.nwords;
    for (uint32_t i = 0; i < in.nb; ++i) {
        if (in.b[i].nbytes == 0) {   // no tile, no scanner: its count and bitmap are set here
            if (hipMemsetAsync(in.b[i].n_out, 0, sizeof(uint64_t), stream) != hipSuccess) return -EIO;
            if (in.b[i].probed_dead &&
                hipMemsetAsync(in.b[i].probed_dead, 0, (size_t)(ds.nwords ? ds.nwords : 1) * sizeof(uint64_t),
                               stream) != hipSuccess)
                return -EIO;
            continue;
        }
        // the batch's scanner zeroes its bitmap; with every shard alive nothing sets it afterwards
        p.b[p.nb++] = in.b[i];
        if (ds.dead && p.b[p.nb - 1].probed_dead) replay = true;
    }
    if (p.nb == 0) return 0;
    // 8+ batches: each batch's tiles on one XCD class; its scanner (block j) shares that class
    const bool xl = !(ABL & ABL_NO_XCD_LOCAL) && p.nb >= 8;
    p.xcd_local = xl ? 1u : 0u;
    uint32_t cls_tiles[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t sb = 0;
    for (uint32_t j = 0; j < p.nb; ++j) {
        BatchDesc &d = p.b[j];
        d.ntiles = (uint32_t)((d.nbytes + T - 1) / T);
        d.sbase = sb;
        sb += d.ntiles;
        d.cls = xl ? (j + 7u * p.nb) % 8u : 0u;   // (nb + cls) % 8 == j % 8
        d.tile0 = cls_tiles[d.cls];
        cls_tiles[d.cls] += d.ntiles;
    }
    if (sb > ds.max_tiles) return -EINVAL;
    // The class table dealt by block index (launch_header_batch in route_kernel.hpp): row r serves the
    // blocks B = nb + g = r (mod 8); entry = (the first B / 8 past batch j's tiles) << 6 | j. 8+ batches:
    // row r is class (r - nb) mod 8, whose tile ci runs on block B = nb + 8 ci + class, so B / 8 =
    // ci + ceil((nb - r) / 8). Fewer: every row holds every batch, tile g on block nb + g, and
    // g >= end <=> B / 8 >= ceil((end + nb - r) / 8).
    for (int c = 0; c < 8; ++c)
        for (int k = 0; k < kPerClass; ++k) p.cls_tab[c][k] = ~0u;
    {
        int fill[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint32_t j = 0; j < p.nb; ++j) {   // j ascending = tile0 ascending within a class
            const BatchDesc &d = p.b[j];
            const uint32_t end = d.tile0 + d.ntiles;
            for (uint32_t r = 0; r < 8; ++r) {
                uint32_t thr;
                if (xl) {
                    if (((r + 8u - p.nb % 8u) & 7u) != d.cls) continue;
                    thr = end + (p.nb - r + 7u) / 8u;   // nb >= 8 > r
                } else {
                    const int64_t v = (int64_t)end + p.nb - r;
                    thr = v <= 0 ? 0u : (uint32_t)((v + 7) / 8);
                }
                if (fill[r] >= kPerClass || thr >= (1u << 26)) return -EINVAL;
                p.cls_tab[r][fill[r]++] = (thr << 6) | j;
            }
        }
    }
    uint32_t grid_tiles = cls_tiles[0];
    if (xl) {
        uint32_t mx = 0;
        for (int c = 0; c < 8; ++c) mx = cls_tiles[c] > mx ? cls_tiles[c] : mx;
        grid_tiles = 8 * mx;
    }
    p.total_blocks = p.nb + grid_tiles;   // scanners first, then the tiles
    // Two or more dead shards: probes past their first pick are deferred to probe_defer_kernel,
    // the record marked pending and the hash kept by record index (in the batch's hash array, or else
    // in the context's scratch, grown outside stream capture; a launch that cannot have the scratch
    // runs every probe in the route kernel).
    p.defer = 0;
    p.picks = ds.dead >= 2 ? ds.defer_picks : 2u;
    // some shards dead (not all), at most 1024: the tiles note the dead shards their probes visit
    // (MARK_LDS in route_kernel.hpp), probe_defer_kernel and probe_wide_kernel theirs; no replay
    p.mark = (replay && ds.marks_in_kernel()) ? 1u : 0u;
    uint32_t max_recs = 0;
    if (ds.dead >= 2 && ds.dead < ds.nds) {
        uint64_t need = 0;
        for (uint32_t j = 0; j < p.nb; ++j) {
            if (!p.b[j].hashes) need += p.b[j].max_records;
            max_recs = p.b[j].max_records > max_recs ? p.b[j].max_records : max_recs;
        }
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        const bool capturing = hipStreamIsCapturing(stream, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
        if (need == 0 || need <= ds.defer_cap || (!capturing && ds.reserve_defer(need) == 0)) {
            p.defer = 1;
            uint64_t off = 0;
            for (uint32_t j = 0; j < p.nb; ++j) {
                if (p.b[j].hashes) {
                    p.b[j].dhash = p.b[j].hashes;
                } else {
                    p.b[j].dhash = ds.d_defer + off;
                    off += p.b[j].max_records;
                }
            }
        }
    }
    // one pick before deferring: every probe that meets a dead shard is deferred and redone whole by
    // probe_defer_kernel, which notes the dead shards it visits; the route kernel need not
    p.mark_tiles = (p.mark && !(p.defer && p.picks == 1)) ? 1u : 0u;
    if (ds.wide() && hipMemsetAsync(&ds.d_ctl->pending, 0, sizeof(uint32_t), stream) != hipSuccess) return -EIO;
    // Route + pack with every dead first pick deferred and at most kOverlay dead (no wide probes), at most
    // 1024 shards: the packing's counting pass runs the deferred probes (no probe_defer_kernel)
    const bool fused = ds.fuse_defer && p.defer && p.picks == 1 && !p.mark_tiles && ds.dead <= (uint32_t)kOverlay &&
                       ds.nwords <= kReplayCheckWords && (p.mark || !replay);
    ds.last_fused = fused;
    if (fused) {
        ds.fd_mark = p.mark;
        for (uint32_t j = 0; j < p.nb; ++j) ds.fd_dhash[j] = p.b[j].dhash;
    }
    // KV_DEFER1 (route_kernel.hpp): two or more of at most 64 shards dead, every dead first pick deferred
    const bool defer1 = !(ABL & KV_ALIVE) && ds.dead >= 2 && ds.dead < ds.nds && ds.nds <= 64 && p.defer &&
                        p.picks == 1 && !p.mark_tiles;
    constexpr unsigned kD1 = (ABL & KV_ALIVE) ? ABL : (ABL | KV_DEFER1);
    // KV_DEAD1: exactly one dead shard (two picks end every probe)
    const bool dead1 = !(ABL & KV_ALIVE) && ds.dead == 1 && ds.nds >= 2;
    constexpr unsigned kK1 = (ABL & KV_ALIVE) ? ABL : (ABL | KV_DEAD1);
    // A route + pack launch with one dead shard (KV_DEAD1 | KV_HIST1, nothing deferred): the packing's
    // mtu_scan_kernel ORs the tiles' probed-dead slots into the bitmaps (pack_ors_marks); no
    // probe_defer_kernel (7.2 us per C2 launch for that OR alone)
    const bool slots_to_pack = ds.pack_ors_marks && dead1 && p.mark_tiles && p.hist && (ABL & KV_PICKS) != 0 &&
                               !(ABL & KV_CHUNKS);
    ds.last_marks_pending = slots_to_pack;
    if constexpr ((ABL & KV_CHUNKS) != 0) {
        static_assert(BLOCK == 256, "route_chunk_kernel: 256 lanes of 64 bytes per 16 KiB tile");
        // its probe stops after the first picks: with two or more dead shards it needs the deferral
        // (no scratch for it, e.g. inside a stream capture: the uniform kernel probes in full)
        if (ds.dead >= 2 && ds.dead < ds.nds && !p.defer)
            hipLaunchKernelGGL((route_kernel<BLOCK, KV_UNIFORM>), dim3(p.total_blocks), dim3(BLOCK), 0, stream, p);
        else if (defer1)
            hipLaunchKernelGGL((route_chunk_kernel<kD1>), dim3(p.total_blocks), dim3(256), 0, stream, p);
        else if (dead1)
            hipLaunchKernelGGL((route_chunk_kernel<kK1>), dim3(p.total_blocks), dim3(256), 0, stream, p);
        else
            hipLaunchKernelGGL((route_chunk_kernel<ABL>), dim3(p.total_blocks), dim3(256), 0, stream, p);
    } else if constexpr ((ABL & KV_PICKS) != 0) {
        // the picks-only variant needs the deferral once two or more shards are dead
        if (ds.dead >= 2 && ds.dead < ds.nds && !p.defer)
            hipLaunchKernelGGL((route_kernel<BLOCK, (ABL & ~KV_PICKS)>), dim3(p.total_blocks), dim3(BLOCK), 0, stream, p);
        else if (defer1)
            hipLaunchKernelGGL((route_kernel<BLOCK, kD1>), dim3(p.total_blocks), dim3(BLOCK), 0, stream, p);
        else if (dead1 && p.hist)
            hipLaunchKernelGGL((route_kernel<BLOCK, kK1 | KV_HIST1>), dim3(p.total_blocks), dim3(BLOCK), 0, stream, p);
        else if (dead1)
            hipLaunchKernelGGL((route_kernel<BLOCK, kK1>), dim3(p.total_blocks), dim3(BLOCK), 0, stream, p);
        else
            hipLaunchKernelGGL((route_kernel<BLOCK, ABL>), dim3(p.total_blocks), dim3(BLOCK), 0, stream, p);
    } else {
        hipLaunchKernelGGL((route_kernel<BLOCK, ABL>), dim3(p.total_blocks), dim3(BLOCK), 0, stream, p);
    }
    if (hipGetLastError() != hipSuccess) return -EIO;
    // the key histograms exist only where route_kernel counted them: every shard alive, or exactly one
    // dead (KV_DEAD1: two picks end every probe in the kernel). (Counting them in the general picks-only
    // variant cost it 5 us per C2 launch in SGPR spills: profiles/r05/hist_one_dead_ab_r5h.jsonl.)
    ds.last_hist = p.hist && !(ABL & KV_CHUNKS) && ((ABL & KV_ALIVE) || ((ABL & KV_PICKS) && dead1));
    if ((p.defer || p.mark) && !fused && !slots_to_pack) {   // the probes past their first two picks and the OR of the tiles' probed-dead
                               // slots (probe_defer_kernel), grid y = batch
        // blocks past a batch's record count return at once; the rest loop over chunks of 4 waves
        const uint32_t bx = p.defer ? (max_recs + 4u * kDeferChunk - 1u) / (4u * kDeferChunk) : 1u;
        const dim3 grid(bx ? (bx < 128u ? bx : 128u) : 1u, p.nb);
        if (ds.dead <= 4) hipLaunchKernelGGL(probe_defer_kernel<4>, grid, dim3(256), 0, stream, p);
        else if (ds.dead <= 8) hipLaunchKernelGGL(probe_defer_kernel<8>, grid, dim3(256), 0, stream, p);
        else hipLaunchKernelGGL(probe_defer_kernel<kOverlay>, grid, dim3(256), 0, stream, p);
        if (hipGetLastError() != hipSuccess) return -EIO;
    }
    if (ds.wide()) {
        ensure_dyn_lds((const void *)probe_wide_kernel, 160 * 1024);
        hipLaunchKernelGGL(probe_wide_kernel, dim3(256), dim3(64), (size_t)ds.nds * sizeof(uint16_t), stream, p);
        if (hipGetLastError() != hipSuccess) return -EIO;
    }
    if (replay && !p.mark) {   // dead shards and a bitmap asked for: replay the probes (sr-main.c:106)
        p.nwords_check = ds.nwords <= kReplayCheckWords ? ds.nwords : 0u;
        hipLaunchKernelGGL(probed_dead_kernel, dim3(kReplayBlocks, p.nb), dim3(256), 0, stream, p);
        if (hipGetLastError() != hipSuccess) return -EIO;
    }
    return 0;
}

}  // namespace srk
