// sr_route.hip — the C ABI of include/sr_route.h on MI355X (gfx950).
//
// Device code: route_kernel.hpp (one pass per batch: tokenise, validate, sdbm name hash, shard
// pick; reference sr-main.c:86-191). Host helpers: route_host.hpp. This file only adds the
// exported entry points, their argument checking and the host<->device copies of the
// host-memory variant.

#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <new>

#include "../../include/sr_route.h"
#include "exchange.hpp"
#include "mtu_kernel.hpp"
#include "regroup_kernel.hpp"
#include "route_host.hpp"

using namespace srk;

struct sr_ctx {
    int device;
    hipStream_t own_stream;
    hipStream_t stream;
    DeviceState ds;
    // buffers of the host-memory path (sr_route_batch)
    uint8_t *d_in;
    sr_record *d_out;
    size_t d_out_cap;
    uint64_t *d_hash;
    size_t d_hash_cap;
    uint64_t *d_count;
    uint64_t *d_probed;           // probed-dead bitmap of the host-memory path
    uint64_t *h_probed;           // its copy after the last sr_route_batch
    // scratch of sr_pack_by_owner
    uint2 *d_pack_tiles;          // tile counts | tile bases
    size_t pack_tiles_cap;        // entries per array
    uint64_t *d_owner_start;
    // scratch of sr_pack_packets (capacities: record tiles, chunks)
    uint32_t mtu_ntiles, mtu_chunks;
    uint32_t *d_mtu_tiles, *d_mtu_keys, *d_mtu_chunks;
    uint64_t *d_mtu_table;
    uint32_t *d_mtu_gp;    // per chunk: bytes per packet start (kMtuChunk u16), then the first prefix sums
    // sr_pack_owner_sizes / sr_pack_owner_scatter: the split sizes of the pack in progress, and where its
    // scatter wrote owner `own`'s chunk (sr_exchange_data then skips that chunk's copy)
    uint64_t *own_counts;
    uint64_t own_shape;   // key of that pack's batches and owners (pack_shape; the scatter must match)
    int own_set, own;
    uint8_t *own_bytes;
    sr_record *own_recs;
    // buffers of sr_route_pack_batch
    sr_record *d_sorted;
    size_t d_sorted_cap;
    sr_packet *d_packets;
    size_t d_packets_cap;
    uint16_t *d_fill;             // [3][nds]: two chained outputs, then the uploaded fill of a submission
    int fill_cur;                 // region of d_fill holding the last submission's output (0 or 1)
    uint64_t *d_mcounts;          // 3 u64
    int trace;                    // sr_set_trace: submissions also return input-order records + hashes
    // packing knobs (sr_set_knob): forced chunk lines (0: by shape), XCD-local chunks, chain walked in emit
    uint32_t mtu_chunk;
    int mtu_xcd, mtu_walk;
    int hist;                     // SR_KNOB_HIST: route + pack launches hand the tiles' histograms over
    int fuse_defer;               // SR_KNOB_FUSE_DEFER: the counting pass runs the route launch's deferred probes
    // page-locked, device-mapped outputs of sr_route_pack_submit: slots 0 and 1, slot 2 is
    // sr_route_pack_batch's own
    struct Slot {
        uint8_t *host;            // one allocation: records | packets | fill out | probed | counts | fill in
        uint8_t *dev;             // its device-mapped address
        size_t rec_cap, pk_cap;
        hipEvent_t done;
        int busy;                 // submitted, result not taken
        sr_record *sorted;
        sr_packet *packets;
        uint16_t *fill, *fill_in;
        uint64_t *probed, *counts;
        // sr_set_trace: input-order records and per-line hashes (one more page-locked allocation)
        uint8_t *thost, *tdev;
        size_t trec_cap;
        int traced;               // the batch in the slot was submitted with trace on
    } slot[3];
};

static void free_ptr(void *p) { (void)hipFree(p); }

#ifndef SR_CHUNK_ABL
#define SR_CHUNK_ABL 0u   // developer ablation builds of route_chunk_kernel only (chunk_kernel.hpp)
#endif

// The product launches KV_UNIFORM, KV_SEGMENTS or KV_CHUNKS (identical records;
// DeviceState::choose_segments picks by the lane-layout policy). Ablation variants (records wrong by design in some of them)
// exist only in builds made with -DSR_ABLATION_VARIANTS (`make VARIANTS=1`, developer A/B runs;
// never the shipped library): SR_VARIANT in the environment then selects one.
static int launch_product(DeviceState &ds, const RouteParams &p, hipStream_t stream) {
    const bool seg = ds.choose_segments(stream);
    if (ds.last_layout == SR_LAYOUT_CHUNKS) {
        if (ds.dead == 0) return launch_route<kBlock, KV_CHUNKS | KV_ALIVE | SR_CHUNK_ABL>(ds, p, stream);
        return launch_route<kBlock, KV_CHUNKS | SR_CHUNK_ABL>(ds, p, stream);
    }
    if (ds.dead == 0) {   // every shard alive: the variants without the probe
        if (seg) return launch_route<kBlock, KV_SEGMENTS | KV_ALIVE>(ds, p, stream);
        return launch_route<kBlock, KV_UNIFORM | KV_ALIVE>(ds, p, stream);
    }
    if (seg) return launch_route<kBlock, KV_SEGMENTS | KV_PICKS>(ds, p, stream);
    return launch_route<kBlock, KV_UNIFORM | KV_PICKS>(ds, p, stream);
}
#ifdef SR_ABLATION_VARIANTS
static int launch_variant(DeviceState &ds, const RouteParams &p, hipStream_t stream) {
    static const int v = [] {
        const char *e = getenv("SR_VARIANT");
        if (!e || !*e) return 0;
        if (!strcmp(e, "no_mid_base")) return 14;
        // upper bounds, not routing (records wrong or missing; line counts still exact)
        if (!strcmp(e, "fake_base")) return 7;
        if (!strcmp(e, "no_hash")) return 8;
        if (!strcmp(e, "no_lines")) return 9;
        return 0;
    }();
    switch (v) {
    case 14: return launch_route<kBlock, ABL_NO_MID_BASE>(ds, p, stream);
    case 7: return launch_route<kBlock, ABL_FAKE_BASE>(ds, p, stream);
    case 8: return launch_route<kBlock, ABL_NO_HASH>(ds, p, stream);
    case 9: return launch_route<kBlock, ABL_NO_LINES>(ds, p, stream);
    default: return launch_product(ds, p, stream);
    }
}
#else
static int launch_variant(DeviceState &ds, const RouteParams &p, hipStream_t stream) {
    return launch_product(ds, p, stream);
}
#endif

extern "C" {

size_t sr_frame_datagram(uint8_t *dst, const uint8_t *src, size_t len) {
    // udp_read_cb: recv(fd, buffer, DATA_BUF_SIZE - 1, 0) (sr-main.c:163), then append '\n'
    // unless the datagram already ends with one (sr-main.c:171-173). Empty -> nothing (:170).
    size_t n = len < SR_MAX_DATAGRAM ? len : SR_MAX_DATAGRAM;
    if (n == 0) return 0;
    memcpy(dst, src, n);
    if (dst[n - 1] != '\n') dst[n++] = '\n';
    return n;
}

size_t sr_frame_datagrams(uint8_t *dst, size_t dst_cap, const uint8_t *const *dgrams, const size_t *lens,
                          size_t count) {
    size_t pos = 0;
    for (size_t i = 0; i < count; ++i) {
        const size_t need = (lens[i] < SR_MAX_DATAGRAM ? lens[i] : SR_MAX_DATAGRAM) + 1;
        if (pos + need > dst_cap) return (size_t)-1;
        pos += sr_frame_datagram(dst + pos, dgrams[i], lens[i]);
    }
    return pos;
}

void *sr_alloc_host(size_t bytes) {
    void *p = nullptr;
    return hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}

void sr_free_host(void *p) {
    if (p) (void)hipHostFree(p);
}

const char *sr_version(void) {
    return "statsd-router-mi355x 0.5 (gfx950 route_kernel: 16 KiB tiles x 256 threads, per-batch scanners, up to 32 batches per launch)";
}

void sr_close(sr_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->ds.release();
    (void)hipFree(c->d_in);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_hash);
    (void)hipFree(c->d_count);
    (void)hipFree(c->d_probed);
    free(c->h_probed);
    (void)hipFree(c->d_pack_tiles);
    (void)hipFree(c->d_owner_start);
    free_ptr(c->d_mtu_tiles);
    free_ptr(c->d_mtu_keys);
    free_ptr(c->d_mtu_chunks);
    free_ptr(c->d_mtu_table);
    free_ptr(c->d_mtu_gp);
    free_ptr(c->d_sorted);
    free_ptr(c->d_packets);
    free_ptr(c->d_fill);
    free_ptr(c->d_mcounts);
    for (auto &sl : c->slot) {
        if (sl.host) (void)hipHostFree(sl.host);
        if (sl.thost) (void)hipHostFree(sl.thost);
        if (sl.done) (void)hipEventDestroy(sl.done);
    }
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    free(c);
}

int sr_open(sr_ctx **out, int device, size_t max_batch_bytes, uint32_t n_downstreams) {
    if (!out) return -EINVAL;
    *out = nullptr;
    if (max_batch_bytes == 0 || max_batch_bytes > 0xFFFFFFF0ull || n_downstreams > SR_MAX_DOWNSTREAMS)
        return -EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return -ENODEV;
    if (hipSetDevice(device) != hipSuccess) return -ENODEV;
    sr_ctx *c = (sr_ctx *)calloc(1, sizeof(sr_ctx));
    if (!c) return -ENOMEM;
    new (&c->ds) DeviceState();
    c->device = device;
    c->mtu_xcd = 1;
    c->mtu_walk = 1;
    c->hist = 1;
    c->fuse_defer = 0;   // measured level or slower (C4: too few counting waves): profiles/r05/fused_deferral_ab_r5r.jsonl
    int rc = -ENOMEM;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) goto fail;
    c->stream = c->own_stream;
    if ((rc = c->ds.init(max_batch_bytes, n_downstreams)) != 0) goto fail;
    rc = -ENOMEM;
    if (hipMalloc(&c->d_in, max_batch_bytes) != hipSuccess) goto fail;
    if (hipMalloc(&c->d_count, sizeof(uint64_t)) != hipSuccess) goto fail;
    if (hipMalloc(&c->d_probed, (c->ds.nwords ? c->ds.nwords : 1) * sizeof(uint64_t)) != hipSuccess) goto fail;
    if (!(c->h_probed = (uint64_t *)calloc(c->ds.nwords ? c->ds.nwords : 1, sizeof(uint64_t)))) goto fail;
    *out = c;
    return 0;
fail:
    sr_close(c);
    return rc;
}

int sr_set_alive(sr_ctx *c, const uint64_t *alive) {
    if (!c || (!alive && c->ds.nds)) return -EINVAL;
    (void)hipSetDevice(c->device);
    return c->ds.set_alive(alive, c->stream);
}

int sr_set_stream(sr_ctx *c, void *stream) {
    if (!c) return -EINVAL;
    c->stream = stream ? (hipStream_t)stream : c->own_stream;
    return 0;
}

int sr_set_layout(sr_ctx *c, int layout) {
    if (!c || layout < SR_LAYOUT_AUTO || layout > SR_LAYOUT_CHUNKS) return -EINVAL;
    c->ds.layout_mode = layout;
    return 0;
}

int sr_last_layout(const sr_ctx *c) { return c ? c->ds.last_layout : -EINVAL; }

int sr_set_knob(sr_ctx *c, int knob, int64_t v) {
    if (!c) return -EINVAL;
    switch (knob) {
    case SR_KNOB_LB_SPIN:
        if (v < 0 || v > 0xFFFFFFFFll) return -EINVAL;
        c->ds.lb_spin = (uint32_t)v;
        return 0;
    case SR_KNOB_FUSE_DEFER:
        if (v != 0 && v != 1) return -EINVAL;
        c->fuse_defer = (int)v;
        return 0;
    case SR_KNOB_PREFETCH:
        if (v < 0 || v > 4096) return -EINVAL;
        c->ds.prefetch = (uint32_t)v;
        return 0;
    case SR_KNOB_DEFER_PICKS:
        if (v != 1 && v != 2) return -EINVAL;
        c->ds.defer_picks = (uint32_t)v;
        return 0;
    case SR_KNOB_MTU_CHUNK:
        if (v != 0 && v != kMtuChunkSmall && v != kMtuChunk) return -EINVAL;
        c->mtu_chunk = (uint32_t)v;
        return 0;
    case SR_KNOB_MTU_XCD:
    case SR_KNOB_MTU_WALK:
    case SR_KNOB_HIST:
        if (v != 0 && v != 1) return -EINVAL;
        (knob == SR_KNOB_MTU_XCD ? c->mtu_xcd : knob == SR_KNOB_MTU_WALK ? c->mtu_walk : c->hist) = (int)v;
        return 0;
    default:
        return -EINVAL;
    }
}

int sr_set_trace(sr_ctx *c, int on) {
    if (!c) return -EINVAL;
    c->trace = on ? 1 : 0;
    return 0;
}

int sr_sync(sr_ctx *c) {
    if (!c) return -EINVAL;
    (void)hipSetDevice(c->device);
    return hipStreamSynchronize(c->stream) == hipSuccess ? 0 : -EIO;
}

int sr_last_probed_dead(const sr_ctx *c, uint64_t *bitmap) {
    if (!c || (!bitmap && c->ds.nwords)) return -EINVAL;
    if (c->ds.nwords) memcpy(bitmap, c->h_probed, c->ds.nwords * sizeof(uint64_t));
    return 0;
}

int sr_route_device(sr_ctx *c, const uint8_t *d_bytes, size_t nbytes, sr_record *d_out, size_t max_records,
                    uint64_t *d_hashes, uint64_t *d_n_records) {
    if (!c || !d_n_records || (nbytes && !d_bytes) || nbytes > c->ds.max_batch) return -EINVAL;
    if (max_records && !d_out) return -EINVAL;
    (void)hipSetDevice(c->device);
    const RouteParams p = c->ds.params(d_bytes, nbytes, d_out, max_records, d_hashes, d_n_records);
    return launch_variant(c->ds, p, c->stream);
}

int sr_route_device_many(sr_ctx *c, const sr_batch *batches, size_t count) {
    static_assert(SR_MAX_BATCHES_PER_LAUNCH == (unsigned)kMaxBatches, "launch batch limit");
    if (!c || (count && !batches)) return -EINVAL;
    for (size_t i = 0; i < count; ++i) {
        const sr_batch &b = batches[i];
        if (!b.d_n_records || (b.nbytes && !b.d_bytes) || b.nbytes > c->ds.max_batch) return -EINVAL;
        if (b.max_records && !b.d_out) return -EINVAL;
    }
    (void)hipSetDevice(c->device);
    for (size_t i0 = 0; i0 < count; i0 += kMaxBatches) {
        RouteParams p = c->ds.params();
        for (size_t i = i0; i < count && i < i0 + kMaxBatches; ++i)
            DeviceState::add_batch(p, batches[i].d_bytes, batches[i].nbytes, batches[i].d_out, batches[i].max_records,
                                   batches[i].d_hashes, batches[i].d_n_records, batches[i].d_probed_dead);
        const int rc = launch_variant(c->ds, p, c->stream);
        if (rc) return rc;
    }
    return 0;
}

// The owner pack's tile: 256 records per chunk, two chunks per tile when the pack's lines are short,
// one when they are long (more than 192 bytes per record slot on average: C5's mixed lines, C3, C4).
// Every call with the same batches picks the same (sr_pack_owner_sizes and _scatter share the tiles).
static int pack_chunks_for(const PackBatch *in, uint32_t nb) {
    uint64_t bytes = 0, recs = 0;
    for (uint32_t j = 0; j < nb; ++j) {
        bytes += in[j].nbytes;
        recs += in[j].max_records;
    }
    return bytes > 192ull * (recs ? recs : 1) ? 1 : kPackMaxChunks;
}

// The owner pack: kPackSizes = count + scan (the split sizes into d_owner_counts), kPackScatter =
// the lines and records (owner `own` into own_bytes / own_recs when own >= 0)
enum : int { kPackSizes = 1, kPackScatter = 2 };
static int pack_launch(sr_ctx *c, const PackBatch *in, uint32_t nb, uint32_t n_owners, uint8_t *d_out_bytes,
                       size_t out_cap, sr_record *d_out_recs, uint64_t *d_owner_counts, int phases = kPackSizes | kPackScatter,
                       int own = -1, uint8_t *own_bytes = nullptr, sr_record *own_recs = nullptr) {
    PackParams p;
    memset(&p, 0, sizeof(p));
    const int ch = pack_chunks_for(in, nb);
    const uint32_t tile = (uint32_t)(kPackBlock * ch);
    uint32_t ntiles = 0;
    for (uint32_t j = 0; j < nb; ++j) {
        p.b[j] = in[j];
        p.b[j].tile0 = ntiles;
        ntiles += (in[j].max_records + tile - 1) / tile;
    }
    p.nb = nb ? nb : 1;
    p.n_owners = n_owners;
    p.ntiles = ntiles;
    const size_t need = (size_t)(ntiles ? ntiles : 1) * n_owners;
    if (need > c->pack_tiles_cap) {
        (void)hipFree(c->d_pack_tiles);
        c->d_pack_tiles = nullptr;
        c->pack_tiles_cap = 0;
        if (hipMalloc(&c->d_pack_tiles, 2 * need * sizeof(uint2)) != hipSuccess) return -ENOMEM;
        c->pack_tiles_cap = need;
    }
    if (!c->d_owner_start && hipMalloc(&c->d_owner_start, 2 * SR_MAX_OWNERS * sizeof(uint64_t)) != hipSuccess)
        return -ENOMEM;
    p.tile_counts = c->d_pack_tiles;
    p.tile_base = c->d_pack_tiles + c->pack_tiles_cap;
    p.owner_start = c->d_owner_start;
    p.owner_counts = d_owner_counts;
    p.out_bytes = d_out_bytes;
    p.out_cap = out_cap;
    p.out_recs = d_out_recs;
    p.own = own;
    p.own_bytes = own_bytes;
    p.own_recs = own_recs;
    if ((phases & kPackSizes) && ntiles) {
        const dim3 grid((ntiles + kCountTiles - 1) / kCountTiles);
        if (ch == 1) hipLaunchKernelGGL(pack_count_kernel<1>, grid, dim3(kPackBlock), 0, c->stream, p);
        else hipLaunchKernelGGL(pack_count_kernel<kPackMaxChunks>, grid, dim3(kPackBlock), 0, c->stream, p);
        if (hipGetLastError() != hipSuccess) return -EIO;
    }
    if (phases & kPackSizes) {
        hipLaunchKernelGGL(pack_scan_kernel, dim3(1), dim3(1024), 0, c->stream, p);
        if (hipGetLastError() != hipSuccess) return -EIO;
    }
    if ((phases & kPackScatter) && ntiles) {
        if (ch == 1) hipLaunchKernelGGL(pack_scatter_kernel<1>, dim3(ntiles), dim3(kPackBlock), 0, c->stream, p);
        else hipLaunchKernelGGL(pack_scatter_kernel<kPackMaxChunks>, dim3(ntiles), dim3(kPackBlock), 0, c->stream, p);
        if (hipGetLastError() != hipSuccess) return -EIO;
    }
    return 0;
}

int sr_pack_by_owner(sr_ctx *c, const uint8_t *d_bytes, size_t nbytes, const sr_record *d_recs,
                     const uint64_t *d_n_records, size_t max_records, uint32_t n_owners, uint8_t *d_out_bytes,
                     size_t out_cap, sr_record *d_out_recs, uint64_t *d_owner_counts) {
    if (!c || !d_n_records || !d_owner_counts || n_owners == 0 || n_owners > SR_MAX_OWNERS) return -EINVAL;
    // the packed layout is addressed with u32 offsets: its worst case must fit 32 bits, and the
    // caller's buffer must hold that worst case (the kernels never truncate silently)
    if (max_records > 0xFFFFFFFFull || SR_PACK_CAPACITY((uint64_t)nbytes) > 0xFFFFFFFFull) return -EINVAL;
    if (out_cap < SR_PACK_CAPACITY((uint64_t)nbytes)) return -EINVAL;
    if (out_cap > 0xFFFFFFFFull) out_cap = 0xFFFFFFFFull;
    if (max_records && (!d_recs || !d_out_recs || !d_bytes || !d_out_bytes)) return -EINVAL;
    (void)hipSetDevice(c->device);
    PackBatch b{d_bytes, d_recs, d_n_records, (uint32_t)nbytes, (uint32_t)max_records, 0, 0};
    c->own_set = 0;
    c->own_counts = nullptr;
    return pack_launch(c, &b, 1, n_owners, d_out_bytes, out_cap, d_out_recs, d_owner_counts);
}

// The key sr_pack_owner_scatter must match: the batch descriptors (pointers, sizes) and owners of the
// context's last sr_pack_owner_sizes, whose tile bases and split sizes the scatter uses (FNV-1a)
static uint64_t pack_shape(const PackBatch *in, size_t count, uint32_t n_owners) {
    uint64_t h = 0xcbf29ce484222325ull;
    auto mix = [&h](uint64_t v) {
        for (int i = 0; i < 8; ++i, v >>= 8) h = (h ^ (v & 0xFFu)) * 0x100000001b3ull;
    };
    mix(n_owners);
    mix(count);
    for (size_t j = 0; j < count; ++j) {
        mix((uint64_t)(uintptr_t)in[j].bytes);
        mix((uint64_t)(uintptr_t)in[j].recs);
        mix((uint64_t)(uintptr_t)in[j].n_records);
        mix((uint64_t)in[j].nbytes << 32 | in[j].max_records);
    }
    return h;
}

static int pack_many_args(const sr_batch *batches, size_t count, uint32_t n_owners, PackBatch *in,
                          uint64_t *total_bytes) {
    if (n_owners == 0 || n_owners > SR_MAX_OWNERS) return -EINVAL;
    if (count == 0 || count > SR_MAX_BATCHES_PER_LAUNCH || !batches) return -EINVAL;
    *total_bytes = 0;
    for (size_t j = 0; j < count; ++j) {
        const sr_batch &b = batches[j];
        if (!b.d_n_records || b.max_records > 0xFFFFFFFFull || b.nbytes > 0xFFFFFFF0ull) return -EINVAL;
        if (b.max_records && (!b.d_out || !b.d_bytes)) return -EINVAL;
        *total_bytes += b.nbytes;
        in[j] = PackBatch{b.d_bytes, b.d_out, b.d_n_records, (uint32_t)b.nbytes, (uint32_t)b.max_records, 0, 0};
    }
    return SR_PACK_CAPACITY(*total_bytes) > 0xFFFFFFFFull ? -EINVAL : 0;
}

int sr_pack_many_by_owner(sr_ctx *c, const sr_batch *batches, size_t count, uint32_t n_owners, uint8_t *d_out_bytes,
                          size_t out_cap, sr_record *d_out_recs, uint64_t *d_owner_counts) {
    if (!c || !d_owner_counts) return -EINVAL;
    uint64_t total_bytes = 0;
    PackBatch in[kPackMaxBatches];
    int rc = pack_many_args(batches, count, n_owners, in, &total_bytes);
    if (rc) return rc;
    if (out_cap < SR_PACK_CAPACITY(total_bytes)) return -EINVAL;
    if (out_cap > 0xFFFFFFFFull) out_cap = 0xFFFFFFFFull;
    if (!d_out_bytes || !d_out_recs) return -EINVAL;
    (void)hipSetDevice(c->device);
    c->own_set = 0;
    c->own_counts = nullptr;
    return pack_launch(c, in, (uint32_t)count, n_owners, d_out_bytes, out_cap, d_out_recs, d_owner_counts);
}

int sr_pack_owner_sizes(sr_ctx *c, const sr_batch *batches, size_t count, uint32_t n_owners, uint64_t *d_owner_counts) {
    if (!c || !d_owner_counts) return -EINVAL;
    uint64_t total_bytes = 0;
    PackBatch in[kPackMaxBatches];
    int rc = pack_many_args(batches, count, n_owners, in, &total_bytes);
    if (rc) return rc;
    (void)hipSetDevice(c->device);
    c->own_set = 0;
    c->own_counts = d_owner_counts;
    c->own_shape = pack_shape(in, count, n_owners);
    rc = pack_launch(c, in, (uint32_t)count, n_owners, nullptr, 0, nullptr, d_owner_counts, kPackSizes);
    if (rc) c->own_counts = nullptr;
    return rc;
}

int sr_pack_owner_scatter(sr_ctx *c, const sr_batch *batches, size_t count, uint32_t n_owners, int own,
                          uint8_t *d_own_bytes, sr_record *d_own_recs, uint8_t *d_out_bytes, size_t out_cap,
                          sr_record *d_out_recs) {
    if (!c || !c->own_counts || own < -1 || own >= (int)n_owners) return -EINVAL;
    uint64_t total_bytes = 0;
    PackBatch in[kPackMaxBatches];
    int rc = pack_many_args(batches, count, n_owners, in, &total_bytes);
    if (rc) return rc;
    if (pack_shape(in, count, n_owners) != c->own_shape) return -EINVAL;
    if (out_cap < SR_PACK_CAPACITY(total_bytes)) return -EINVAL;
    if (out_cap > 0xFFFFFFFFull) out_cap = 0xFFFFFFFFull;
    if (!d_out_bytes || !d_out_recs) return -EINVAL;
    if (own >= 0 && (!d_own_bytes || !d_own_recs || ((uintptr_t)d_own_bytes & 3u))) return -EINVAL;
    (void)hipSetDevice(c->device);
    // sr_exchange_data finds the own chunk in place and does not copy it
    c->own_set = own >= 0;
    c->own = own;
    c->own_bytes = d_own_bytes;
    c->own_recs = d_own_recs;
    return pack_launch(c, in, (uint32_t)count, n_owners, d_out_bytes, out_cap, d_out_recs, c->own_counts, kPackScatter,
                       own, d_own_bytes, d_own_recs);
}

// Scratch of the packing kernels for one launch (grown, never shrunk; not in stream capture).
static int mtu_reserve(sr_ctx *c, uint32_t tiles, uint32_t chunks, uint32_t nb) {
    const uint32_t nds = c->ds.nds;
    if (tiles > c->mtu_ntiles) {
        free_ptr(c->d_mtu_tiles);
        c->d_mtu_tiles = nullptr;
        c->mtu_ntiles = 0;
        if (hipMalloc(&c->d_mtu_tiles, (size_t)(nds + 1) * tiles * sizeof(uint32_t)) != hipSuccess) return -ENOMEM;
        c->mtu_ntiles = tiles;
    }
    if (!c->d_mtu_keys) {   // keys and closed counts for the most batches a launch can hold
        const size_t words = (size_t)kMtuMaxBatches * (2 * (size_t)nds + 4) + (size_t)kMtuMaxBatches * nds;
        if (hipMalloc(&c->d_mtu_keys, words * sizeof(uint32_t)) != hipSuccess) return -ENOMEM;
    }
    (void)nb;
    if (chunks > c->mtu_chunks) {
        free_ptr(c->d_mtu_chunks);
        free_ptr(c->d_mtu_table);
        free_ptr(c->d_mtu_gp);
        c->d_mtu_chunks = nullptr;
        c->d_mtu_table = nullptr;
        c->d_mtu_gp = nullptr;
        c->mtu_chunks = 0;
        // shard, entry, open, first descriptor per chunk
        if (hipMalloc(&c->d_mtu_chunks, 4 * (size_t)chunks * sizeof(uint32_t)) != hipSuccess) return -ENOMEM;
        // the tables, then next(i) - i of every line of every chunk
        if (hipMalloc(&c->d_mtu_table, (size_t)chunks * (kMtuX * sizeof(uint64_t) + kMtuChunk) + 16) != hipSuccess)
            return -ENOMEM;
        if (hipMalloc(&c->d_mtu_gp, (size_t)chunks * (kMtuChunk * sizeof(uint16_t) + (kMtuP0 + 1) * sizeof(uint32_t))) !=
            hipSuccess)
            return -ENOMEM;
        c->mtu_chunks = chunks;
    }
    return 0;
}

#ifdef SR_MTU_STAMPS
static uint64_t *g_mtu_dbg = nullptr;
static size_t g_mtu_dbg_n = 0;
extern "C" size_t sr_mtu_stamps(uint64_t *dst, size_t max_chunks) {
    const size_t n = g_mtu_dbg_n < max_chunks ? g_mtu_dbg_n : max_chunks;
    if (g_mtu_dbg && n) (void)hipMemcpy(dst, g_mtu_dbg, n * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost);
    return n;
}
#endif

// hist (group mode): the key histograms of the route kernel's tiles for these batches, written by the
// context's last route launch (RouteParams::hist); route_bytes: each batch's bytes in that launch
// (its tiles: ceil(bytes / 16 KiB), numbered in batch order as launch_route numbers them)
static int pack_many_impl(sr_ctx *c, const sr_pack_batch *batches, size_t count, uint32_t *hist,
                          const size_t *route_bytes, bool fused = false, const uint64_t *tile_pd = nullptr) {
    if (!c || !batches || count == 0 || count > (size_t)kMtuMaxBatches) return -EINVAL;
    const uint32_t nds = c->ds.nds;
    if (nds > SR_MAX_PACK_DOWNSTREAMS) return -EINVAL;
    MtuLaunch L;
    memset(&L, 0, sizeof(L));
    // Chunk size: a shard's chunks are composed one after another (mtu_chain), so few shards with
    // many lines each want long chunks; many shards (short chains) want more, smaller chunks in
    // flight (2048 lines: 16 KiB of LDS per table workgroup, ten per CU instead of five).
    uint64_t all_records = 0;
    for (size_t j = 0; j < count; ++j) all_records += batches[j].max_records;
    uint32_t ch = all_records <= (uint64_t)(nds ? nds : 1) * 32u * kMtuChunk ? (uint32_t)kMtuChunkSmall
                                                                            : (uint32_t)kMtuChunk;
    if (c->mtu_chunk) ch = c->mtu_chunk;   // SR_KNOB_MTU_CHUNK (A/B runs)
    uint32_t tiles = 0, chunks = 0, groups = 0;
    constexpr uint32_t kGroup = 8;   // route tiles per scatter wave (C2: 2048 records, C4: 128)
    for (size_t j = 0; j < count; ++j) {
        const sr_pack_batch &b = batches[j];
        if (!b.d_n_records || !b.d_counts || (nds && !b.d_fill_out) || b.max_records > 0xFFFFFFF0ull) return -EINVAL;
        if (b.max_records && (!b.d_recs || !b.d_sorted)) return -EINVAL;
        if (b.max_packets && !b.d_packets) return -EINVAL;
        MtuBatchArg &a = L.b[j];
        a.recs = b.d_recs;
        a.n_records = b.d_n_records;
        a.fill_in = b.d_fill_in;
        a.probed_dead = b.d_probed_dead;
        a.sorted = b.d_sorted;
        a.packets = b.d_packets;
        a.counts = b.d_counts;
        a.fill_out = b.d_fill_out;
        a.max_records = (uint32_t)b.max_records;
        a.max_packets = (uint32_t)(b.max_packets > 0xFFFFFFFFull ? 0xFFFFFFFFull : b.max_packets);
        a.tile0 = tiles;
        a.chunk0 = chunks;
        if (hist) {   // the route launch's tiles of this batch
            const uint32_t nt = (uint32_t)((route_bytes[j] + 16383) / 16384);
            a.grp0 = groups;
            groups += (nt + kGroup - 1) / kGroup;
            tiles += nt;
        } else {
            const uint64_t nt = (b.max_records + kMtuTile - 1) / kMtuTile;
            tiles += (uint32_t)(nt ? nt : 1);
        }
        chunks += (uint32_t)((b.max_records + ch - 1) / ch) + nds + 1;
    }
    (void)hipSetDevice(c->device);
    int rc = mtu_reserve(c, hist ? 0u : tiles, chunks, (uint32_t)count);
    if (rc) return rc;
    L.nds = nds;
    L.group = hist ? kGroup : 0u;
    L.groups = groups;
    L.nb = (uint32_t)count;
    L.tiles = tiles;
    L.chunks = chunks;
    L.chunk_lines = ch;
    L.tile_counts = hist ? hist : c->d_mtu_tiles;
    L.keys = c->d_mtu_keys;
    L.closed = c->d_mtu_keys + (size_t)kMtuMaxBatches * (2 * (size_t)nds + 4);
    L.chunk_shard = c->d_mtu_chunks;
    L.chunk_entry = c->d_mtu_chunks + (size_t)chunks;
    L.chunk_open = c->d_mtu_chunks + 2 * (size_t)chunks;
    L.chunk_pk = c->d_mtu_chunks + 3 * (size_t)chunks;
    L.table = c->d_mtu_table;
    L.nx = reinterpret_cast<uint8_t *>(c->d_mtu_table + (((size_t)c->mtu_chunks * kMtuX + 1) & ~(size_t)1));
    L.plen = reinterpret_cast<uint16_t *>(c->d_mtu_gp);
    // group mode after a one-dead-shard launch: mtu_scan ORs the route tiles' probed-dead slots
    L.tile_pd = hist ? tile_pd : nullptr;
    L.pd_words = c->ds.nwords;
    L.gp0 = c->d_mtu_gp + (size_t)c->mtu_chunks * kMtuChunk / 2;
    if (fused) {   // the route launch's deferred probes, run by the counting pass
        if (hist) return -EIO;
        const DeviceState &ds = c->ds;
        L.probe = ProbeArgs{ds.nds, ds.dead, 2u, 0u, ds.magic_n, ds.d_alive, ds.d_magic};
        L.fd_mark = ds.fd_mark;
        L.nwords = ds.nwords;
        for (size_t j = 0; j < count; ++j) L.b[j].dhash = ds.fd_dhash[j];
    }
#ifdef SR_MTU_STAMPS   // developer timeline: 8 stamps per chunk, read back with sr_mtu_stamps
    static uint64_t *d_dbg = nullptr;
    static size_t dbg_cap = 0;
    if (chunks > dbg_cap) {
        if (d_dbg) (void)hipFree(d_dbg);
        dbg_cap = chunks;
        if (hipMalloc(&d_dbg, dbg_cap * 8 * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
    }
    (void)hipMemsetAsync(d_dbg, 0, (size_t)chunks * 8 * sizeof(uint64_t), c->stream);
    L.dbg = d_dbg;
    g_mtu_dbg = d_dbg;
    g_mtu_dbg_n = chunks;
#else
    L.dbg = nullptr;
#endif
    // the chunk kernels' grid: eight batches or more put each batch's chunks on one XCD
    // (mtu_chunk_slot): eight times the most slots any XCD takes
    uint32_t chunk_grid = chunks;
    L.xcd = (c->mtu_xcd && count >= 8) ? 1u : 0u;   // SR_KNOB_MTU_XCD 0: chunks dealt in launch order
    if (L.xcd) {
        uint32_t per[8] = {0, 0, 0, 0, 0, 0, 0, 0}, mx = 0;
        for (size_t j = 0; j < count; ++j) {
            const uint32_t s1 = j + 1 < count ? L.b[j + 1].chunk0 : chunks;
            per[j & 7] += s1 - L.b[j].chunk0;
        }
        for (int x = 0; x < 8; ++x) mx = per[x] > mx ? per[x] : mx;
        chunk_grid = 8 * mx;
    }
    const size_t sort_lds = (size_t)kMtuSortWaves * (nds + 1) * sizeof(uint32_t);
    // up to 4 x 4097 counters: past the 64 KiB default
    ensure_dyn_lds((const void *)mtu_count_kernel<false>, 96 * 1024);
    ensure_dyn_lds((const void *)mtu_count_kernel<true>, 64 * 1024);
    ensure_dyn_lds((const void *)mtu_scatter_kernel, 96 * 1024);
    if (hist) {   // the route kernel counted the keys: scan its tiles' histograms, scatter by groups of tiles
        ensure_dyn_lds((const void *)mtu_scatter_groups_kernel, 96 * 1024);
        const uint32_t gblocks = (groups + kMtuSortWaves - 1) / kMtuSortWaves;
        hipLaunchKernelGGL(mtu_scan_kernel, dim3((uint32_t)count), dim3(1024), 0, c->stream, L);
        if (gblocks)
            hipLaunchKernelGGL(mtu_scatter_groups_kernel, dim3(gblocks), dim3(64 * kMtuSortWaves), sort_lds, c->stream, L);
    } else {
        const uint32_t sort_blocks = (tiles + kMtuSortWaves - 1) / kMtuSortWaves;
        if (fused)
            hipLaunchKernelGGL(mtu_count_kernel<true>, dim3(sort_blocks), dim3(64 * kMtuSortWaves), sort_lds, c->stream, L);
        else
            hipLaunchKernelGGL(mtu_count_kernel<false>, dim3(sort_blocks), dim3(64 * kMtuSortWaves), sort_lds, c->stream, L);
        hipLaunchKernelGGL(mtu_scan_kernel, dim3((uint32_t)count), dim3(1024), 0, c->stream, L);
        hipLaunchKernelGGL(mtu_scatter_kernel, dim3(sort_blocks), dim3(64 * kMtuSortWaves), sort_lds, c->stream, L);
    }
    if (ch == (uint32_t)kMtuChunk)
        hipLaunchKernelGGL(mtu_table_kernel<kMtuChunk>, dim3(chunk_grid), dim3(kMtuTableBlock), 0, c->stream, L);
    else
        hipLaunchKernelGGL(mtu_table_kernel<kMtuChunkSmall>, dim3(chunk_grid), dim3(kMtuTableBlock), 0, c->stream, L);
    // the chain inside the emit kernel (one lane per shard) up to 64 shards, else mtu_chain
    // (a batch's fill_out read as some batch's fill_in would change under the walks: mtu_chain reads
    // every fill_in before the shard's fill_out is written)
    bool walk = c->mtu_walk && nds <= 64;   // SR_KNOB_MTU_WALK 0: mtu_chain
    for (size_t a = 0; walk && a < count; ++a)
        for (size_t b = 0; walk && b < count; ++b) {
            const uint16_t *in = batches[b].d_fill_in, *out = batches[a].d_fill_out;
            if (in && out && in < out + nds && out < in + nds) walk = false;
        }
    if (!walk) hipLaunchKernelGGL(mtu_chain_kernel, dim3((uint32_t)count), dim3(1024), 0, c->stream, L);
    if (ch == (uint32_t)kMtuChunk) {
        if (walk) hipLaunchKernelGGL((mtu_emit_kernel<kMtuChunk, true>), dim3(chunk_grid), dim3(kMtuBlock), 0, c->stream, L);
        else hipLaunchKernelGGL((mtu_emit_kernel<kMtuChunk, false>), dim3(chunk_grid), dim3(kMtuBlock), 0, c->stream, L);
    } else {
        if (walk) hipLaunchKernelGGL((mtu_emit_kernel<kMtuChunkSmall, true>), dim3(chunk_grid), dim3(kMtuBlock), 0, c->stream, L);
        else hipLaunchKernelGGL((mtu_emit_kernel<kMtuChunkSmall, false>), dim3(chunk_grid), dim3(kMtuBlock), 0, c->stream, L);
    }
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int sr_pack_packets_many(sr_ctx *c, const sr_pack_batch *batches, size_t count) {
    return pack_many_impl(c, batches, count, nullptr, nullptr);
}

// Route (one launch) and pack. With every shard alive (or exactly one dead: KV_DEAD1) and at most
// kHistKeys - 1 shards the route
// kernel (uniform / segment layouts) also writes each tile's key histogram and the packing skips
// mtu_count, its own pass over the records: C2 packing 0.118-0.120 -> 0.108-0.114 ms, C3 0.075-0.077
// -> 0.069-0.071 per 32 batches. Batches whose record capacity says fewer than 32 lines per 16 KiB
// tile (C4's 1024-byte lines: 16) keep the counting pass, which is cheaper there than scanning
// kHistKeys x 1024 tile counts per batch (C4 packing 0.062-0.066 against 0.071-0.076 ms;
// profiles/r05/pack_hist_ab_r5e.jsonl).
static int route_pack_impl(sr_ctx *c, const sr_batch *route, const sr_pack_batch *pack, size_t count) {
    DeviceState &ds = c->ds;
    bool want = c->hist && ds.dead <= 1 && ds.nds >= 1 && ds.nds < (uint32_t)kHistKeys;
    for (size_t i = 0; want && i < count; ++i)
        want = route[i].max_records * 512 >= route[i].nbytes;
    if (want && !ds.d_hist) {
        const size_t words = (size_t)(ds.max_tiles ? ds.max_tiles : 1) * kHistKeys;
        if (hipMalloc(&ds.d_hist, words * sizeof(uint32_t)) != hipSuccess) ds.d_hist = nullptr;
    }
    RouteParams p = ds.params();
    size_t bytes[kMaxBatches];
    for (size_t i = 0; i < count; ++i) {
        DeviceState::add_batch(p, route[i].d_bytes, route[i].nbytes, route[i].d_out, route[i].max_records,
                               route[i].d_hashes, route[i].d_n_records, route[i].d_probed_dead);
        bytes[i] = route[i].nbytes;
    }
    p.hist = want ? ds.d_hist : nullptr;
    ds.last_hist = false;
    ds.fuse_defer = c->fuse_defer && !want;
    ds.pack_ors_marks = want;
    ds.last_marks_pending = false;
    int rc = launch_variant(ds, p, c->stream);
    ds.fuse_defer = false;
    ds.pack_ors_marks = false;
    if (rc) return rc;
    const bool fused = ds.last_fused;
    ds.last_fused = false;
    const bool marks = ds.last_marks_pending;   // the tiles' probed-dead slots, for mtu_scan to OR
    ds.last_marks_pending = false;
    if (marks && !ds.last_hist) return -EIO;   // (never: such launches ran the KV_HIST1 kernel)
    return pack_many_impl(c, pack, count, ds.last_hist ? ds.d_hist : nullptr, bytes, fused,
                          marks ? ds.d_tile_pd : nullptr);
}

int sr_route_pack_many(sr_ctx *c, const sr_batch *route, const sr_pack_batch *pack, size_t count) {
    if (!c || !route || !pack || count == 0 || count > (size_t)kMaxBatches) return -EINVAL;
    for (size_t i = 0; i < count; ++i) {
        const sr_batch &b = route[i];
        if (!b.d_n_records || (b.nbytes && !b.d_bytes) || b.nbytes > c->ds.max_batch) return -EINVAL;
        if (b.max_records && !b.d_out) return -EINVAL;
        // the packing reads what the route writes
        if (pack[i].d_recs != b.d_out || pack[i].d_n_records != b.d_n_records || pack[i].max_records != b.max_records ||
            pack[i].d_probed_dead != b.d_probed_dead)
            return -EINVAL;
    }
    (void)hipSetDevice(c->device);
    return route_pack_impl(c, route, pack, count);
}

int sr_pack_packets(sr_ctx *c, const sr_record *d_recs, const uint64_t *d_n_records, size_t max_records,
                    const uint16_t *d_fill_in, const uint64_t *d_probed_dead, sr_record *d_sorted,
                    sr_packet *d_packets, size_t max_packets, uint64_t *d_counts, uint16_t *d_fill_out) {
    const sr_pack_batch b{d_recs, d_n_records, max_records, d_fill_in, d_probed_dead,
                          d_sorted, d_packets, max_packets, d_counts, d_fill_out};
    return sr_pack_packets_many(c, &b, 1);
}

static int grow(void **ptr, size_t *cap, size_t need, size_t elem) {
    if (need <= *cap) return 0;
    free_ptr(*ptr);
    *ptr = nullptr;
    *cap = 0;
    if (hipMalloc(ptr, (need ? need : 1) * elem) != hipSuccess) return -ENOMEM;
    *cap = need;
    return 0;
}

// Host outputs of a slot for batches of up to nbytes (grown, never shrunk; the slot is idle).
static size_t up256(size_t x) { return (x + 255) & ~(size_t)255; }
static int slot_reserve(sr_ctx *c, int k, size_t nbytes) {
    sr_ctx::Slot &sl = c->slot[k];
    const size_t nds = c->ds.nds, nw = c->ds.nwords ? c->ds.nwords : 1;
    const size_t rec = nbytes, pk = (size_t)SR_MAX_PACKETS(nbytes, c->ds.nds);
    if (!sl.done && hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess) {
        sl.done = nullptr;
        return -ENOMEM;
    }
    if (sl.host && rec <= sl.rec_cap && pk <= sl.pk_cap) return 0;
    if (sl.host) (void)hipHostFree(sl.host);
    sl.host = sl.dev = nullptr;
    sl.rec_cap = sl.pk_cap = 0;
    const size_t o_pk = up256(rec * sizeof(sr_record)), o_fill = o_pk + up256(pk * sizeof(sr_packet));
    const size_t o_pr = o_fill + up256(nds * sizeof(uint16_t) + 2), o_cnt = o_pr + up256(nw * sizeof(uint64_t));
    const size_t o_fin = o_cnt + 256, total = o_fin + up256(nds * sizeof(uint16_t) + 2);
    void *h = nullptr;
    if (hipHostMalloc(&h, total, hipHostMallocMapped) != hipSuccess) return -ENOMEM;
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipHostFree(h);
        return -EIO;
    }
    sl.host = (uint8_t *)h;
    sl.dev = (uint8_t *)d;
    sl.rec_cap = rec;
    sl.pk_cap = pk;
    sl.sorted = (sr_record *)sl.host;
    sl.packets = (sr_packet *)(sl.host + o_pk);
    sl.fill = (uint16_t *)(sl.host + o_fill);
    sl.probed = (uint64_t *)(sl.host + o_pr);
    sl.counts = (uint64_t *)(sl.host + o_cnt);
    sl.fill_in = (uint16_t *)(sl.host + o_fin);
    return 0;
}

// sr_set_trace: the slot's input-order records and hashes (grown, never shrunk; the slot is idle)
static int slot_trace_reserve(sr_ctx *c, int k, size_t nbytes) {
    sr_ctx::Slot &sl = c->slot[k];
    if (sl.thost && nbytes <= sl.trec_cap) return 0;
    if (sl.thost) (void)hipHostFree(sl.thost);
    sl.thost = sl.tdev = nullptr;
    sl.trec_cap = 0;
    void *h = nullptr, *d = nullptr;
    if (hipHostMalloc(&h, up256(nbytes * sizeof(sr_record)) + nbytes * sizeof(uint64_t) + 8, hipHostMallocMapped) !=
        hipSuccess)
        return -ENOMEM;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipHostFree(h);
        return -EIO;
    }
    sl.thost = (uint8_t *)h;
    sl.tdev = (uint8_t *)d;
    sl.trec_cap = nbytes;
    return 0;
}

static int pack_submit(sr_ctx *c, int k, const uint8_t *bytes, size_t nbytes, const uint16_t *fill) {
    sr_ctx::Slot &sl = c->slot[k];
    if (sl.busy) return -EBUSY;
    if ((nbytes && !bytes) || nbytes > c->ds.max_batch) return -EINVAL;
    if (c->ds.nds > SR_MAX_PACK_DOWNSTREAMS) return -EINVAL;
    if (nbytes && bytes[nbytes - 1] != '\n') return -EINVAL;
    (void)hipSetDevice(c->device);
    const size_t nds = c->ds.nds, nw = c->ds.nwords;
    int rc;
    // every buffer is sized for the context's largest batch at the first submission (an empty one
    // pre-allocates): growing page-locked memory or freeing device memory mid-stream would stall the
    // data thread while its socket fills
    const size_t full = c->ds.max_batch, fullp = (size_t)SR_MAX_PACKETS(full, nds);
    if ((rc = slot_reserve(c, k, full))) return rc;
    if (c->trace && (rc = slot_trace_reserve(c, k, full))) return rc;
    const size_t cap = nbytes ? nbytes : 1;   // never more lines than bytes
    const size_t pcap = (size_t)SR_MAX_PACKETS(cap, nds);
    if ((rc = grow((void **)&c->d_out, &c->d_out_cap, full, sizeof(sr_record)))) return rc;
    if ((rc = grow((void **)&c->d_sorted, &c->d_sorted_cap, full, sizeof(sr_record)))) return rc;
    if ((rc = grow((void **)&c->d_packets, &c->d_packets_cap, fullp, sizeof(sr_packet)))) return rc;
    if (!c->d_fill) {
        if (hipMalloc(&c->d_fill, (3 * nds + 2) * sizeof(uint16_t)) != hipSuccess) {
            c->d_fill = nullptr;
            return -ENOMEM;
        }
        if (hipMemsetAsync(c->d_fill, 0, (3 * nds + 2) * sizeof(uint16_t), c->stream) != hipSuccess) return -EIO;
        c->fill_cur = 0;
    }
    if (!c->d_mcounts && hipMalloc(&c->d_mcounts, 4 * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
    uint16_t *const f_in = fill ? c->d_fill + 2 * nds : c->d_fill + (size_t)c->fill_cur * nds;
    uint16_t *const f_out = c->d_fill + (size_t)(c->fill_cur ^ 1) * nds;
    if (fill && nds) {   // staged in the slot's page-locked memory: the caller's array is free on return
        memcpy(sl.fill_in, fill, nds * sizeof(uint16_t));
        if (hipMemcpyAsync(f_in, sl.fill_in, nds * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream) != hipSuccess)
            return -EIO;
    }
    if (nbytes == 0) {   // no lines: the fills carry over, nothing is probed
        if (nds && hipMemcpyAsync(f_out, f_in, nds * sizeof(uint16_t), hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
            return -EIO;
        if (hipMemsetAsync(c->d_mcounts, 0, 4 * sizeof(uint64_t), c->stream) != hipSuccess) return -EIO;
    } else {
        if (hipMemcpyAsync(c->d_in, bytes, nbytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) return -EIO;
        // over 1024 shards with some dead the route kernel also writes the hashes: the probed-dead
        // replay then reads 8 bytes per line instead of re-hashing the names (probed_dead_kernel);
        // up to 1024 the probes note the dead shards themselves
        // TRACE (sr_set_trace) needs every line's hash too (sr-main.c:91)
        uint64_t *hashes = nullptr;
        if (c->trace || c->ds.replay_wants_hashes()) {
            if ((rc = grow((void **)&c->d_hash, &c->d_hash_cap, full, sizeof(uint64_t)))) return rc;
            hashes = c->d_hash;
        }
        const sr_batch rb{c->d_in, nbytes, c->d_out, cap, hashes, c->d_count, c->d_probed};
        const sr_pack_batch pb{c->d_out, c->d_count, cap, f_in, c->d_probed, c->d_sorted, c->d_packets, pcap,
                               c->d_mcounts, f_out};
        if ((rc = route_pack_impl(c, &rb, &pb, 1))) return rc;
    }
    c->fill_cur ^= 1;
    PackOut o;
    o.sorted = c->d_sorted;
    o.packets = c->d_packets;
    o.fill = f_out;
    o.probed = (nbytes && c->ds.dead) ? c->d_probed : nullptr;
    o.counts = c->d_mcounts;
    o.rec_cap = sl.rec_cap;
    o.pk_cap = sl.pk_cap;
    o.nds = (uint32_t)nds;
    o.nwords = (uint32_t)nw;
    o.h_sorted = (sr_record *)(sl.dev + ((uint8_t *)sl.sorted - sl.host));
    o.h_packets = (sr_packet *)(sl.dev + ((uint8_t *)sl.packets - sl.host));
    o.h_fill = (uint16_t *)(sl.dev + ((uint8_t *)sl.fill - sl.host));
    o.h_probed = (uint64_t *)(sl.dev + ((uint8_t *)sl.probed - sl.host));
    o.h_counts = (uint64_t *)(sl.dev + ((uint8_t *)sl.counts - sl.host));
    sl.traced = c->trace;
    o.recs = (c->trace && nbytes) ? c->d_out : nullptr;   // input order, and the hashes (sr_route_pack_trace)
    o.hashes = (c->trace && nbytes) ? c->d_hash : nullptr;
    o.h_recs = c->trace ? (sr_record *)sl.tdev : nullptr;
    o.h_hashes = c->trace ? (uint64_t *)(sl.tdev + up256(sl.trec_cap * sizeof(sr_record))) : nullptr;
    // one workgroup per 512 records (two per thread), at most 1024 workgroups (grid-stride beyond)
    const uint64_t want = (cap + 511) / 512;
    hipLaunchKernelGGL(pack_out_kernel, dim3((uint32_t)(want < 1024 ? (want ? want : 1) : 1024)), dim3(256), 0,
                       c->stream, o);
    if (hipGetLastError() != hipSuccess) return -EIO;
    if (hipEventRecord(sl.done, c->stream) != hipSuccess) return -EIO;
    sl.busy = 1;
    return 0;
}

static int pack_result(sr_ctx *c, int k, sr_pack_result *res) {
    sr_ctx::Slot &sl = c->slot[k];
    if (!sl.busy) return -EBUSY;
    sl.busy = 0;
    (void)hipSetDevice(c->device);
    if (hipEventSynchronize(sl.done) != hipSuccess) return -EIO;
    const uint64_t np = sl.counts[0], nv = sl.counts[1], nr = sl.counts[2];
    res->sorted = sl.sorted;
    res->packets = sl.packets;
    res->fill = sl.fill;
    res->probed_dead = sl.probed;
    res->n_records = (size_t)(nr < sl.rec_cap ? nr : sl.rec_cap);
    res->n_valid = (size_t)(nv < res->n_records ? nv : res->n_records);
    res->n_packets = (size_t)(np < sl.pk_cap ? np : sl.pk_cap);
    return (nr > sl.rec_cap || np > sl.pk_cap) ? -ENOSPC : 0;
}

int sr_route_pack_trace(sr_ctx *c, int slot, const sr_record **records, const uint64_t **hashes, size_t *n) {
    if (!c || !records || !hashes || !n || slot < 0 || slot > 2) return -EINVAL;
    const sr_ctx::Slot &sl = c->slot[slot];
    if (sl.busy || !sl.traced || !sl.thost || !sl.counts) return -EBUSY;
    const uint64_t nr = sl.counts[2];
    *n = (size_t)(nr < sl.trec_cap ? nr : sl.trec_cap);
    *records = (const sr_record *)sl.thost;
    *hashes = (const uint64_t *)(sl.thost + up256(sl.trec_cap * sizeof(sr_record)));
    return 0;
}

int sr_route_pack_submit(sr_ctx *c, int slot, const uint8_t *bytes, size_t nbytes, const uint16_t *fill) {
    if (!c || slot < 0 || slot > 1) return -EINVAL;
    return pack_submit(c, slot, bytes, nbytes, fill);
}

int sr_route_pack_result(sr_ctx *c, int slot, sr_pack_result *res) {
    if (!c || !res || slot < 0 || slot > 1) return -EINVAL;
    return pack_result(c, slot, res);
}

int sr_route_pack_batch(sr_ctx *c, const uint8_t *bytes, size_t nbytes, uint16_t *fill, sr_record *sorted,
                        size_t max_records, size_t *n_records, size_t *n_valid, sr_packet *packets,
                        size_t max_packets, size_t *n_packets, uint64_t *probed_dead) {
    if (!c || !n_records || !n_valid || !n_packets || (nbytes && !bytes) || nbytes > c->ds.max_batch) return -EINVAL;
    if ((c->ds.nds && !fill) || (max_records && !sorted) || (max_packets && !packets)) return -EINVAL;
    if (c->ds.nds > SR_MAX_PACK_DOWNSTREAMS) return -EINVAL;
    *n_records = *n_valid = *n_packets = 0;
    const uint32_t nw = c->ds.nwords;
    if (nbytes == 0) {
        if (probed_dead && nw) memset(probed_dead, 0, nw * sizeof(uint64_t));
        return 0;
    }
    int rc = pack_submit(c, 2, bytes, nbytes, fill);
    if (rc) return rc;
    sr_pack_result r;
    rc = pack_result(c, 2, &r);
    if (rc && rc != -ENOSPC) return rc;
    const size_t cr = r.n_records < max_records ? r.n_records : max_records;
    const size_t cp = r.n_packets < max_packets ? r.n_packets : max_packets;
    if (cr) memcpy(sorted, r.sorted, cr * sizeof(sr_record));
    if (cp) memcpy(packets, r.packets, cp * sizeof(sr_packet));
    if (c->ds.nds) memcpy(fill, r.fill, c->ds.nds * sizeof(uint16_t));
    if (probed_dead && nw) memcpy(probed_dead, r.probed_dead, nw * sizeof(uint64_t));
    *n_records = r.n_records;
    *n_valid = r.n_valid;
    *n_packets = r.n_packets;
    return (rc || r.n_records > max_records || r.n_packets > max_packets) ? -ENOSPC : 0;
}

int sr_route_batch(sr_ctx *c, const uint8_t *bytes, size_t nbytes, sr_record *out, size_t max_records,
                   size_t *n_records, uint64_t *hashes) {
    if (!c || !n_records || (nbytes && !bytes) || nbytes > c->ds.max_batch) return -EINVAL;
    if (max_records && !out) return -EINVAL;
    *n_records = 0;
    if (nbytes == 0) {
        if (c->ds.nwords) memset(c->h_probed, 0, c->ds.nwords * sizeof(uint64_t));
        return 0;
    }
    if (bytes[nbytes - 1] != '\n') return -EINVAL;
    // every shard alive: nothing can be probed dead (the device bitmap is skipped)
    if (c->ds.nwords) memset(c->h_probed, 0, c->ds.nwords * sizeof(uint64_t));
    (void)hipSetDevice(c->device);
    // device record capacity: never more lines than bytes
    const size_t cap = max_records < nbytes ? max_records : nbytes;
    if (cap > c->d_out_cap) {
        (void)hipFree(c->d_out);
        c->d_out = nullptr;
        c->d_out_cap = 0;
        if (hipMalloc(&c->d_out, cap * sizeof(sr_record)) != hipSuccess) return -ENOMEM;
        c->d_out_cap = cap;
    }
    // hashes: asked for, or for the probed-dead replay (probed_dead_kernel; over 1024 shards)
    const bool want_hash = hashes || c->ds.replay_wants_hashes();
    if (want_hash && cap > c->d_hash_cap) {
        (void)hipFree(c->d_hash);
        c->d_hash = nullptr;
        c->d_hash_cap = 0;
        if (hipMalloc(&c->d_hash, cap * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
        c->d_hash_cap = cap;
    }
    if (hipMemcpyAsync(c->d_in, bytes, nbytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) return -EIO;
    RouteParams p = c->ds.params();
    DeviceState::add_batch(p, c->d_in, nbytes, c->d_out, cap, want_hash ? c->d_hash : nullptr, c->d_count, c->d_probed);
    int rc = launch_variant(c->ds, p, c->stream);
    if (rc) return rc;
    if (c->ds.dead && c->ds.nwords &&
        hipMemcpyAsync(c->h_probed, c->d_probed, c->ds.nwords * sizeof(uint64_t), hipMemcpyDeviceToHost,
                       c->stream) != hipSuccess)
        return -EIO;
    uint64_t n = 0;
    if (hipMemcpyAsync(&n, c->d_count, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        return -EIO;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -EIO;
    const size_t ncopy = n < cap ? (size_t)n : cap;
    if (ncopy) {
        if (hipMemcpyAsync(out, c->d_out, ncopy * sizeof(sr_record), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
            return -EIO;
        if (hashes &&
            hipMemcpyAsync(hashes, c->d_hash, ncopy * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
            return -EIO;
        if (hipStreamSynchronize(c->stream) != hipSuccess) return -EIO;
    }
    *n_records = (size_t)n;
    return n > max_records ? -ENOSPC : 0;
}

}  // extern "C"

// ---- multi-GPU exchange (exchange.hpp) ----------------------------------------------------------
struct sr_comm {
    void *nccl;
    int world, rank, device;
    uint64_t *h_sizes;   // pinned, mapped, coherent: [2][world][2] sent, received, then the sequence word
    uint64_t *d_sizes;   // its device address (nullptr: copies and a stream synchronisation instead)
    uint64_t seq;
};

extern "C" {

int sr_comm_id(uint8_t id[SR_COMM_ID_BYTES]) {
    RcclApi *r = rccl_api();
    if (!id) return -EINVAL;
    if (!r) return -ENOSYS;
    return r->get_unique_id(id) == 0 ? 0 : -EIO;
}

int sr_comm_open(sr_comm **out, const uint8_t id[SR_COMM_ID_BYTES], int world, int rank, int device) {
    if (!out || !id || world < 1 || world > (int)kMaxOwners || rank < 0 || rank >= world) return -EINVAL;
    *out = nullptr;
    RcclApi *r = rccl_api();
    if (!r) return -ENOSYS;
    if (hipSetDevice(device) != hipSuccess) return -ENODEV;
    sr_comm *c = new (std::nothrow) sr_comm{nullptr, world, rank, device, nullptr, nullptr, 0};
    if (!c) return -ENOMEM;
    if (hipHostMalloc((void **)&c->h_sizes, (4 * (size_t)world + 1) * sizeof(uint64_t),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        delete c;
        return -ENOMEM;
    }
    memset(c->h_sizes, 0, (4 * (size_t)world + 1) * sizeof(uint64_t));
    if (hipHostGetDevicePointer((void **)&c->d_sizes, c->h_sizes, 0) != hipSuccess) c->d_sizes = nullptr;
    CommId cid;
    memcpy(cid.b, id, sizeof(cid.b));
    if (((InitRankFn)r->comm_init_rank)(&c->nccl, world, cid, rank) != 0) {
        (void)hipHostFree(c->h_sizes);
        delete c;
        return -EIO;
    }
    *out = c;
    return 0;
}

void sr_comm_close(sr_comm *c) {
    if (!c) return;
    RcclApi *r = rccl_api();
    if (r && c->nccl) (void)r->comm_destroy(c->nccl);
    (void)hipHostFree(c->h_sizes);
    delete c;
}

int sr_exchange_sizes(sr_ctx *ctx, sr_comm *comm, const uint64_t *d_owner_counts, uint64_t *d_recv_counts,
                      uint64_t *h_sent, uint64_t *h_received) {
    if (!ctx || !comm || !d_owner_counts || !d_recv_counts || !h_sent || !h_received) return -EINVAL;
    RcclApi *r = rccl_api();
    if (!r) return -ENOSYS;
    (void)hipSetDevice(ctx->device);
    const size_t w2 = 2 * (size_t)comm->world;
    if (comm->d_sizes) {
        // one rank: nothing to exchange (the received sizes are the sent ones, written by the publish
        // kernel); then the host spins on the sequence word, checking the stream now and then for errors
        if (comm->world > 1 &&
            r->all_to_all(d_owner_counts, d_recv_counts, 2, kNcclUint64, comm->nccl, ctx->stream) != 0)
            return -EIO;
        const uint64_t seq = ++comm->seq;
        hipLaunchKernelGGL(sizes_publish_kernel, dim3(1), dim3(256), 0, ctx->stream, d_owner_counts,
                           comm->world > 1 ? d_recv_counts : nullptr, d_recv_counts, comm->d_sizes,
                           (uint32_t)w2, seq);
        if (hipGetLastError() != hipSuccess) return -EIO;
        volatile const uint64_t *hs = comm->h_sizes;
        for (uint32_t k = 1; hs[2 * w2] != seq; ++k) {
            if ((k & 255u) == 0) {
                const hipError_t q = hipStreamQuery(ctx->stream);
                if (q == hipSuccess) {
                    if (hs[2 * w2] == seq) break;
                    return -EIO;
                }
                if (q != hipErrorNotReady) return -EIO;
            }
            __builtin_ia32_pause();
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        for (size_t i = 0; i < w2; ++i) {
            h_sent[i] = hs[i];
            h_received[i] = hs[w2 + i];
        }
        return 0;
    }
    if (r->all_to_all(d_owner_counts, d_recv_counts, 2, kNcclUint64, comm->nccl, ctx->stream) != 0) return -EIO;
    if (hipMemcpyAsync(comm->h_sizes, d_owner_counts, w2 * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream) !=
            hipSuccess ||
        hipMemcpyAsync(comm->h_sizes + w2, d_recv_counts, w2 * sizeof(uint64_t), hipMemcpyDeviceToHost,
                       ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
        return -EIO;
    memcpy(h_sent, comm->h_sizes, w2 * sizeof(uint64_t));
    memcpy(h_received, comm->h_sizes + w2, w2 * sizeof(uint64_t));
    return 0;
}

static int rebase_launch(hipStream_t stream, sr_record *d_recs, const sr_exchange_peer *peers, int world) {
    RebaseArgs a;
    int rc = rebase_args(peers, world, a);
    if (rc) return rc;
    if (a.n_lines > a.first) {   // (one source, or every source before the first that moves: nothing to add)
        hipLaunchKernelGGL(exchange_rebase_kernel, dim3((a.n_lines - a.first + 255u) / 256u), dim3(256), 0, stream, d_recs, a);
        if (hipGetLastError() != hipSuccess) return -EIO;
    }
    return 0;
}

// The RCCL transport of sr_exchange_data: every call enqueued on the context's stream. Both chunk
// kinds travel as bytes (the record chunk is 8 bytes per line on both sides of a pair).
struct RcclTransport {
    RcclApi *r;
    sr_comm *comm;
    hipStream_t stream;
    sr_ctx *ctx;
};

static int rccl_group_start(void *u) { return ((RcclTransport *)u)->r->group_start() == 0 ? 0 : -EIO; }
static int rccl_group_end(void *u) { return ((RcclTransport *)u)->r->group_end() == 0 ? 0 : -EIO; }
static int rccl_send(void *u, const void *buf, size_t bytes, int peer, int) {
    RcclTransport *t = (RcclTransport *)u;
    return t->r->send(buf, bytes, kNcclUint8, peer, t->comm->nccl, t->stream) == 0 ? 0 : -EIO;
}
static int rccl_recv(void *u, void *buf, size_t bytes, int peer, int) {
    RcclTransport *t = (RcclTransport *)u;
    return t->r->recv(buf, bytes, kNcclUint8, peer, t->comm->nccl, t->stream) == 0 ? 0 : -EIO;
}
static int rccl_copy(void *u, void *dst, const void *src, size_t bytes) {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ((RcclTransport *)u)->stream) == hipSuccess
               ? 0 : -EIO;
}
static int rccl_rebase(void *u, sr_record *recs, const sr_exchange_peer *peers, int world, uint64_t) {
    return rebase_launch(((RcclTransport *)u)->stream, recs, peers, world);
}

int sr_exchange_data(sr_ctx *ctx, sr_comm *comm, const uint8_t *d_packed, const sr_record *d_packed_recs,
                     const uint64_t *h_sent, const uint64_t *h_received, uint8_t *d_recv_bytes,
                     sr_record *d_recv_recs) {
    if (!ctx || !comm || !h_sent || !h_received) return -EINVAL;
    RcclApi *r = rccl_api();
    if (!r) return -ENOSYS;
    (void)hipSetDevice(ctx->device);
    RcclTransport rt{r, comm, ctx->stream, ctx};
    const sr_transport t{&rt, rccl_group_start, rccl_group_end, rccl_send, rccl_recv, rccl_copy, rccl_rebase};
    // the own chunk already in its place (sr_pack_owner_scatter into these receive buffers): no copy
    bool in_place = false;
    if (ctx->own_set && ctx->own == comm->rank) {
        sr_exchange_peer peers[kMaxOwners];
        uint64_t tot[4];
        if (exchange_plan(comm->world, comm->rank, h_sent, h_received, peers, tot) == 0) {
            const sr_exchange_peer &e = peers[comm->rank];
            in_place = ctx->own_bytes == d_recv_bytes + e.recv_byte0 && ctx->own_recs == d_recv_recs + e.recv_line0;
        }
    }
    ctx->own_set = 0;
    return exchange_run(t, comm->world, comm->rank, h_sent, h_received, d_packed, d_packed_recs, d_recv_bytes,
                        d_recv_recs, in_place);
}

// One route launch's regroup on any transport (sr_regroup_run): the split sizes, the size exchange
// (the one host round trip), the plan, the scatter with the rank's own chunk written straight into its
// place in the receive buffers, then the exchange without the own chunk's copy and the rebase.
// sr_regroup_launch is this on RCCL: both run this one sequence.
static int regroup_run(sr_ctx *ctx, const sr_transport &t, sr_sizes_fn sizes, int world, int rank,
                       const sr_batch *batches, size_t count, uint64_t *d_owner_counts, uint64_t *d_recv_counts,
                       uint8_t *d_packed, size_t packed_cap, sr_record *d_packed_recs, uint8_t *d_recv_bytes,
                       size_t recv_bytes_cap, sr_record *d_recv_recs, size_t recv_recs_cap, uint64_t *h_sent,
                       uint64_t *h_received) {
    if (!ctx || !sizes || !d_owner_counts || !d_recv_counts || !d_recv_bytes || !d_recv_recs || !h_sent ||
        !h_received || world < 1 || world > (int)kMaxOwners || rank < 0 || rank >= world)
        return -EINVAL;
    int rc = sr_pack_owner_sizes(ctx, batches, count, (uint32_t)world, d_owner_counts);
    if (rc) return rc;
    if ((rc = sizes(t.user, d_owner_counts, d_recv_counts, h_sent, h_received))) return rc;
    sr_exchange_peer peers[kMaxOwners];
    uint64_t tot[4];
    if ((rc = exchange_plan(world, rank, h_sent, h_received, peers, tot))) return rc;
    if (tot[2] > recv_recs_cap || tot[3] > recv_bytes_cap) return -ENOSPC;
    const sr_exchange_peer &e = peers[rank];
    rc = sr_pack_owner_scatter(ctx, batches, count, (uint32_t)world, rank, d_recv_bytes + e.recv_byte0,
                               d_recv_recs + e.recv_line0, d_packed, packed_cap, d_packed_recs);
    ctx->own_set = 0;   // consumed here: the exchange below is told the own chunk is in place
    if (rc) return rc;
    return exchange_run(t, world, rank, h_sent, h_received, d_packed, d_packed_recs, d_recv_bytes, d_recv_recs,
                        true);
}

static int rccl_sizes(void *u, const uint64_t *d_owner_counts, uint64_t *d_recv_counts, uint64_t *h_sent,
                      uint64_t *h_received) {
    RcclTransport *t = (RcclTransport *)u;
    return sr_exchange_sizes(t->ctx, t->comm, d_owner_counts, d_recv_counts, h_sent, h_received);
}

int sr_regroup_launch(sr_ctx *ctx, sr_comm *comm, const sr_batch *batches, size_t count,
                      uint64_t *d_owner_counts, uint64_t *d_recv_counts, uint8_t *d_packed, size_t packed_cap,
                      sr_record *d_packed_recs, uint8_t *d_recv_bytes, size_t recv_bytes_cap,
                      sr_record *d_recv_recs, size_t recv_recs_cap, uint64_t *h_sent, uint64_t *h_received) {
    if (!ctx || !comm) return -EINVAL;
    RcclApi *r = rccl_api();
    if (!r) return -ENOSYS;
    (void)hipSetDevice(ctx->device);
    RcclTransport rt{r, comm, ctx->stream, ctx};
    const sr_transport t{&rt, rccl_group_start, rccl_group_end, rccl_send, rccl_recv, rccl_copy, rccl_rebase};
    return regroup_run(ctx, t, rccl_sizes, comm->world, comm->rank, batches, count, d_owner_counts, d_recv_counts,
                       d_packed, packed_cap, d_packed_recs, d_recv_bytes, recv_bytes_cap, d_recv_recs, recv_recs_cap,
                       h_sent, h_received);
}

int sr_regroup_run(sr_ctx *ctx, const sr_transport *t, sr_sizes_fn sizes, int world, int rank,
                   const sr_batch *batches, size_t count, uint64_t *d_owner_counts, uint64_t *d_recv_counts,
                   uint8_t *d_packed, size_t packed_cap, sr_record *d_packed_recs, uint8_t *d_recv_bytes,
                   size_t recv_bytes_cap, sr_record *d_recv_recs, size_t recv_recs_cap, uint64_t *h_sent,
                   uint64_t *h_received) {
    if (!ctx || !t) return -EINVAL;
    (void)hipSetDevice(ctx->device);
    return regroup_run(ctx, *t, sizes, world, rank, batches, count, d_owner_counts, d_recv_counts, d_packed,
                       packed_cap, d_packed_recs, d_recv_bytes, recv_bytes_cap, d_recv_recs, recv_recs_cap, h_sent,
                       h_received);
}

int sr_exchange_plan(int world, int rank, const uint64_t *h_sent, const uint64_t *h_received,
                     sr_exchange_peer *peers, uint64_t *totals) {
    uint64_t tot[4];
    const int rc = exchange_plan(world, rank, h_sent, h_received, peers, tot);
    if (!rc && totals) memcpy(totals, tot, sizeof(tot));
    return rc;
}

int sr_exchange_run(const sr_transport *t, int world, int rank, const uint64_t *h_sent, const uint64_t *h_received,
                    const uint8_t *packed, const sr_record *packed_recs, uint8_t *recv_bytes, sr_record *recv_recs) {
    if (!t) return -EINVAL;
    return exchange_run(*t, world, rank, h_sent, h_received, packed, packed_recs, recv_bytes, recv_recs);
}

int sr_exchange_rebase(sr_ctx *ctx, sr_record *d_recv_recs, const sr_exchange_peer *peers, int world) {
    if (!ctx || !peers) return -EINVAL;
    RebaseArgs a;
    int rc = rebase_args(peers, world, a);
    if (rc) return rc;
    if (a.n_lines && !d_recv_recs) return -EINVAL;
    (void)hipSetDevice(ctx->device);
    return rebase_launch(ctx->stream, d_recv_recs, peers, world);
}

}  // extern "C"
