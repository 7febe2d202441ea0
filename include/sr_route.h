/*
 * sr_route.h — C ABI of the MI355X-native statsd-router hot path.
 *
 * The reference (hulu/statsd-router) has no plugin or FFI API: its hot path is the libev
 * callback `udp_read_cb` (sr-main.c:149-191), which frames one datagram and, per '\n'-terminated
 * line, calls `process_data_line` (sr-main.c:137-147) -> `hash` (sr-main.c:120-134) ->
 * `find_downstream` (sr-main.c:86-117) -> `push_to_downstream` (sr-main.c:73-83).
 * This header replaces the per-line calls with one call per BATCH of framed datagrams:
 * the GPU classifies every line (length gate, ':' presence, sdbm name hash, consistent-hash
 * shard pick) and returns one record per line in input order. The host caller keeps the
 * reference's side effects: it walks the records and does push_to_downstream, the WARN log
 * lines (exact reference text) and the dead-downstream buffer drop (sr-main.c:106).
 *
 * Conventions (mirroring the reference):
 *   - every function returns 0 or a negative errno value; nothing aborts;
 *   - a context is not thread-safe: use one per data thread / HIP stream, like one libev loop
 *     per thread (sr-main.c:237-308);
 *   - the alive bitmap is a snapshot (the reference reads the `alive:1` bit of
 *     ds_health_client_s (sr-types.h:25) racily per line; a per-batch snapshot is a valid
 *     linearisation of that).
 *
 * No torch or HIP types appear in the signatures: device pointers are plain pointers and the
 * stream is an opaque `void *` (a hipStream_t).
 */
#ifndef SR_ROUTE_H
#define SR_ROUTE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants of the reference contract ------------------------------------------------ */
#define SR_DATA_BUF_SIZE        4096u  /* sr-main.h:46: recv buffer; recv() reads at most 4095 B */
#define SR_MAX_DATAGRAM         (SR_DATA_BUF_SIZE - 1u)   /* sr-main.c:163 */
#define SR_DOWNSTREAM_BUF_SIZE  1450u  /* sr-types.h:30: a valid line is shorter than this      */
#define SR_MIN_LINE_LENGTH      6u     /* sr-main.c:180: `line_length > 5`                        */
#define SR_MAX_LINE_LENGTH      (SR_DOWNSTREAM_BUF_SIZE - 1u)  /* sr-main.c:180: `< 1450`         */
#define SR_MAX_DOWNSTREAMS      65533u /* shard ids must fit below the SR_ROUTE_* codes         */

/* ---- per-line verdicts -------------------------------------------------------------------- */
enum sr_verdict {
    SR_VALID          = 0, /* routed: process_data_line -> find_downstream -> push (sr-main.c:103) */
    SR_INVALID_LENGTH = 1, /* WARN "udp_read_cb: invalid length %d of metric %.*s" (sr-main.c:184)  */
    SR_INVALID_FORMAT = 2, /* WARN "process_data_line: invalid metric %s" (sr-main.c:142)            */
    SR_ALL_DEAD       = 3  /* WARN "find_downstream: all downstreams are dead" (sr-main.c:115)       */
};

/* `route` field: the shard id (0..n_downstreams-1) for SR_VALID, else one of these codes. */
#define SR_ROUTE_INVALID_LENGTH 0xFFFDu
#define SR_ROUTE_INVALID_FORMAT 0xFFFEu
#define SR_ROUTE_ALL_DEAD       0xFFFFu

/* One record per '\n'-terminated line, in input order. 8 bytes, little-endian, no padding. */
typedef struct sr_record {
    uint32_t offset; /* byte offset of the line's first byte in the batch                  */
    uint16_t length; /* bytes including the '\n' (saturates at 0xFFFF; lines > 4096 B only  */
                     /* occur when the caller breaks the framing contract)                  */
    uint16_t route;  /* shard id, or SR_ROUTE_*                                             */
} sr_record;

static inline int sr_record_verdict(const sr_record *r) {
    return r->route < SR_ROUTE_INVALID_LENGTH ? SR_VALID : (int)(r->route - 0xFFFCu);
}

/* ---- host-side framing (no GPU) ----------------------------------------------------------- */
/* Frame one received datagram exactly as udp_read_cb does (sr-main.c:163-173): keep at most
 * SR_MAX_DATAGRAM bytes (the recv() cap) and append '\n' if the last kept byte is not one.
 * Writes at most len+1 (<= 4096) bytes to dst; returns the framed length (0 for an empty datagram).
 * dst must not overlap src. */
size_t sr_frame_datagram(uint8_t *dst, const uint8_t *src, size_t len);

/* Frame `count` datagrams back to back into dst (capacity dst_cap). Returns the total framed
 * length, or (size_t)-1 if dst_cap is too small. */
size_t sr_frame_datagrams(uint8_t *dst, size_t dst_cap, const uint8_t *const *dgrams,
                          const size_t *lens, size_t count);

/* ---- context -------------------------------------------------------------------------------- */
typedef struct sr_ctx sr_ctx;

/* Open a context on HIP device `device` for batches of at most max_batch_bytes framed bytes and
 * n_downstreams shards (the order of the `downstream=` list in statsd-router.conf, sr-init.c:61-121).
 * All downstreams start alive. Allocates device buffers and a HIP stream.
 * Returns 0, -EINVAL, -ENODEV or -ENOMEM. */
int sr_open(sr_ctx **ctx, int device, size_t max_batch_bytes, uint32_t n_downstreams);

/* Snapshot of the health checker's alive bits (sr-health-client.c:15-18,37-40):
 * bit k of alive_bitmap[k/64] = downstream k alive. ceil(n_downstreams/64) words. */
int sr_set_alive(sr_ctx *ctx, const uint64_t *alive_bitmap);

/* Enqueue work on `stream` (a hipStream_t) instead of the context's own stream (NULL restores it). */
int sr_set_stream(sr_ctx *ctx, void *stream);

/* Lane layout of the route kernel. Timing only: the records are identical bit for bit.
 *   SR_LAYOUT_UNIFORM  every line of a tile gets the same lane group, sized by the tile's mean
 *                      line length (best for uniform lengths);
 *   SR_LAYOUT_SEGMENTS a tile of mixed lengths gets one lane per 64-byte name segment, lines packed
 *                      back to back (best when short and long lines share tiles);
 *   SR_LAYOUT_CHUNKS   every lane hashes the 64 bytes it loaded; lines spanning lanes are joined
 *                      by a block scan of partial hashes, lines spanning tiles by a look-back
 *                      (independent of the line lengths; best for mixed lengths);
 *   SR_LAYOUT_AUTO     (default) every 32nd launch outside stream capture (and the first) is a
 *                      segment-layout probe that weighs the traffic; chunks while at least a quarter
 *                      of the tiles of the last probe took the segment layout (back below a tenth),
 *                      uniform otherwise. A graph captured from the context keeps the layout of its
 *                      capture.
 * Returns 0 or -EINVAL. */
#define SR_LAYOUT_AUTO 0
#define SR_LAYOUT_UNIFORM 1
#define SR_LAYOUT_SEGMENTS 2
#define SR_LAYOUT_CHUNKS 3
int sr_set_layout(sr_ctx *ctx, int layout);

/* The layout the last route launch of the context used (SR_LAYOUT_UNIFORM, _SEGMENTS or _CHUNKS;
 * 0 before the first launch), or -EINVAL. */
int sr_last_layout(const sr_ctx *ctx);

/* Host-memory batch: copy `bytes` (concatenated framed datagrams; the last byte must be '\n'
 * unless nbytes == 0) to the device, classify every line, copy min(n, max_records) records (and,
 * if hashes != NULL, the 64-bit sdbm name hashes; 0 for invalid lines) back, and synchronise.
 * *n_records = number of lines n. Returns 0, or -ENOSPC if n > max_records (the first
 * max_records records are still valid), -EINVAL, -EIO. */
int sr_route_batch(sr_ctx *ctx, const uint8_t *bytes, size_t nbytes, sr_record *out,
                   size_t max_records, size_t *n_records, uint64_t *hashes);

/* The dead-downstream side effect of the last sr_route_batch call: find_downstream zeroes
 * active_buffer_length of every DEAD downstream its probe visits (sr-main.c:106). With the batch's
 * alive snapshot a dead downstream receives no line in that batch, so the caller reproduces the
 * effect exactly by dropping the pending buffer of every downstream whose bit is set here, before
 * it pushes the batch's lines. Writes ceil(n_downstreams/64) words (none when n_downstreams == 0).
 * Returns 0 or -EINVAL. */
int sr_last_probed_dead(const sr_ctx *ctx, uint64_t *bitmap);

/* Device-resident batch (asynchronous, enqueued on the context's stream): d_bytes, d_out,
 * d_hashes (may be NULL) and d_n_records are device pointers. Lines past max_records are counted
 * but not written; the line count is stored to *d_n_records when the work completes.
 * The input buffer needs no padding. Returns 0 or -EINVAL / -EIO (launch failure). */
int sr_route_device(sr_ctx *ctx, const uint8_t *d_bytes, size_t nbytes, sr_record *d_out,
                    size_t max_records, uint64_t *d_hashes, uint64_t *d_n_records);

/* Several device-resident batches in ONE launch (asynchronous, on the context's stream): the
 * batches of several data threads (the reference's threads_num sockets, sr-main.c:237-308) are
 * routed together, each exactly as sr_route_device would route it alone. Up to
 * SR_MAX_BATCHES_PER_LAUNCH batches share a kernel launch; larger counts are split into several
 * launches. Each batch must fit max_batch_bytes. Returns 0 or -EINVAL / -EIO. */
#define SR_MAX_BATCHES_PER_LAUNCH 32u
typedef struct sr_batch {
    const uint8_t *d_bytes;  /* framed datagrams, device memory                         */
    size_t nbytes;
    sr_record *d_out;        /* max_records records, device memory                      */
    size_t max_records;
    uint64_t *d_hashes;      /* NULL or max_records u64, device memory                  */
    uint64_t *d_n_records;   /* device u64: the batch's line count                      */
    uint64_t *d_probed_dead; /* NULL, or max(1, ceil(n_downstreams/64)) device u64: bit k  */
                             /* set iff some line of the batch probed dead downstream k   */
                             /* (find_downstream zeroes its active buffer, sr-main.c:106) */
} sr_batch;
int sr_route_device_many(sr_ctx *ctx, const sr_batch *batches, size_t count);

/* ---- multi-GPU regroup ------------------------------------------------------ */
/* Pack the VALID lines of a routed batch by owner GPU (owner of shard s = s % n_owners), ready for
 * an all-to-all: for owner 0..n_owners-1 in turn, its lines in input order, each starting at a
 * 4-byte aligned position (zero fill in between); d_out_recs gets one record per packed line in
 * the same order, with `offset` relative to the start of its owner's chunk. d_owner_counts
 * receives {lines, bytes} per owner (2*n_owners u64: the all-to-all split sizes). Lines routed
 * to no shard are not packed (their WARN stays with the GPU that received them).
 * d_recs / d_n_records: the output of sr_route_device for the same batch (same stream).
 * out_cap must be >= SR_PACK_CAPACITY(nbytes) (else -EINVAL), and SR_PACK_CAPACITY(nbytes) must fit
 * 32 bits (nbytes up to ~2.8 GB); d_out_recs needs max_records entries.
 * Asynchronous on the context's stream. n_owners in 1..64. Returns 0, -EINVAL, -ENOMEM, -EIO.
 * The first call (or one with a larger max_records / n_owners) allocates scratch: not inside
 * stream capture. */
#define SR_MAX_OWNERS 64u
#define SR_PACK_CAPACITY(nbytes) ((nbytes) + (nbytes) / 2u + 4u)
int sr_pack_by_owner(sr_ctx *ctx, const uint8_t *d_bytes, size_t nbytes, const sr_record *d_recs,
                     const uint64_t *d_n_records, size_t max_records, uint32_t n_owners,
                     uint8_t *d_out_bytes, size_t out_cap, sr_record *d_out_recs,
                     uint64_t *d_owner_counts);

/* sr_pack_by_owner over the batches of one route launch at once (one size exchange per launch):
 * batches[j].d_bytes / nbytes / d_out (its records) / max_records / d_n_records as given to
 * sr_route_device_many. Owner chunks hold batch 0's lines, then batch 1's, ..., each in input
 * order; record offsets are relative to the owner's chunk. out_cap >= SR_PACK_CAPACITY(total
 * bytes) (< 4 GiB), d_out_recs >= sum of max_records. count <= SR_MAX_BATCHES_PER_LAUNCH. */
int sr_pack_many_by_owner(sr_ctx *ctx, const sr_batch *batches, size_t count, uint32_t n_owners,
                          uint8_t *d_out_bytes, size_t out_cap, sr_record *d_out_recs,
                          uint64_t *d_owner_counts);

/* sr_pack_many_by_owner in two calls, so that the rank's own chunk can be written straight into its
 * place in the exchange's receive buffers (no local copy in sr_exchange_data):
 * sr_pack_owner_sizes: the split sizes alone into d_owner_counts (u64 [n_owners][2], as
 *   sr_pack_many_by_owner's), e.g. for sr_exchange_sizes; the context remembers d_owner_counts.
 * sr_pack_owner_scatter: the lines and records of the same batches (the next pack call on the context),
 *   owner `own`'s chunk to d_own_bytes / d_own_recs (its d_owner_counts bytes / lines, offsets relative to
 *   the chunk as always), every other owner's to d_out_bytes / d_out_recs at the usual places (out_cap as
 *   sr_pack_many_by_owner). With own = the comm's rank and d_own_* = d_recv_bytes + recv_byte0 /
 *   d_recv_recs + recv_line0 of peers[rank] (sr_exchange_plan), the following sr_exchange_data on this
 *   context skips the own chunk's copies. d_own_bytes must be 4-byte aligned. own = -1: every chunk to
 *   d_out_bytes / d_out_recs (sr_pack_many_by_owner's output; d_own_* unused). Both asynchronous on the
 *   context's stream. Returns 0, -EINVAL (scatter without sizes, own out of range), -ENOMEM, -EIO.
 * The two calls pair one to one: the scatter uses the tile bases and split sizes of the context's last
 * sizes call, and must be given the same batch descriptors and n_owners (else -EINVAL); a sizes call in
 * between replaces them. */
int sr_pack_owner_sizes(sr_ctx *ctx, const sr_batch *batches, size_t count, uint32_t n_owners,
                        uint64_t *d_owner_counts);
int sr_pack_owner_scatter(sr_ctx *ctx, const sr_batch *batches, size_t count, uint32_t n_owners, int own,
                          uint8_t *d_own_bytes, sr_record *d_own_recs, uint8_t *d_out_bytes, size_t out_cap,
                          sr_record *d_out_recs);

/* ---- multi-GPU exchange of owner packs (RCCL over xGMI) -------------------------------------- */
/* One process per GPU; shard s is owned by GPU s % world. After sr_pack_by_owner /
 * sr_pack_many_by_owner (n_owners = world), two collective calls per route launch move every
 * owner's lines to it. RCCL is loaded at sr_comm_open (dlopen of librccl.so.1; a copy already in
 * the process is shared); without it sr_comm_open returns -ENOSYS.
 *
 * sr_comm_id: a fresh communicator id, made by one rank and handed to the others out of band.
 * sr_comm_open: join the communicator as `rank` of `world` on HIP device `device` (collective:
 *   every rank calls it). Returns 0, -EINVAL, -ENOSYS (no RCCL), -EIO. */
#define SR_COMM_ID_BYTES 128u
typedef struct sr_comm sr_comm;
int sr_comm_id(uint8_t id[SR_COMM_ID_BYTES]);
int sr_comm_open(sr_comm **comm, const uint8_t id[SR_COMM_ID_BYTES], int world, int rank, int device);
void sr_comm_close(sr_comm *comm);

/* Collective, on the context's stream: all-to-all of the split sizes d_owner_counts (u64
 * [world][2] {lines, bytes} per owner, the pack's output) into d_recv_counts (u64 [world][2] per
 * source rank; one rank: a device copy, no collective), then both to the host: h_sent / h_received
 * (u64 [world][2]) are valid on return (the launch's one host round trip). One kernel writes them to
 * mapped pinned memory behind a sequence word the host spins on (polling the stream for errors), so the
 * call returns as soon as the sizes land, not when the stream drains: the caller's later work on the
 * context's stream is ordered after them as usual. Returns 0, -EINVAL, -EIO. */
int sr_exchange_sizes(sr_ctx *ctx, sr_comm *comm, const uint64_t *d_owner_counts, uint64_t *d_recv_counts,
                      uint64_t *h_sent, uint64_t *h_received);

/* Collective, asynchronous on the context's stream: every owner chunk of d_packed / d_packed_recs
 * (the pack's output) goes to its owner; the chunks received from sources 0, 1, ... land back to
 * back in d_recv_bytes (sum of h_received bytes) and d_recv_recs (sum of h_received lines), each
 * record's offset rebased into d_recv_bytes. Per source, every shard's lines keep their input
 * order. h_sent / h_received as sr_exchange_sizes returned them. Returns 0, -EINVAL, -EIO. */
int sr_exchange_data(sr_ctx *ctx, sr_comm *comm, const uint8_t *d_packed, const sr_record *d_packed_recs,
                     const uint64_t *h_sent, const uint64_t *h_received, uint8_t *d_recv_bytes,
                     sr_record *d_recv_recs);

/* The plan of one exchange (host only, no GPU): what sr_exchange_data moves to and from each peer.
 * For peer q, the pack's records [send_line0, send_line0 + send_lines) and bytes [send_byte0, +send_bytes)
 * go to q; q's chunk lands at records [recv_line0, +recv_lines) and bytes [recv_byte0, +recv_bytes) of
 * the receive buffers, and its records' offsets move by recv_byte0 (the rebase). peers[rank] is the
 * rank's own chunk: a local copy, not a send. The reference analogue is the SO_REUSEPORT split of
 * datagrams over data threads (sr-main.c:253-271,363-367); the plan is what regroups them by owner. */
typedef struct sr_exchange_peer {
    uint64_t send_line0, send_lines, send_byte0, send_bytes;
    uint64_t recv_line0, recv_lines, recv_byte0, recv_bytes;
} sr_exchange_peer;

/* Fill peers[world] from the split sizes (u64 [world][2] {lines, bytes}, as sr_exchange_sizes returns
 * them) and totals[4] = {lines sent, bytes sent, lines received, bytes received} (totals may be NULL).
 * Returns 0, or -EINVAL: bad world/rank, the own chunk's sent and received sizes differ, or a received
 * total does not fit the u32 record offsets. */
int sr_exchange_plan(int world, int rank, const uint64_t *h_sent, const uint64_t *h_received,
                     sr_exchange_peer *peers, uint64_t *totals);

/* The transport an exchange runs on. sr_exchange_data uses RCCL (ncclSend/ncclRecv in one group, the
 * own chunk by hipMemcpyAsync, the rebase by a kernel, all on the context's stream); a host that moves
 * the chunks another way (tests: torch.distributed gloo over host memory) supplies its own. Every
 * callback returns 0 or a negative errno. tag 0 = line bytes, 1 = records (a send of `bytes` bytes to
 * `peer` matches that peer's recv of the same tag from this rank). rebase: add peers[p].recv_byte0 to
 * the offset of records [recv_line0, +recv_lines) of every source p. */
typedef struct sr_transport {
    void *user;
    int (*group_start)(void *user);
    int (*group_end)(void *user);
    int (*send)(void *user, const void *buf, size_t bytes, int peer, int tag);
    int (*recv)(void *user, void *buf, size_t bytes, int peer, int tag);
    int (*copy)(void *user, void *dst, const void *src, size_t bytes);
    int (*rebase)(void *user, sr_record *recs, const sr_exchange_peer *peers, int world, uint64_t n_lines);
} sr_transport;

/* One exchange on a caller-supplied transport: sr_exchange_plan, then within one group_start/group_end
 * the sends and receives of every peer q != rank in rank order (bytes, then records; zero-sized ones
 * skipped), then the own chunk's copies, then one rebase of all received records. Buffers are whatever
 * the transport addresses (device memory for RCCL). Returns 0, -EINVAL or the first callback error. */
int sr_exchange_run(const sr_transport *t, int world, int rank, const uint64_t *h_sent,
                    const uint64_t *h_received, const uint8_t *packed, const sr_record *packed_recs,
                    uint8_t *recv_bytes, sr_record *recv_recs);

/* One route launch's whole regroup in one call, for the host loop that runs it every launch:
 * sr_pack_owner_sizes (n_owners = the comm's world), sr_exchange_sizes (the one host round trip),
 * sr_exchange_plan, then sr_pack_owner_scatter with the rank's own chunk written into its place in the
 * receive buffers and sr_exchange_data. Only the host work between the sizes arriving and the scatter's
 * launch stays on the critical path (no interpreter in between). h_sent / h_received (u64 [world][2])
 * hold the split sizes on return, also when the receive buffers are too small: then nothing is
 * scattered or sent and -ENOSPC is returned; the caller allocates the sizes' totals (sr_exchange_plan)
 * and finishes with sr_pack_owner_scatter and sr_exchange_data as above. packed_cap / d_packed_recs as
 * sr_pack_many_by_owner's out_cap / d_out_recs; recv_bytes_cap / recv_recs_cap in bytes / records.
 * Returns 0, -ENOSPC, -EINVAL, -ENOMEM, -EIO. Collective: every rank of the comm calls it. */
int sr_regroup_launch(sr_ctx *ctx, sr_comm *comm, const sr_batch *batches, size_t count,
                      uint64_t *d_owner_counts, uint64_t *d_recv_counts, uint8_t *d_packed, size_t packed_cap,
                      sr_record *d_packed_recs, uint8_t *d_recv_bytes, size_t recv_bytes_cap,
                      sr_record *d_recv_recs, size_t recv_recs_cap, uint64_t *h_sent, uint64_t *h_received);

/* sr_regroup_launch on any transport: the same sequence (split sizes, size exchange, plan, scatter with
 * the own chunk in place, exchange without the own chunk's copy, rebase) with `sizes` in place of
 * sr_exchange_sizes and `t` in place of RCCL; sr_regroup_launch is this call on RCCL. `sizes` gets t->user
 * and must leave h_sent / h_received (u64 [world][2]) valid and d_recv_counts written (ordered before
 * the context's later work) when it returns; it is collective like the transport. The device work of the
 * call is enqueued on the context's stream and not waited for: a transport that reads or writes device
 * buffers from the host first waits for that stream (sr_sync). Used to run the multi-rank sequence
 * without RCCL (ranks as threads on one GPU, or processes over gloo). Returns as sr_regroup_launch; after
 * -ENOSPC (the sizes exchanged, nothing scattered or sent: the peers' sends to this rank stay posted)
 * the caller finishes with sr_pack_owner_scatter (own = -1) and sr_exchange_run on the same transport. */
typedef int (*sr_sizes_fn)(void *user, const uint64_t *d_owner_counts, uint64_t *d_recv_counts, uint64_t *h_sent,
                           uint64_t *h_received);
int sr_regroup_run(sr_ctx *ctx, const sr_transport *t, sr_sizes_fn sizes, int world, int rank,
                   const sr_batch *batches, size_t count, uint64_t *d_owner_counts, uint64_t *d_recv_counts,
                   uint8_t *d_packed, size_t packed_cap, sr_record *d_packed_recs, uint8_t *d_recv_bytes,
                   size_t recv_bytes_cap, sr_record *d_recv_recs, size_t recv_recs_cap, uint64_t *h_sent,
                   uint64_t *h_received);

/* The rebase of sr_exchange_data alone (asynchronous on the context's stream): records
 * [peers[p].recv_line0, +recv_lines) of d_recv_recs move by peers[p].recv_byte0, p = 0..world-1.
 * world <= SR_MAX_OWNERS; the sources' record ranges must be back to back from 0. Returns 0, -EINVAL, -EIO. */
int sr_exchange_rebase(sr_ctx *ctx, sr_record *d_recv_recs, const sr_exchange_peer *peers, int world);

/* ---- per-downstream MTU packing ------------------------------------------ */
/* push_to_downstream (sr-main.c:73-83) appends each routed line to its downstream's active buffer,
 * flushing the buffer first when the line would not fit in DOWNSTREAM_BUF_SIZE (1450) bytes
 * (ds_schedule_flush, sr-main.c:49-71): per downstream a greedy packing of its lines in arrival
 * order, starting from the bytes already pending. sr_pack_packets computes it on the device.
 *
 * Records are first regrouped stably ("sorted"): the valid lines of downstream 0, 1, ..., N-1 in
 * arrival order, then every unrouted line (invalid length / format, all dead) in input order.
 * A packet is a run of consecutive sorted lines, led by `carry` bytes of the downstream's buffer
 * pending before the batch (only a downstream's first packet of the batch can have carry > 0).
 * Per downstream with lines in the batch: every packet the batch flushes (open = 0), in order,
 * then its new pending buffer (open = 1, last). Downstreams without lines get no descriptor; their
 * pending bytes carry over unchanged, except those probed dead, which are dropped (sr-main.c:106). */
typedef struct sr_packet {
    uint32_t first;   /* index in the sorted records of the packet's first line of this batch */
    uint16_t nlines;  /* lines of this batch in the packet                                   */
    uint16_t shard;   /* downstream                                                          */
    uint16_t length;  /* bytes of those lines                                                */
    uint16_t carry;   /* pending bytes from before the batch that lead the packet            */
    uint32_t open;    /* 1: the downstream's pending buffer after the batch (not flushed)    */
} sr_packet;

#define SR_MAX_PACK_DOWNSTREAMS 4096u
/* Descriptor room that always suffices (two consecutive flushed packets hold > 1450 bytes). */
#define SR_MAX_PACKETS(nbytes, n_downstreams) \
    (2u * (uint64_t)(nbytes) / SR_DOWNSTREAM_BUF_SIZE + 5u * (uint64_t)(n_downstreams) + 4u)

/* Device-resident packing of a routed batch (asynchronous on the context's stream):
 *   d_recs, d_n_records, max_records: the output of sr_route_device(_many) for the batch;
 *   d_fill_in  : NULL (nothing pending) or n_downstreams u16, pending bytes per downstream (<= 1450);
 *   d_probed_dead: NULL or the batch's probed-dead bitmap (sr_batch.d_probed_dead);
 *   d_sorted   : max_records records; d_packets: max_packets descriptors;
 *   d_counts   : 3 u64 = {descriptors, valid lines, lines} (descriptors past max_packets are not
 *                written: check d_counts[0] <= max_packets);
 *   d_fill_out : n_downstreams u16, pending bytes after the batch (may alias d_fill_in only if the
 *                caller does not need d_fill_in afterwards).
 * n_downstreams <= SR_MAX_PACK_DOWNSTREAMS. The first call (or one with a larger max_records)
 * allocates scratch: not inside stream capture. Returns 0, -EINVAL, -ENOMEM, -EIO. */
int sr_pack_packets(sr_ctx *ctx, const sr_record *d_recs, const uint64_t *d_n_records, size_t max_records,
                    const uint16_t *d_fill_in, const uint64_t *d_probed_dead, sr_record *d_sorted,
                    sr_packet *d_packets, size_t max_packets, uint64_t *d_counts, uint16_t *d_fill_out);

/* Several batches packed in one set of launches (the batches of several data threads, each with
 * its own pending bytes: batches are independent). Fields as in sr_pack_packets. count <=
 * SR_MAX_BATCHES_PER_LAUNCH. Same allocation rule as sr_pack_packets. */
typedef struct sr_pack_batch {
    const sr_record *d_recs;         /* routed records and their count (sr_route_device(_many))   */
    const uint64_t *d_n_records;
    size_t max_records;
    const uint16_t *d_fill_in;       /* NULL or n_downstreams u16                                 */
    const uint64_t *d_probed_dead;   /* NULL or the batch's probed-dead bitmap                    */
    sr_record *d_sorted;
    sr_packet *d_packets;
    size_t max_packets;
    uint64_t *d_counts;              /* 3 u64: {descriptors, valid lines, lines}                  */
    uint16_t *d_fill_out;
} sr_pack_batch;
int sr_pack_packets_many(sr_ctx *ctx, const sr_pack_batch *batches, size_t count);

/* Route and pack device-resident batches in one call: sr_route_device_many over `route` (one launch)
 * followed by sr_pack_packets_many over `pack`, whose batch i must read what route batch i writes
 * (pack[i].d_recs == route[i].d_out, same d_n_records, max_records and d_probed_dead; -EINVAL
 * otherwise). Identical outputs; with every shard alive and at most 16 downstreams the route kernel
 * also hands each 16 KiB tile's per-downstream line counts to the packing, which then sorts the
 * records without a counting pass of its own over them. count <= SR_MAX_BATCHES_PER_LAUNCH. */
int sr_route_pack_many(sr_ctx *ctx, const sr_batch *route, const sr_pack_batch *pack, size_t count);

/* Host-memory batch, routed and packed in one call (what a data thread's read callback needs):
 * `fill` (n_downstreams u16) is the pending bytes per downstream before the batch and receives the
 * pending bytes after it; `sorted` (max_records) the regrouped records; `packets` (max_packets) the
 * descriptors; probed_dead (ceil(n/64) words, may be NULL) the dead downstreams whose pending
 * buffer the batch drops. Synchronous: one stream synchronisation (sr_route_pack_submit /
 * sr_route_pack_result on a slot of its own). Returns 0, -ENOSPC (records or descriptors did not
 * fit: outputs incomplete), -EINVAL, -ENOMEM, -EIO. */
int sr_route_pack_batch(sr_ctx *ctx, const uint8_t *bytes, size_t nbytes, uint16_t *fill, sr_record *sorted,
                        size_t max_records, size_t *n_records, size_t *n_valid, sr_packet *packets,
                        size_t max_packets, size_t *n_packets, uint64_t *probed_dead);

/* sr_route_pack_batch in two halves, for a data thread that overlaps a batch's GPU work with its own
 * work on the previous batch (double buffering; reference: udp_read_cb, sr-main.c:149-191).
 * sr_route_pack_submit enqueues on the context's stream the copy of `bytes` to the device, the route,
 * the packing and one copy-out kernel that writes the batch's outputs (counts included) into
 * page-locked memory the context owns for slot `slot` (0 or 1), and returns without waiting.
 * fill: the pending bytes per downstream before the batch, or NULL to continue from the pending
 * bytes the previous submission (of either slot, or sr_route_pack_batch) leaves on the device, all
 * zero before the first: consecutive batches chain without a host round trip. `bytes` must stay
 * unchanged until the slot's result is taken. sr_route_pack_result waits for the slot (its one
 * synchronisation) and points *res at its outputs, valid until the slot is submitted again.
 * A slot holds one batch at a time. Returns 0, -EBUSY (slot in use / not submitted), -ENOSPC
 * (result: records or descriptors did not fit), -EINVAL, -ENOMEM, -EIO. */
typedef struct sr_pack_result {
    const sr_record *sorted;      /* n_records: valid lines by downstream, then the unrouted lines */
    size_t n_records, n_valid;
    const sr_packet *packets;     /* n_packets descriptors (sr_pack_packets)                       */
    size_t n_packets;
    const uint16_t *fill;         /* n_downstreams: pending bytes after the batch                  */
    const uint64_t *probed_dead;  /* ceil(n_downstreams/64) words (sr-main.c:106)                  */
} sr_pack_result;
int sr_route_pack_submit(sr_ctx *ctx, int slot, const uint8_t *bytes, size_t nbytes, const uint16_t *fill);
int sr_route_pack_result(sr_ctx *ctx, int slot, sr_pack_result *res);

/* TRACE logging (log_level 0, the reference's default: sr-init.c:252). The reference logs, per line
 * that reaches find_downstream, its sdbm hash and its first live pick (sr-main.c:91,102), so a router
 * at that level needs every line's verdict, hash and shard in INPUT order. With sr_set_trace(ctx, 1)
 * every later sr_route_pack_submit / sr_route_pack_batch also has the route kernel write each line's
 * hash (0 for lines that fail the length or ':' test) and the copy-out kernel return the records in
 * input order with the hashes; sr_route_pack_trace points at them after sr_route_pack_result(slot),
 * valid until the slot is submitted again (slot 2: the last sr_route_pack_batch). Off by default: it
 * costs 16 bytes per line of PCIe and host memory. Returns 0, -EINVAL, -EBUSY (not traced). */
int sr_set_trace(sr_ctx *ctx, int on);
int sr_route_pack_trace(sr_ctx *ctx, int slot, const sr_record **records, const uint64_t **hashes,
                        size_t *n_records);

/* Developer and test knobs of one context (A/B runs and tests only; the library reads no environment
 * variable and no knob changes any record, packet or count, only which kernels produce them):
 *   SR_KNOB_LB_SPIN       polls of a predecessor tile's tail granules before route_chunk_kernel
 *                         computes the straddling line itself (default 65536; 0 always computes it);
 *   SR_KNOB_DEFER_PICKS   first picks the route kernel makes before deferring a probe when two or
 *                         more shards are dead (1 default, or 2);
 *   SR_KNOB_MTU_CHUNK     packing chunk lines: 0 = by the launch's shape (default), 2048 or 4608;
 *   SR_KNOB_MTU_XCD       1 (default): batches' packing chunks on one XCD from eight batches up;
 *   SR_KNOB_MTU_WALK      1 (default): the chain walked inside mtu_emit up to 64 shards; 0: mtu_chain;
 *   SR_KNOB_HIST          1 (default): sr_route_pack_many / sr_route_pack_* hand the route kernel's tile
 *                         histograms to the packing; 0: the packing counts the records itself;
 *   SR_KNOB_PREFETCH      tiles ahead (default 96; 0 off; up to 4096) whose 128-byte lines a chunk-layout
 *                         tile workgroup touches after issuing its own loads (an L2 / memory-side cache
 *                         warm-up for the tile its XCD runs later);
 *   SR_KNOB_FUSE_DEFER    1: a route + pack launch with two or more (at most 16) dead shards leaves its
 *                         deferred probes to the packing's counting pass; 0 (default): probe_defer_kernel
 *                         (measured level on C3 / C5, slower on C4).
 * Returns 0 or -EINVAL (unknown knob or value). */
#define SR_KNOB_LB_SPIN 1
#define SR_KNOB_DEFER_PICKS 2
#define SR_KNOB_MTU_CHUNK 3
#define SR_KNOB_MTU_XCD 4
#define SR_KNOB_MTU_WALK 5
#define SR_KNOB_HIST 7
#define SR_KNOB_PREFETCH 8
#define SR_KNOB_FUSE_DEFER 9
int sr_set_knob(sr_ctx *ctx, int knob, int64_t value);

/* Page-locked host memory for the batches and outputs of the host-memory calls (their copies then
 * run at full link rate). NULL on failure. */
void *sr_alloc_host(size_t bytes);
void sr_free_host(void *p);

/* Wait for all work enqueued by this context. */
int sr_sync(sr_ctx *ctx);

void sr_close(sr_ctx *ctx);

/* Version / build information string (static storage). */
const char *sr_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SR_ROUTE_H */
