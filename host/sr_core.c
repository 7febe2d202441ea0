/*
 * sr_core.c — one data thread of the MI355X statsd-router (include/sr_router.h).
 *
 * Per batch of framed datagrams the GPU does the per-line work and the per-downstream packing
 * (sr_route_pack_batch: tokenise, length / ':' verdict, sdbm hash, shard pick, greedy 1450-byte
 * packets); this file keeps the reference's host-side state and side effects:
 *   - the pending (active) buffer of every downstream and its traffic / packet counters
 *     (downstream_s, sr-types.h:36-63);
 *   - the flush of a packet: counters, then the bytes to the emit callback (ds_schedule_flush,
 *     sr-main.c:49-71; the send itself, ds_flush_cb :21-46, is the caller's);
 *   - the drop of a probed dead downstream's pending buffer (find_downstream, sr-main.c:106);
 *   - the WARN lines with the reference's texts (sr-main.c:115,142,184) and, at log_level 0, the
 *     TRACE lines (sr-main.c:91,102,174) in input order, from the GPU's per-line hashes;
 *   - the flush timer (ds_flush_timer_cb, :194-204) and the self-metrics (ping_cb, :206-235), whose
 *     few lines are routed on the GPU too and appended here with push_to_downstream's rule (:73-83).
 * There is no CPU routing path: the shard of every line, data or ping, comes from the GPU.
 */
#include "../include/sr_router.h"

#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct ds_state {
    uint8_t pending[SR_DOWNSTREAM_BUF_SIZE]; /* active buffer (sr-types.h:40-41) */
    uint32_t fill;                           /* active_buffer_length            */
    int32_t traffic, packets;                /* sr-types.h:52,54                */
    char conn_metric[SR_METRIC_SIZE];        /* per_downstream_counter_metric   */
    int conn_len;
    char traffic_metric[SR_METRIC_SIZE];
    char packet_metric[SR_METRIC_SIZE];
} ds_state;

struct sr_core {
    sr_ctx *ctx;
    uint32_t n, nwords;
    int log_level;
    ds_state *ds;
    uint64_t *alive;
    char alive_metric[SR_METRIC_SIZE];
    sr_core_emit_fn emit;
    sr_core_log_fn log;
    sr_core_flush_fn flush;
    void *user;
    /* per-batch buffers (page-locked) */
    size_t max_batch;
    uint8_t *in[2];                          /* the two slots' framed datagrams                 */
    const uint8_t *in_flight_bytes;          /* the framed bytes of the batch in flight          */
    size_t in_flight_len;
    int in_flight;                           /* slot whose batch is on the GPU, or -1            */
    unsigned fail_submit, submits;           /* fault injection (sr_core_inject_faults, tests)   */
    unsigned fail_finish, finishes;
    int trace;                               /* log_level TRACE: per-line hashes from the GPU     */
    uint32_t *dg_ends[2];                    /* TRACE: datagram ends of the batch in each slot    */
    size_t dg_n[2], dg_cap[2];
    uint64_t *ping_hash;                     /* TRACE: the ping names' hashes                      */
    int host_fills;                          /* the host changed pending buffers since the last  */
                                             /* submission: upload them with the next one         */
    uint16_t *fill16;
    sr_record *sorted;                       /* the ping names' records (sr_route_batch)         */
    size_t sorted_cap;
    uint64_t *probed;
    struct iovec *iov;
    char *msg;
    size_t msg_cap;
    uint8_t *ping;                           /* the ping names routed by sr_core_ping */
    size_t ping_cap;
};

static void core_log(sr_core *c, int level, const char *fmt, ...) __attribute__((format(printf, 3, 4)));
static void core_log(sr_core *c, int level, const char *fmt, ...) {
    if (level < c->log_level || !c->log) return;
    va_list ap;
    va_start(ap, fmt);
    int n = vsnprintf(c->msg, c->msg_cap, fmt, ap);
    va_end(ap);
    if (n < 0) return;
    if ((size_t)n >= c->msg_cap) n = (int)c->msg_cap - 1;
    c->log(c->user, level, c->msg, (size_t)n);
}

/* ds_schedule_flush (sr-main.c:49-71): count the packet, hand the pending buffer over, start a new one */
static void schedule_flush(sr_core *c, uint32_t s) {
    ds_state *d = &c->ds[s];
    d->packets += 1;                                               /* :61 */
    d->traffic = (int32_t)((uint32_t)d->traffic + d->fill);        /* :62 */
    struct iovec v = {d->pending, d->fill};
    c->emit(c->user, s, &v, 1, d->fill);
    d->fill = 0;                                                   /* :65 */
}

/* push_to_downstream (sr-main.c:73-83) for the host-side lines (ping) */
static void push(sr_core *c, uint32_t s, const char *line, size_t len) {
    ds_state *d = &c->ds[s];
    if (d->fill + len > SR_DOWNSTREAM_BUF_SIZE) schedule_flush(c, s); /* :75-78 */
    memcpy(d->pending + d->fill, line, len);                         /* :80    */
    d->fill += (uint32_t)len;                                        /* :82    */
}

static int alive_bit(const sr_core *c, uint32_t k) { return (int)((c->alive[k >> 6] >> (k & 63)) & 1u); }

static void build_names(sr_core *c, const sr_core_config *cfg) {
    /* sr-init.c:57: "%s.%s-%d.%s" prefix, hostname, data_port + thread, "healthy_downstreams" */
    snprintf(c->alive_metric, SR_METRIC_SIZE, "%s.%s-%d.%s", cfg->ping_prefix, cfg->hostname, cfg->data_port,
             "healthy_downstreams");
    /* sr-init.c:90-96: the host with '.' -> '_' written over ONE buffer shared by all downstreams and
     * never terminated, so a shorter host keeps the tail of a longer previous one (the reference's
     * buffer starts as stack garbage; zeros here) */
    char mh[SR_METRIC_SIZE];
    memset(mh, 0, sizeof(mh));
    for (uint32_t i = 0; i < c->n; i++) {
        const char *h = cfg->ds_hosts[i], *port = cfg->ds_data_ports[i];
        for (size_t j = 0; h[j] && j < SR_METRIC_SIZE - 1; j++) mh[j] = h[j] == '.' ? '_' : h[j];
        ds_state *d = &c->ds[i];
        /* sr-init.c:112-118 */
        d->conn_len = snprintf(d->conn_metric, SR_METRIC_SIZE, "%s.%s-%d-%s-%s.%s\n%s.%s-%s.%s\n", cfg->ping_prefix,
                               cfg->hostname, cfg->data_port, mh, port, "connections:1|c", cfg->ping_prefix, mh, port,
                               "connections:1|c");
        if (d->conn_len >= (int)SR_METRIC_SIZE) d->conn_len = SR_METRIC_SIZE - 1;
        snprintf(d->packet_metric, SR_METRIC_SIZE, "%s.%s-%s.%s", cfg->ping_prefix, mh, port, "packets");
        snprintf(d->traffic_metric, SR_METRIC_SIZE, "%s.%s-%s.%s", cfg->ping_prefix, mh, port, "traffic");
    }
}

void sr_core_close(sr_core *c) {
    if (!c) return;
    if (c->ctx) sr_close(c->ctx);
    sr_free_host(c->in[0]);
    sr_free_host(c->in[1]);
    sr_free_host(c->sorted);
    free(c->fill16);
    free(c->probed);
    free(c->iov);
    free(c->msg);
    free(c->ping);
    free(c->ping_hash);
    free(c->dg_ends[0]);
    free(c->dg_ends[1]);
    free(c->alive);
    free(c->ds);
    free(c);
}

int sr_core_open(sr_core **out, const sr_core_config *cfg, sr_core_emit_fn emit, sr_core_log_fn log,
                 sr_core_flush_fn flush, void *user) {
    if (!out || !cfg || !emit || cfg->max_batch_bytes == 0) return -EINVAL;
    if (cfg->n_downstreams == 0 || cfg->n_downstreams > SR_MAX_PACK_DOWNSTREAMS) return -EINVAL;
    if (!cfg->ds_hosts || !cfg->ds_data_ports || !cfg->ping_prefix || !cfg->hostname) return -EINVAL;
    *out = NULL;
    sr_core *c = calloc(1, sizeof(*c));
    if (!c) return -ENOMEM;
    c->n = cfg->n_downstreams;
    c->nwords = (c->n + 63) / 64;
    c->log_level = cfg->log_level;
    c->emit = emit;
    c->log = log;
    c->flush = flush;
    c->user = user;
    c->max_batch = cfg->max_batch_bytes;
    int rc = sr_open(&c->ctx, cfg->device, cfg->max_batch_bytes, c->n);
    if (rc) {
        sr_core_close(c);
        return rc;
    }
    c->in_flight = -1;
    c->host_fills = 1;
    /* TRACE (sr-init.c:252 default): every line's hash from the route kernel, records in input order */
    c->trace = c->log_level <= SR_TRACE && c->log != NULL;
    if (c->trace && (rc = sr_set_trace(c->ctx, 1))) {
        sr_core_close(c);
        return rc;
    }
    c->msg_cap = 3 * SR_DATA_BUF_SIZE;
    c->ds = calloc(c->n, sizeof(ds_state));
    c->alive = calloc(c->nwords, sizeof(uint64_t));
    c->fill16 = calloc(c->n, sizeof(uint16_t));
    c->probed = calloc(c->nwords, sizeof(uint64_t));
    c->iov = calloc(SR_DOWNSTREAM_BUF_SIZE + 2, sizeof(struct iovec));
    c->msg = malloc(c->msg_cap);
    c->ping_cap = ((size_t)c->n + 1) * (SR_METRIC_SIZE + 8);
    c->ping = malloc(c->ping_cap);
    c->sorted_cap = (size_t)c->n + 1;   /* the ping batch: one line per name */
    c->in[0] = sr_alloc_host(cfg->max_batch_bytes);
    c->in[1] = sr_alloc_host(cfg->max_batch_bytes);
    c->sorted = sr_alloc_host(c->sorted_cap * sizeof(sr_record));
    c->ping_hash = calloc(c->sorted_cap, sizeof(uint64_t));
    if (!c->ds || !c->alive || !c->fill16 || !c->probed || !c->iov || !c->msg || !c->ping || !c->in[0] ||
        !c->in[1] || !c->sorted || !c->ping_hash) {
        sr_core_close(c);
        return -ENOMEM;
    }
    /* every health client starts dead (sr-init.c:85) */
    if ((rc = sr_set_alive(c->ctx, c->alive))) {
        sr_core_close(c);
        return rc;
    }
    /* both slots' buffers allocated now (an empty batch each), not while the socket fills */
    for (int k = 0; k < 2; k++) {
        sr_pack_result r;
        if ((rc = sr_route_pack_submit(c->ctx, k, NULL, 0, c->fill16)) || (rc = sr_route_pack_result(c->ctx, k, &r))) {
            sr_core_close(c);
            return rc;
        }
    }
    build_names(c, cfg);
    *out = c;
    return 0;
}

int sr_core_set_alive(sr_core *c, const uint64_t *alive) {
    if (!c || !alive) return -EINVAL;
    int rc = sr_core_drain(c);
    if (rc) return rc;
    memcpy(c->alive, alive, c->nwords * sizeof(uint64_t));
    if (c->n & 63) c->alive[c->nwords - 1] &= (1ull << (c->n & 63)) - 1;
    return sr_set_alive(c->ctx, c->alive);
}

uint8_t *sr_core_batch_buffer(sr_core *c, size_t *cap) { return sr_core_slot_buffer(c, 0, cap); }

uint8_t *sr_core_slot_buffer(sr_core *c, int slot, size_t *cap) {
    if (!c || slot < 0 || slot > 1) return NULL;
    if (cap) *cap = c->max_batch;
    return c->in[slot];
}

static void drop_probed(sr_core *c) {
    /* find_downstream zeroes the active buffer of each dead downstream it probes (sr-main.c:106) */
    for (uint32_t w = 0; w < c->nwords; w++)
        for (uint64_t m = c->probed[w]; m; m &= m - 1) c->ds[w * 64 + (uint32_t)__builtin_ctzll(m)].fill = 0;
}

/* The WARN line of an unrouted record, with the reference's text. */
static void warn_line(sr_core *c, const uint8_t *framed, const sr_record *r) {
    const char *line = (const char *)framed + r->offset;
    const int len = r->length;
    if (r->route == SR_ROUTE_INVALID_LENGTH) {
        /* sr-main.c:184 */
        core_log(c, SR_WARN, "%s: invalid length %d of metric %.*s", "udp_read_cb", len, len, line);
    } else if (r->route == SR_ROUTE_INVALID_FORMAT) {
        /* sr-main.c:141-142: the '\n' becomes NUL and the line is printed with %s */
        core_log(c, SR_WARN, "%s: invalid metric %.*s", "process_data_line", len - 1, line);
    } else {
        core_log(c, SR_WARN, "%s: all downstreams are dead", "find_downstream"); /* sr-main.c:115 */
    }
}

/* find_downstream's TRACE lines for a line that passed the length and ':' tests (sr-main.c:91,102):
 * its hash, then its first live pick, or the WARN when every downstream is dead (:115). */
static void trace_line(sr_core *c, const char *line, int len, uint64_t h, uint32_t route) {
    core_log(c, SR_TRACE, "%s: hash = %lx, length = %d, line = %.*s", "find_downstream", (unsigned long)h, len, len,
             line);
    if (route < c->n) core_log(c, SR_TRACE, "%s: pushing to downstream %d", "find_downstream", (int)route);
    else core_log(c, SR_WARN, "%s: all downstreams are dead", "find_downstream");
}

/* TRACE: every message of udp_read_cb for the batch in slot `slot`, in input order: per datagram
 * "got packet" (sr-main.c:174), then per line its WARN (:142,184) or its find_downstream lines. */
static int trace_batch(sr_core *c, int slot, const uint8_t *framed, size_t nbytes) {
    const sr_record *rec;
    const uint64_t *hs;
    size_t n = 0, i = 0, d0 = 0;
    int rc = sr_route_pack_trace(c->ctx, slot, &rec, &hs, &n);
    if (rc) {
        core_log(c, SR_ERROR, "%s: sr_route_pack_trace() failed %s", "udp_read_cb", strerror(-rc));
        c->dg_n[slot] = 0;
        return rc;
    }
    const size_t nd = c->dg_n[slot];
    for (size_t g = 0; g <= nd; g++) {   /* the datagrams, then whatever no boundary covers */
        const size_t end = g < nd ? c->dg_ends[slot][g] : nbytes;
        if (g < nd)
            core_log(c, SR_TRACE, "%s: got packet %.*s", "udp_read_cb", (int)(end - d0), (const char *)framed + d0);
        for (; i < n && (g == nd || rec[i].offset < end); i++) {
            if (rec[i].route == SR_ROUTE_INVALID_LENGTH || rec[i].route == SR_ROUTE_INVALID_FORMAT)
                warn_line(c, framed, &rec[i]);
            else
                trace_line(c, (const char *)framed + rec[i].offset, rec[i].length, hs[i], rec[i].route);
        }
        d0 = end;
    }
    c->dg_n[slot] = 0;
    return 0;
}

/* The host's half of a batch (udp_read_cb's per-line side effects, sr-main.c:175-189, for a whole
 * batch): drop probed dead buffers, the log lines in input order, then the packets per downstream. */
static void complete(sr_core *c, int slot, const uint8_t *framed, size_t nbytes, const sr_pack_result *r) {
    memcpy(c->probed, r->probed_dead, c->nwords * sizeof(uint64_t));
    drop_probed(c);
    /* without the TRACE inputs (the slot was not traced) the WARN lines still come, from the sorted
     * records' unrouted tail, in input order */
    if ((!c->trace || trace_batch(c, slot, framed, nbytes) != 0) && c->log_level <= SR_WARN)
        for (size_t i = r->n_valid; i < r->n_records; i++) warn_line(c, framed, &r->sorted[i]);
    for (size_t q = 0; q < r->n_packets; q++) {
        const sr_packet *p = &r->packets[q];
        ds_state *d = &c->ds[p->shard];
        const sr_record *rec = r->sorted + p->first;
        if (p->open) {
            /* the new active buffer: the carried bytes (already in place) + this batch's lines */
            uint32_t f = p->carry;
            for (uint32_t k = 0; k < p->nlines; k++) {
                memcpy(d->pending + f, framed + rec[k].offset, rec[k].length);
                f += rec[k].length;
            }
            d->fill = f;
            continue;
        }
        int iv = 0;
        if (p->carry) c->iov[iv++] = (struct iovec){d->pending, p->carry};
        for (uint32_t k = 0; k < p->nlines; k++)
            c->iov[iv++] = (struct iovec){(void *)(framed + rec[k].offset), rec[k].length};
        const uint32_t bytes = (uint32_t)p->carry + p->length;
        d->packets += 1;
        d->traffic = (int32_t)((uint32_t)d->traffic + bytes);
        c->emit(c->user, p->shard, c->iov, iv, bytes);
        d->fill = 0;
    }
    if (c->flush) c->flush(c->user);
}

/* Start a batch on the GPU; the pending bytes are the device's own unless the host changed them. */
static int submit(sr_core *c, int slot, const uint8_t *framed, size_t nbytes) {
    const uint16_t *fill = NULL;
    if (c->host_fills) {   /* nothing is in flight here: the host's fills are current */
        for (uint32_t s = 0; s < c->n; s++) c->fill16[s] = (uint16_t)c->ds[s].fill;
        fill = c->fill16;
    }
    int rc = sr_route_pack_submit(c->ctx, slot, framed, nbytes, fill);
    if (rc) return rc;
    c->host_fills = 0;
    return 0;
}

static int finish(sr_core *c, int slot, const uint8_t *framed, size_t nbytes) {
    sr_pack_result r;
    int rc = sr_route_pack_result(c->ctx, slot, &r);
    if (!rc && c->fail_finish && ++c->finishes == c->fail_finish) rc = -EIO;   /* fault injection */
    if (rc) {
        c->host_fills = 1;   /* the device's chain is no longer what the host holds */
        c->dg_n[slot] = 0;
        return rc;
    }
    complete(c, slot, framed, nbytes, &r);
    return 0;
}

int sr_core_drain(sr_core *c) {
    if (!c) return -EINVAL;
    if (c->in_flight < 0) return 0;
    const int slot = c->in_flight;
    c->in_flight = -1;
    return finish(c, slot, c->in_flight_bytes, c->in_flight_len);
}

/* TRACE: the datagram ends of the batch about to go into `slot` (copied) */
static int note_datagrams(sr_core *c, int slot, const uint32_t *ends, size_t n) {
    c->dg_n[slot] = 0;
    if (!c->trace || !n) return 0;
    if (!ends) return -EINVAL;
    if (n > c->dg_cap[slot]) {
        uint32_t *p = realloc(c->dg_ends[slot], n * sizeof(uint32_t));
        if (!p) return -ENOMEM;
        c->dg_ends[slot] = p;
        c->dg_cap[slot] = n;
    }
    memcpy(c->dg_ends[slot], ends, n * sizeof(uint32_t));
    c->dg_n[slot] = n;
    return 0;
}

int sr_core_submit_datagrams(sr_core *c, int slot, size_t nbytes, const uint32_t *ends, size_t n_datagrams) {
    if (!c || slot < 0 || slot > 1 || nbytes > c->max_batch) return -EINVAL;
    if (c->in_flight == slot) return -EBUSY;
    if (nbytes == 0) return 0;
    if (c->fail_submit && ++c->submits == c->fail_submit) return -EIO;   /* as a failed sr_route_pack_submit */
    int rc = note_datagrams(c, slot, ends, n_datagrams);
    if (rc) return rc;
    if ((rc = submit(c, slot, c->in[slot], nbytes))) {
        c->dg_n[slot] = 0;
        return rc;   /* nothing submitted: sr_core_in_flight() is not `slot` */
    }
    const int prev = c->in_flight;
    const uint8_t *prev_bytes = c->in_flight_bytes;
    const size_t prev_len = c->in_flight_len;
    c->in_flight = slot;
    c->in_flight_bytes = c->in[slot];
    c->in_flight_len = nbytes;
    if (prev < 0) return 0;
    if ((rc = finish(c, prev, prev_bytes, prev_len)) == 0) return 0;
    /* The previous batch failed, so its packets never reached the pending buffers the new batch's
     * device-chained fills assume: take the new batch back and route it again from the host's fills
     * (finish() set host_fills), so that host and device agree on every pending buffer. */
    sr_pack_result r;
    const int rc_back = sr_route_pack_result(c->ctx, slot, &r);
    if (rc_back && rc_back != -ENOSPC)
        core_log(c, SR_ERROR, "%s: taking back the batch after a failed one failed %s", "udp_read_cb",
                 strerror(-rc_back));
    c->in_flight = -1;
    if (submit(c, slot, c->in[slot], nbytes) == 0) c->in_flight = slot;   /* (its datagram ends kept) */
    else c->dg_n[slot] = 0;
    return rc;
}

int sr_core_submit(sr_core *c, int slot, size_t nbytes) { return sr_core_submit_datagrams(c, slot, nbytes, NULL, 0); }

int sr_core_in_flight(const sr_core *c) { return c ? c->in_flight : -EINVAL; }

int sr_core_route_datagrams(sr_core *c, const uint8_t *framed, size_t nbytes, const uint32_t *ends,
                            size_t n_datagrams) {
    if (!c || (nbytes && !framed) || nbytes > c->max_batch) return -EINVAL;
    int rc = sr_core_drain(c);
    if (rc) return rc;
    if (nbytes == 0) return 0;
    if ((rc = note_datagrams(c, 0, ends, n_datagrams))) return rc;
    if ((rc = submit(c, 0, framed, nbytes))) {
        c->dg_n[0] = 0;
        return rc;
    }
    return finish(c, 0, framed, nbytes);
}

int sr_core_route(sr_core *c, const uint8_t *framed, size_t nbytes) {
    return sr_core_route_datagrams(c, framed, nbytes, NULL, 0);
}

sr_ctx *sr_core_context(sr_core *c) { return c ? c->ctx : NULL; }

int sr_core_inject_faults(sr_core *c, unsigned fail_submit, unsigned fail_finish) {
    if (!c) return -EINVAL;
    c->fail_submit = fail_submit;
    c->fail_finish = fail_finish;
    c->submits = c->finishes = 0;
    return 0;
}

int sr_core_flush_timer(sr_core *c) {
    if (!c) return -EINVAL;
    int rc = sr_core_drain(c);
    if (rc) return rc;
    c->host_fills = 1;
    for (uint32_t s = 0; s < c->n; s++)
        if (c->ds[s].fill > 0) schedule_flush(c, s); /* sr-main.c:199-203 */
    if (c->flush) c->flush(c->user);
    return 0;
}

int sr_core_ping(sr_core *c) {
    if (!c) return -EINVAL;
    int rc = sr_core_drain(c);
    if (rc) return rc;
    c->host_fills = 1;
    /* The shard of a ping line depends only on its name (the bytes before ':') and the alive bits,
     * so the n + 1 names are routed on the GPU in one batch first; the texts, whose counters change
     * as earlier lines are pushed, are formatted afterwards in the reference's order. */
    size_t pos = 0;
    uint8_t *b = c->ping;
    for (uint32_t i = 0; i <= c->n; i++) {
        const char *name = i < c->n ? c->ds[i].traffic_metric : c->alive_metric;
        int k = snprintf((char *)b + pos, c->ping_cap - pos, "%s:0|%c\n", name, i < c->n ? 'c' : 'g');
        if (k < 0 || pos + (size_t)k >= c->ping_cap) return -ENOSPC;
        pos += (size_t)k;
    }
    if (pos > c->max_batch) return -ENOSPC;
    size_t nr = 0;
    rc = sr_route_batch(c->ctx, b, pos, c->sorted, c->sorted_cap, &nr, c->trace ? c->ping_hash : NULL);
    if (rc) return rc;
    if (nr != c->n + 1) return -EIO;
    if ((rc = sr_last_probed_dead(c->ctx, c->probed))) return rc;
    drop_probed(c); /* only dead downstreams: none of them receives a ping line */
    char buf[2 * SR_METRIC_SIZE + 64];
    int count = 0;
    for (uint32_t i = 0; i < c->n; i++) {
        ds_state *d = &c->ds[i];
        if (alive_bit(c, i)) { /* sr-main.c:220-223 */
            push(c, i, d->conn_metric, (size_t)d->conn_len);
            count++;
        }
        const int32_t traffic = d->traffic, packets = d->packets; /* :224-227 */
        d->traffic = 0;
        d->packets = 0;
        const int n = snprintf(buf, sizeof(buf), "%s:%d|c\n%s:%d|c\n", d->traffic_metric, traffic, d->packet_metric,
                               packets);
        const uint16_t route = c->sorted[i].route; /* process_data_line, :231 */
        if (c->trace) trace_line(c, buf, n, c->ping_hash[i], route);
        else if (route >= c->n) core_log(c, SR_WARN, "%s: all downstreams are dead", "find_downstream");
        if (route < c->n) push(c, route, buf, (size_t)n);
    }
    const int n = snprintf(buf, sizeof(buf), "%s:%d|g\n", c->alive_metric, count); /* :233-234 */
    const uint16_t route = c->sorted[c->n].route;
    if (c->trace) trace_line(c, buf, n, c->ping_hash[c->n], route);
    else if (route >= c->n) core_log(c, SR_WARN, "%s: all downstreams are dead", "find_downstream");
    if (route < c->n) push(c, route, buf, (size_t)n);
    if (c->flush) c->flush(c->user);
    return 0;
}

int sr_core_state(const sr_core *c, uint32_t s, const uint8_t **pending, size_t *len, int32_t *traffic,
                  int32_t *packets) {
    if (!c || s >= c->n) return -EINVAL;
    if (pending) *pending = c->ds[s].pending;
    if (len) *len = c->ds[s].fill;
    if (traffic) *traffic = c->ds[s].traffic;
    if (packets) *packets = c->ds[s].packets;
    return 0;
}

const char *sr_core_metric_name(const sr_core *c, uint32_t s, int which) {
    if (!c) return NULL;
    if (which == 3) return c->alive_metric;
    if (s >= c->n) return NULL;
    return which == 0 ? c->ds[s].conn_metric : which == 1 ? c->ds[s].traffic_metric : c->ds[s].packet_metric;
}
