/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of statsd-router's per-datagram hot path, written from scratch to the
 * semantics of the reference (hulu/statsd-router v0.0.16, /root/reference). It is the parity
 * checker for the HIP path (tests/, __graft_entry__.smoke()) and the CPU baseline timed by
 * bench.py's cpu_baseline leg ("kind": "port"). Nothing in the product (statsd-router_amd/)
 * links, loads or calls it.
 *
 * Pinned against the compiled reference (oracle/_ref, built by oracle/Makefile from the
 * reference's own sources) by tests/golden/make_golden.py; the committed fixtures in
 * tests/golden/ are the reference's outputs.
 *
 * Structure deliberately follows the reference's serial loop (memchr per line, one dependent
 * 64-bit multiply-add per name byte, VLA shuffle per routed line) so that its timing is a fair
 * stand-in for the reference C path.
 */
#include "sr_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* sr-main.c:163-173 — recv(fd, buffer, DATA_BUF_SIZE - 1, 0); append '\n' if missing. */
size_t sro_frame_datagram(uint8_t *dst, const uint8_t *src, size_t len) {
    size_t n = len < SR_MAX_DATAGRAM ? len : SR_MAX_DATAGRAM;
    if (n == 0) return 0; /* sr-main.c:170: an empty datagram yields no lines */
    memcpy(dst, src, n);
    if (dst[n - 1] != '\n') dst[n++] = '\n';
    return n;
}

/* sr-main.c:119-134 — sdbm over the bytes before the first ':'. `char` is signed on the
 * reference's x86-64 build (sr-main.c:122), h is `unsigned long` (64 bit, wraps).
 * Returns 0 and *out when a ':' exists, else 1 (*out untouched). */
int sro_hash(const uint8_t *s, size_t length, uint64_t *out) {
    uint64_t h = 0;
    for (size_t i = 0; i < length; i++) {
        int8_t c = (int8_t)s[i];
        if (c == ':') {
            *out = h;
            return 0;
        }
        h = (h << 6) + (h << 16) - h + (uint64_t)(int64_t)c; /* sr-main.c:131 */
    }
    return 1;
}

static inline int alive_bit(const uint64_t *alive, uint32_t k) {
    return (int)((alive[k >> 6] >> (k & 63)) & 1u);
}

/* sr-main.c:85-117 — hash-seeded partial Fisher-Yates probe over the downstream list.
 * Returns the chosen downstream, or -1 ("all downstreams are dead"). */
int sro_find_downstream(uint64_t hash, uint32_t downstream_num, const uint64_t *alive) {
    if (downstream_num == 0) return -1;
    int ds_index[downstream_num]; /* sr-main.c:88 (VLA) */
    for (uint32_t i = 0; i < downstream_num; i++) ds_index[i] = (int)i; /* :93-95 */
    for (uint32_t i = downstream_num; i > 0; i--) {                     /* :97 */
        uint32_t j = (uint32_t)(hash % i);                              /* :98 */
        int k = ds_index[j];                                           /* :99 */
        if (alive_bit(alive, (uint32_t)k)) return k;                   /* :101-104 */
        if (j != i - 1) {                                              /* :108-111 */
            ds_index[j] = ds_index[i - 1];
            ds_index[i - 1] = k;
        }
        hash = (hash * 7 + 5) / 3; /* :113, u64 wrap before the division */
    }
    return -1; /* :115-116 */
}

/* find_downstream with its dead-downstream side effect recorded: every dead downstream k the
 * probe visits gets active_buffer_length = 0 in the reference (sr-main.c:106); bit k of probed. */
static int find_downstream_probed(uint64_t hash, uint32_t downstream_num, const uint64_t *alive,
                                  uint64_t *probed) {
    if (downstream_num == 0) return -1;
    int ds_index[downstream_num];
    for (uint32_t i = 0; i < downstream_num; i++) ds_index[i] = (int)i;
    for (uint32_t i = downstream_num; i > 0; i--) {
        uint32_t j = (uint32_t)(hash % i);
        int k = ds_index[j];
        if (alive_bit(alive, (uint32_t)k)) return k;
        probed[k >> 6] |= 1ull << (k & 63); /* :106 */
        if (j != i - 1) {
            ds_index[j] = ds_index[i - 1];
            ds_index[i - 1] = k;
        }
        hash = (hash * 7 + 5) / 3;
    }
    return -1;
}

/* The batch's probed-dead bitmap (ceil(n/64) words, zeroed here): the dead downstreams whose
 * pending buffer the reference drops while routing the batch (sr-main.c:106). */
void sro_probed_dead(const uint8_t *buf, size_t nbytes, uint32_t downstream_num,
                     const uint64_t *alive, uint64_t *probed) {
    memset(probed, 0, ((downstream_num + 63) / 64) * sizeof(uint64_t));
    const uint8_t *ptr = buf, *delim;
    size_t rem = nbytes;
    while (rem > 0 && (delim = memchr(ptr, '\n', rem)) != NULL) {
        size_t len = (size_t)(delim + 1 - ptr);
        uint64_t h;
        if (len > 5 && len < SR_DOWNSTREAM_BUF_SIZE && sro_hash(ptr, len, &h) == 0)
            (void)find_downstream_probed(h, downstream_num, alive, probed);
        ptr = delim + 1;
        rem -= len;
    }
}

/* push_to_downstream (sr-main.c:73-83) + the flush it triggers (ds_schedule_flush, :49-71) over a
 * routed batch, in the descriptor form of sr_pack_packets (include/sr_route.h): per downstream, in
 * arrival order, a line that would overflow the DOWNSTREAM_BUF_SIZE buffer first flushes it.
 * Returns 0, or -1 if max_packets is too small. */
int sro_pack_packets(const sr_record *recs, size_t n, uint32_t nds, const uint16_t *fill_in,
                     const uint64_t *probed_dead, sr_record *sorted, sr_packet *packets,
                     size_t max_packets, size_t *n_packets, size_t *n_valid, uint16_t *fill_out) {
    size_t *start = calloc((size_t)nds + 2, sizeof(size_t));
    if (!start) return -1;
    for (size_t i = 0; i < n; i++) start[(recs[i].route < nds ? recs[i].route : nds) + 1]++;
    for (uint32_t k = 0; k <= nds; k++) start[k + 1] += start[k];
    size_t *pos = calloc((size_t)nds + 1, sizeof(size_t));
    if (!pos) return -1;
    memcpy(pos, start, ((size_t)nds + 1) * sizeof(size_t));
    for (size_t i = 0; i < n; i++) sorted[pos[recs[i].route < nds ? recs[i].route : nds]++] = recs[i];
    size_t np = 0;
    int rc = 0;
    for (uint32_t s = 0; s < nds; s++) {
        unsigned fill = fill_in ? fill_in[s] : 0;
        size_t pstart = start[s];
        unsigned pcarry = fill, plen = 0;
        for (size_t q = start[s]; q < start[s + 1]; q++) {
            unsigned L = sorted[q].length;
            if (fill + L > SR_DOWNSTREAM_BUF_SIZE) { /* sr-main.c:75-78 */
                if (np < max_packets)
                    packets[np] = (sr_packet){(uint32_t)pstart, (uint16_t)(q - pstart), (uint16_t)s,
                                              (uint16_t)plen, (uint16_t)pcarry, 0};
                np++;
                fill = 0; /* ds_schedule_flush: a new active buffer, sr-main.c:63-65 */
                pstart = q;
                pcarry = 0;
                plen = 0;
            }
            fill += L; /* :80-82 */
            plen += L;
        }
        if (start[s + 1] > start[s]) {
            if (np < max_packets)
                packets[np] = (sr_packet){(uint32_t)pstart, (uint16_t)(start[s + 1] - pstart), (uint16_t)s,
                                          (uint16_t)plen, (uint16_t)pcarry, 1};
            np++;
        }
        if (probed_dead && ((probed_dead[s >> 6] >> (s & 63)) & 1u)) fill = 0; /* sr-main.c:106 */
        fill_out[s] = (uint16_t)fill;
    }
    if (np > max_packets) rc = -1;
    *n_packets = np;
    *n_valid = start[nds];
    free(start);
    free(pos);
    return rc;
}

/* sr-main.c:175-189 over a batch of framed datagrams laid back to back. Every framed datagram
 * ends in '\n', so the lines of the concatenation are exactly the lines of the datagrams and
 * datagram boundaries need not be known. Bytes after the last '\n' are not a line. */
size_t sro_route_batch(const uint8_t *buf, size_t nbytes, uint32_t downstream_num,
                       const uint64_t *alive, sr_record *out, size_t max_records,
                       uint64_t *hashes) {
    const uint8_t *ptr = buf;
    size_t rem = nbytes;
    size_t n = 0;
    const uint8_t *delim;
    while (rem > 0 && (delim = memchr(ptr, '\n', rem)) != NULL) { /* :175 */
        size_t len = (size_t)(delim + 1 - ptr);                    /* :176-177 */
        uint16_t route;
        uint64_t h = 0;
        if (len > 5 && len < SR_DOWNSTREAM_BUF_SIZE) {             /* :180 */
            if (sro_hash(ptr, len, &h) != 0) {                     /* :140 */
                route = SR_ROUTE_INVALID_FORMAT;                   /* :141-143 */
                h = 0;
            } else {
                int k = sro_find_downstream(h, downstream_num, alive); /* :145 */
                route = k < 0 ? SR_ROUTE_ALL_DEAD : (uint16_t)k;
            }
        } else {
            route = SR_ROUTE_INVALID_LENGTH;                       /* :184 */
        }
        if (n < max_records) {
            out[n].offset = (uint32_t)(ptr - buf);
            out[n].length = len > 0xFFFF ? 0xFFFF : (uint16_t)len;
            out[n].route = route;
            if (hashes) hashes[n] = h;
        }
        n++;
        ptr = delim + 1; /* :187-188 */
        rem -= len;
    }
    return n;
}

size_t sro_route_datagrams(const uint8_t *dgrams, const uint32_t *lens, size_t count,
                           uint8_t *framed, size_t framed_cap, size_t *framed_len,
                           uint32_t downstream_num, const uint64_t *alive, sr_record *out,
                           size_t max_records, uint64_t *hashes) {
    size_t pos = 0, off = 0;
    for (size_t d = 0; d < count; d++) {
        size_t need = (lens[d] < SR_MAX_DATAGRAM ? lens[d] : SR_MAX_DATAGRAM) + 1;
        if (pos + need > framed_cap) return (size_t)-1;
        pos += sro_frame_datagram(framed + pos, dgrams + off, lens[d]);
        off += lens[d];
    }
    *framed_len = pos;
    return sro_route_batch(framed, pos, downstream_num, alive, out, max_records, hashes);
}

/* ---- CPU baseline timing harness ---------------------------------------------------------- */
/* Each thread is one reference data thread (threads_num, sr-main.c:363-367) with its own
 * output array, routing the given batches round-robin until `seconds` of wall time elapse. */
typedef struct {
    const uint8_t *const *batches;
    const size_t *sizes;
    size_t nbatch;
    uint32_t nds;
    const uint64_t *alive;
    double seconds;
    size_t first;
    sr_record *out;
    size_t out_cap;
    uint64_t lines, bytes;
    double elapsed;
} bench_arg;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *bench_thread(void *p) {
    bench_arg *a = (bench_arg *)p;
    double t0 = now_s(), t = t0;
    size_t b = a->first;
    do {
        size_t k = b % a->nbatch;
        a->lines += sro_route_batch(a->batches[k], a->sizes[k], a->nds, a->alive, a->out,
                                    a->out_cap, NULL);
        a->bytes += a->sizes[k];
        b++;
        t = now_s();
    } while (t - t0 < a->seconds);
    a->elapsed = t - t0;
    return NULL;
}

int sro_bench(const uint8_t *const *batches, const size_t *sizes, size_t nbatch, uint32_t nds,
              const uint64_t *alive, int threads, double seconds, uint64_t *lines,
              uint64_t *bytes, double *wall) {
    if (threads < 1 || nbatch == 0) return -1;
    size_t cap = 0;
    for (size_t i = 0; i < nbatch; i++)
        if (sizes[i] > cap) cap = sizes[i];
    pthread_t *tid = calloc((size_t)threads, sizeof(pthread_t));
    bench_arg *args = calloc((size_t)threads, sizeof(bench_arg));
    if (!tid || !args) return -1;
    double t0 = now_s();
    for (int i = 0; i < threads; i++) {
        args[i] = (bench_arg){batches, sizes, nbatch, nds, alive, seconds, (size_t)i, NULL, cap,
                              0, 0, 0.0};
        args[i].out = malloc(cap * sizeof(sr_record));
        pthread_create(&tid[i], NULL, bench_thread, &args[i]);
    }
    uint64_t l = 0, by = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(tid[i], NULL);
        l += args[i].lines;
        by += args[i].bytes;
        free(args[i].out);
    }
    *wall = now_s() - t0;
    *lines = l;
    *bytes = by;
    free(tid);
    free(args);
    return 0;
}
