/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Calibration of the CPU baseline: the reference's own read callback (udp_read_cb, sr-main.c:149-191,
 * compiled unmodified by oracle/Makefile) against the C restatement (sr_oracle.c) on the same
 * datagrams, one thread, both timed here. The reference runs as in production with
 * log_level = ERROR (so TRACE/WARN calls return at sr-util.c:17), its lines pushed into real
 * downstream buffers (push_to_downstream, :73-83); the flush ring is drained after every datagram
 * the way an always-writable socket would (buffer lengths cleared, sr-main.c:38-39), so no packet
 * is dropped by "previous flush is not completed". Each datagram crosses an AF_UNIX socketpair
 * (the recv of :163) for the reference; the restatement routes the same datagrams framed in memory
 * (its timing excludes the recv, as bench.py's cpu_baseline does).
 *
 * usage: sr_ref_bench <n_downstreams> <datagrams file: [u32 len][bytes]...> <seconds>
 * prints one JSON line.
 */
#include "sr-main.h" /* from /root/reference, via -I */

#include <stdint.h>
#include <sys/socket.h>

#include "sr_oracle.h"

void udp_read_cb(struct ev_loop *loop, struct ev_io *watcher, int revents);

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

int main(int argc, char **argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: %s n_downstreams datagrams seconds\n", argv[0]);
        return 2;
    }
    const int n = atoi(argv[1]);
    const double secs = atof(argv[3]);
    FILE *in = fopen(argv[2], "rb");
    if (!in) return 3;
    size_t cap = 1 << 20, used = 0, nd = 0, dcap = 1 << 14;
    uint8_t *blob = malloc(cap);
    uint32_t *lens = malloc(dcap * sizeof(uint32_t));
    uint32_t l;
    while (fread(&l, 4, 1, in) == 1) {
        if (used + l > cap) blob = realloc(blob, cap = 2 * (used + l));
        if (nd == dcap) lens = realloc(lens, (dcap *= 2) * sizeof(uint32_t));
        if (fread(blob + used, 1, l, in) != l) return 4;
        lens[nd++] = l;
        used += l;
    }
    fclose(in);

    log_level = ERROR;
    struct ev_loop *loop = ev_default_loop(0);
    struct downstream_s *ds = calloc((size_t)n, sizeof(struct downstream_s));
    struct ds_health_client_s *hc = calloc((size_t)n, sizeof(struct ds_health_client_s));
    int out_fd = socket(AF_INET, SOCK_DGRAM, 0);
    for (int i = 0; i < n; i++) {
        ds[i].active_buffer = ds[i].buffer;
        ds[i].health_client = &hc[i];
        ds[i].socket_out = &out_fd;
        hc[i].alive = 1;
    }
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_DGRAM, 0, sv) != 0) return 5;
    struct ev_io_ds_s w;
    memset(&w, 0, sizeof(w));
    ev_io_init((struct ev_io *)&w, udp_read_cb, sv[1], EV_READ);
    w.downstream_num = n;
    w.downstream = ds;

    /* lines per pass (framing as the reference does it) */
    uint8_t *framed = malloc(used + nd + 16);
    size_t flen = 0;
    sr_record *recs = malloc((used + nd + 16) * sizeof(sr_record));
    const size_t lines =
        sro_route_datagrams(blob, lens, nd, framed, used + nd + 16, &flen, (uint32_t)n, (uint64_t[]){~0ull}, recs,
                            used + nd + 16, NULL);

    /* the reference: send + udp_read_cb per datagram, the ring drained after each */
    size_t passes = 0;
    double t0 = now(), t = t0;
    do {
        size_t off = 0;
        for (size_t d = 0; d < nd; d++) {
            if (send(sv[0], blob + off, lens[d], 0) != (ssize_t)lens[d]) return 6;
            udp_read_cb(loop, (struct ev_io *)&w, EV_READ);
            off += lens[d];
            for (int i = 0; i < n; i++)
                while (ds[i].flush_buffer_idx != ds[i].active_buffer_idx) {
                    ds[i].buffer_length[ds[i].flush_buffer_idx] = 0;
                    ds[i].flush_buffer_idx = (ds[i].flush_buffer_idx + 1) % DOWNSTREAM_BUF_NUM;
                }
        }
        passes++;
        t = now();
    } while (t - t0 < secs);
    const double ref_rate = (double)(passes * lines) / (t - t0);

    /* the restatement on the same framed datagrams */
    uint64_t alive[1024];
    memset(alive, 0xFF, sizeof(alive));
    passes = 0;
    t0 = now();
    do {
        sro_route_batch(framed, flen, (uint32_t)n, alive, recs, used + nd + 16, NULL);
        passes++;
        t = now();
    } while (t - t0 < secs);
    const double port_rate = (double)(passes * lines) / (t - t0);
    printf("{\"lines_per_pass\": %zu, \"reference_lines_per_s\": %.1f, \"restatement_lines_per_s\": %.1f, "
           "\"restatement_over_reference\": %.4f}\n",
           lines, ref_rate, port_rate, port_rate / ref_rate);
    return 0;
}
