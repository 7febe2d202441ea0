/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Drives the reference's own hot path: the object files compiled by oracle/Makefile from the
 * unmodified sources under /root/reference (sr-main.c with `main` renamed, sr-init.c,
 * sr-control-server.c, sr-health-client.c, sr-util.c) are linked with this file. Each input
 * datagram is sent over an AF_UNIX SOCK_DGRAM socketpair and the reference's
 * udp_read_cb (sr-main.c:149-191) is invoked on the receiving end, exactly as libev would after
 * a readable event. Every call the reference makes to log_msg is intercepted with the linker's
 * --wrap (nothing is printed): the TRACE/WARN events of sr-main.c:91,102,115,142,184 give, in
 * line order, the verdict, the 64-bit hash, the length and the chosen downstream of every line.
 *
 * With a 5th argument the dead-downstream side effect is recorded too: before the first datagram
 * every dead downstream gets active_buffer_length = 1 (a pending byte); find_downstream zeroes it
 * when its probe visits that downstream (sr-main.c:106), and dead downstreams receive no line. The
 * file receives ceil(N/64) u64 words: bit k = dead downstream k was probed.
 *
 * Usage: sr_ref_harness <n_downstreams> <alive words hex, comma separated> <in> <out> [probed]
 *   in : repeated [u32 length][bytes] datagrams (raw, unframed: the reference frames them)
 *   out: one 16-byte event per line: u8 verdict, u8 0, u16 route, i32 length (-1 = not logged),
 *        u64 hash (0 when the reference computed none)
 */
#include "sr-main.h" /* from /root/reference, via -I */

#include <stdint.h>
#include <sys/socket.h>

void udp_read_cb(struct ev_loop *loop, struct ev_io *watcher, int revents);

#pragma pack(push, 1)
typedef struct {
    uint8_t verdict;
    uint8_t zero;
    uint16_t route;
    int32_t length;
    uint64_t hash;
} ref_event;
#pragma pack(pop)

static ref_event *ev_buf;
static size_t ev_n, ev_cap;
static uint64_t cur_hash;
static int cur_len = -1;

static void push_event(uint8_t verdict, uint16_t route, int32_t length, uint64_t hash) {
    if (ev_n == ev_cap) {
        ev_cap = ev_cap ? 2 * ev_cap : 1 << 16;
        ev_buf = realloc(ev_buf, ev_cap * sizeof(ref_event));
        if (!ev_buf) abort();
    }
    ev_buf[ev_n++] = (ref_event){verdict, 0, route, length, hash};
}

/* Replaces every log_msg call of the reference objects (linked with -Wl,--wrap=log_msg). The
 * format strings are matched verbatim against the reference's (sr-main.c line numbers below). */
void __wrap_log_msg(int level, char *format, ...) {
    (void)level;
    va_list ap;
    va_start(ap, format);
    if (strcmp(format, "%s: hash = %lx, length = %d, line = %.*s") == 0) { /* :91 */
        (void)va_arg(ap, char *);
        cur_hash = (uint64_t)va_arg(ap, unsigned long);
        cur_len = va_arg(ap, int);
    } else if (strcmp(format, "%s: pushing to downstream %d") == 0) { /* :102 */
        (void)va_arg(ap, char *);
        int k = va_arg(ap, int);
        push_event(0, (uint16_t)k, cur_len, cur_hash);
    } else if (strcmp(format, "%s: all downstreams are dead") == 0) { /* :115 */
        push_event(3, 0xFFFF, cur_len, cur_hash);
    } else if (strcmp(format, "%s: invalid metric %s") == 0) { /* :142 */
        push_event(2, 0xFFFE, -1, 0);
    } else if (strcmp(format, "%s: invalid length %d of metric %.*s") == 0) { /* :184 */
        (void)va_arg(ap, char *);
        int len = va_arg(ap, int);
        push_event(1, 0xFFFD, len, 0);
    }
    /* "got packet" (:174) and flush-ring warnings (:57) carry no per-line information. */
    va_end(ap);
}

int main(int argc, char **argv) {
    if (argc != 5 && argc != 6) {
        fprintf(stderr, "usage: %s n_downstreams alive_hex_words in out [probed]\n", argv[0]);
        return 2;
    }
    int n = atoi(argv[1]);
    int nw = (n + 63) / 64;
    uint64_t *alive = calloc((size_t)(nw ? nw : 1), sizeof(uint64_t));
    char *save = NULL, *tok = strtok_r(argv[2], ",", &save);
    for (int w = 0; tok && w < nw; w++, tok = strtok_r(NULL, ",", &save))
        alive[w] = strtoull(tok, NULL, 16);

    struct ev_loop *loop = ev_default_loop(0);
    struct downstream_s *ds = calloc((size_t)(n ? n : 1), sizeof(struct downstream_s));
    struct ds_health_client_s *hc = calloc((size_t)(n ? n : 1), sizeof(struct ds_health_client_s));
    int out_fd = socket(AF_INET, SOCK_DGRAM, 0);
    if (!ds || !hc || out_fd < 0) return 3;
    for (int i = 0; i < n; i++) {
        ds[i].active_buffer = ds[i].buffer;
        ds[i].health_client = &hc[i];
        ds[i].socket_out = &out_fd;
        hc[i].id = i;
        hc[i].alive = (alive[i / 64] >> (i % 64)) & 1u;
        if (!hc[i].alive) ds[i].active_buffer_length = 1; /* a pending byte the probe may drop */
    }
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_DGRAM, 0, sv) != 0) return 4;
    int sndbuf = 1 << 20;
    setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &sndbuf, sizeof(sndbuf));
    setsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &sndbuf, sizeof(sndbuf));
    struct ev_io_ds_s watcher;
    memset(&watcher, 0, sizeof(watcher));
    ev_io_init((struct ev_io *)&watcher, udp_read_cb, sv[1], EV_READ);
    watcher.downstream_num = n;
    watcher.downstream = ds;

    FILE *in = fopen(argv[3], "rb");
    if (!in) return 5;
    static uint8_t dg[1 << 16];
    uint32_t len;
    while (fread(&len, 4, 1, in) == 1) {
        if (len > sizeof(dg) || fread(dg, 1, len, in) != len) return 6;
        if (send(sv[0], dg, len, 0) != (ssize_t)len) return 7;
        udp_read_cb(loop, (struct ev_io *)&watcher, EV_READ);
    }
    fclose(in);
    FILE *out = fopen(argv[4], "wb");
    if (!out) return 8;
    if (ev_n && fwrite(ev_buf, sizeof(ref_event), ev_n, out) != ev_n) return 9;
    fclose(out);
    if (argc == 6) {
        uint64_t *probed = calloc((size_t)(nw ? nw : 1), sizeof(uint64_t));
        for (int i = 0; i < n; i++)
            if (!hc[i].alive && ds[i].active_buffer_length == 0) probed[i / 64] |= 1ull << (i % 64);
        FILE *pf = fopen(argv[5], "wb");
        if (!pf || (nw && fwrite(probed, 8, (size_t)nw, pf) != (size_t)nw)) return 10;
        fclose(pf);
    }
    return 0;
}
