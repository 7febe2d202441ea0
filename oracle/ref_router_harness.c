/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Drives one data thread of the REFERENCE router, compiled by oracle/Makefile from the unmodified
 * sources under /root/reference, through a scripted sequence of events and records everything it
 * sends and logs:
 *   - setup: the reference's own init_config (sr-init.c:241-331) on the given statsd-router.conf,
 *     which builds the downstream array, the health clients and the ping metric names
 *     (sr-init.c:57,112-118); thread 0's downstreams are used, as data_pipe_thread does
 *     (sr-main.c:249);
 *   - a datagram  -> sent over an AF_UNIX socketpair, then the reference's udp_read_cb
 *     (sr-main.c:149-191) on the receiving end, as libev would call it;
 *   - an alive snapshot -> the health clients' alive bits (sr-types.h:25);
 *   - a flush tick -> ds_flush_timer_cb (sr-main.c:194-204);
 *   - a ping tick  -> ping_cb (sr-main.c:206-235).
 * After every event each downstream's flush ring is drained with the reference's own ds_flush_cb
 * (sr-main.c:21-46), i.e. a socket that is always writable; its sendto() goes to a UDP socket this
 * harness bound for that downstream (sa_in_data is re-pointed there; the metric names keep the
 * configured ports), and every datagram received is recorded with its downstream.
 * log_msg is intercepted with the linker's --wrap: every message at or above the configured
 * log_level (the reference's own test, sr-util.c:18-20) is recorded as the text the reference formats
 * (without the timestamp / tid prefix of sr-util.c:23-24): WARN and ERROR at log_level 3, and also
 * the TRACE lines of udp_read_cb / find_downstream at log_level 0 (sr-main.c:91,102,174).
 * gethostname is intercepted the same way so that the ping metric names are reproducible
 * (sr-init.c:298): it returns SR_TEST_HOSTNAME.
 *
 * Usage: sr_ref_router <config> <events in> <events out>
 *   in : u32 tag: < 0xFFFFFF00 -> a datagram of that many bytes follows;
 *        0xFFFFFFF1 -> ceil(N/64) u64 alive words follow; 0xFFFFFFF2 flush tick; 0xFFFFFFF3 ping tick
 *   out: u8 1, u16 ds, u16 len, bytes           a packet sent to downstream ds
 *        u8 2, u8 level, u16 len, bytes         a log message (level >= log_level)
 *        u8 3, u16 ds, u16 len, bytes, u32 traffic, u32 packets   final pending buffer + counters
 */
#include "sr-main.h" /* from /root/reference, via -I */

#include <fcntl.h>
#include <stdint.h>
#include <sys/socket.h>

#define SR_TEST_HOSTNAME "sr-test-host"

void udp_read_cb(struct ev_loop *loop, struct ev_io *watcher, int revents);
void ds_flush_cb(struct ev_loop *loop, struct ev_io *watcher, int revents);
void ds_flush_timer_cb(struct ev_loop *loop, struct ev_periodic *p, int revents);
void ping_cb(struct ev_loop *loop, struct ev_periodic *p, int revents);

static FILE *out;

static void put(const void *p, size_t n) {
    if (fwrite(p, 1, n, out) != n) abort();
}

void __wrap_log_msg(int level, char *format, ...) {
    if (level < log_level) return;   /* sr-util.c:18-20 */
    char buf[1 << 14];
    va_list ap;
    va_start(ap, format);
    int n = vsnprintf(buf, sizeof(buf), format, ap);
    va_end(ap);
    if (n < 0) n = 0;
    if (n > (int)sizeof(buf) - 1) n = sizeof(buf) - 1;
    uint8_t t = 2, lv = (uint8_t)level;
    uint16_t len = (uint16_t)n;
    put(&t, 1);
    put(&lv, 1);
    put(&len, 2);
    put(buf, (size_t)n);
}

int __wrap_gethostname(char *name, size_t len) {
    strncpy(name, SR_TEST_HOSTNAME, len);
    return 0;
}

int main(int argc, char **argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: %s config events_in events_out\n", argv[0]);
        return 2;
    }
    out = fopen(argv[3], "wb");
    if (!out) return 3;
    static struct sr_config_s config;
    if (init_config(argv[1], &config) != 0) return 4;
    const int n = config.downstream_num;
    struct downstream_s *ds = config.downstream; /* thread 0 (sr-main.c:249) */
    struct ev_loop *loop = ev_default_loop(0);
    int out_fd = socket(AF_INET, SOCK_DGRAM, IPPROTO_UDP);
    int *sink = calloc((size_t)n, sizeof(int));
    if (out_fd < 0 || !sink) return 5;
    for (int i = 0; i < n; i++) {
        ds[i].socket_out = &out_fd;
        sink[i] = socket(AF_INET, SOCK_DGRAM, 0);
        struct sockaddr_in a;
        memset(&a, 0, sizeof(a));
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        a.sin_port = 0;
        int rb = 1 << 22;
        setsockopt(sink[i], SOL_SOCKET, SO_RCVBUF, &rb, sizeof(rb));
        if (bind(sink[i], (struct sockaddr *)&a, sizeof(a)) != 0) return 6;
        socklen_t al = sizeof(a);
        getsockname(sink[i], (struct sockaddr *)&a, &al);
        ds[i].sa_in_data.sin_addr = a.sin_addr;
        ds[i].sa_in_data.sin_port = a.sin_port;
        fcntl(sink[i], F_SETFL, O_NONBLOCK);
    }
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_DGRAM, 0, sv) != 0) return 7;
    int sb = 1 << 20;
    setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &sb, sizeof(sb));
    setsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &sb, sizeof(sb));
    struct ev_io_ds_s watcher;
    memset(&watcher, 0, sizeof(watcher));
    ev_io_init((struct ev_io *)&watcher, udp_read_cb, sv[1], EV_READ);
    watcher.downstream_num = n;
    watcher.downstream = ds;
    struct ev_periodic_ds_s flush_w, ping_w;
    memset(&flush_w, 0, sizeof(flush_w));
    memset(&ping_w, 0, sizeof(ping_w));
    flush_w.downstream_num = ping_w.downstream_num = n;
    flush_w.downstream = ping_w.downstream = ds;
    ping_w.string = config.thread_config[0].alive_downstream_metric_name;

    FILE *in = fopen(argv[2], "rb");
    if (!in) return 8;
    static uint8_t dg[1 << 16];
    static char pkt[1 << 16];
    const int nw = (n + 63) / 64;
    uint64_t *alive = calloc((size_t)(nw ? nw : 1), sizeof(uint64_t));
    uint32_t tag;
    while (fread(&tag, 4, 1, in) == 1) {
        if (tag == 0xFFFFFFF1u) {
            if (fread(alive, 8, (size_t)nw, in) != (size_t)nw) return 9;
            for (int i = 0; i < n; i++) config.health_client[i].alive = (alive[i / 64] >> (i % 64)) & 1u;
            continue;
        } else if (tag == 0xFFFFFFF2u) {
            ds_flush_timer_cb(loop, (struct ev_periodic *)&flush_w, 0);
        } else if (tag == 0xFFFFFFF3u) {
            ping_cb(loop, (struct ev_periodic *)&ping_w, 0);
        } else {
            if (tag > sizeof(dg) || fread(dg, 1, tag, in) != tag) return 10;
            if (send(sv[0], dg, tag, 0) != (ssize_t)tag) return 11;
            udp_read_cb(loop, (struct ev_io *)&watcher, EV_READ);
        }
        /* drain every flush ring through the reference's ds_flush_cb, then collect what it sent */
        for (int i = 0; i < n; i++) {
            while (ds[i].flush_buffer_idx != ds[i].active_buffer_idx)
                ds_flush_cb(loop, (struct ev_io *)&ds[i], EV_WRITE);
            ssize_t r;
            while ((r = recv(sink[i], pkt, sizeof(pkt), 0)) >= 0) {
                uint8_t t = 1;
                uint16_t d = (uint16_t)i, l = (uint16_t)r;
                put(&t, 1);
                put(&d, 2);
                put(&l, 2);
                put(pkt, (size_t)r);
            }
        }
    }
    fclose(in);
    for (int i = 0; i < n; i++) {
        uint8_t t = 3;
        uint16_t d = (uint16_t)i, l = (uint16_t)ds[i].active_buffer_length;
        uint32_t tr = (uint32_t)ds[i].downstream_traffic_counter, pk = (uint32_t)ds[i].downstream_packet_counter;
        put(&t, 1);
        put(&d, 2);
        put(&l, 2);
        put(ds[i].active_buffer, l);
        put(&tr, 4);
        put(&pk, 4);
    }
    fclose(out);
    _exit(0); /* skip the reference's on_exit cleanup (it closes sockets of threads never started) */
}
