/*
 * sr_router_main.c — statsd-router-mi355x: a drop-in for the reference's statsd-router executable
 * (same command line, config file, UDP/TCP surface and log lines), with every data line routed
 * and packed on the GPU.
 *
 *   main              sr-main.c:310-372   config, control port, health-check timer, data threads
 *   data_pipe_thread  sr-main.c:237-308   per thread: UDP socket on data_port with SO_REUSEPORT,
 *                                         outgoing sockets, read watcher, flush and ping timers
 *   udp_read_cb       sr-main.c:149-191   here: recvmmsg drains the socket (each datagram capped at
 *                                         4095 bytes, '\n' appended when missing, :163-173) into
 *                                         one page-locked batch, routed by sr_core_route
 *   ds_flush_cb       sr-main.c:21-46     here: the packets of a call go out with sendmmsg
 *
 * Batching is adaptive: a read event routes whatever the socket holds (one datagram under light
 * load, up to the batch size under load), so latency stays one GPU round trip and throughput
 * grows with the offered rate.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include "sr_host.h"

#define RECV_VLEN 256      /* datagrams per recvmmsg call */
#define SEND_VLEN 512      /* packets per sendmmsg call */
#define READ_EVENT_SECONDS 0.02  /* a read event returns to the loop (its timers) after this long */

typedef struct data_thread {
    sr_thread *t;
    sr_config *c;
    struct ev_loop *loop;
    ev_io io;
    ev_idle idle;            /* completes the batch in flight once the loop has nothing else to do */
    ev_periodic flush_timer, ping_timer;
    sr_core *core;
    int sock_in;
    int *sock_out;
    /* ingress: two page-locked batches (the core's slots); the one being filled is `slot` */
    uint8_t *batch;          /* framed datagrams back to back: the buffer of `slot` */
    size_t cap, len;
    int slot;
    struct mmsghdr rmsg[RECV_VLEN];
    struct iovec riov[RECV_VLEN];
    /* log_level TRACE: the framed datagrams' end offsets in the batch (sr_core_submit_datagrams) */
    int trace;
    uint32_t *ends;
    size_t nends, ends_cap;
    /* egress: per outgoing socket, packets staged for one sendmmsg */
    int nout;
    struct mmsghdr *smsg;    /* [nout][SEND_VLEN] */
    struct iovec *siov;
    uint8_t *stage;          /* [nout][SEND_VLEN][1450] */
    int *nq;
    uint64_t alive_gen;
    uint64_t *alive;
} data_thread;

static void send_queue(data_thread *d, int o) {
    int sent = 0, n = d->nq[o];
    struct mmsghdr *m = d->smsg + (size_t)o * SEND_VLEN;
    while (sent < n) {
        int r = sendmmsg(d->sock_out[o], m + sent, (unsigned)(n - sent), 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            sr_log(SR_WARN, "%s: sendto() failed %s", "ds_flush_cb", strerror(errno));
            sent++;   /* the reference drops a packet whose sendto fails (sr-main.c:38-45) */
            continue;
        }
        sent += r;
    }
    d->nq[o] = 0;
}

static void on_flush(void *user) {
    data_thread *d = user;
    for (int o = 0; o < d->nout; o++)
        if (d->nq[o]) send_queue(d, o);
}

/* a packet from the core: copied into the staging slot of its outgoing socket */
static void on_emit(void *user, uint32_t ds, const struct iovec *iov, int iovcnt, size_t bytes) {
    data_thread *d = user;
    const int o = (int)(ds % (uint32_t)d->nout);   /* sr-main.c:286-288 */
    if (d->nq[o] == SEND_VLEN) send_queue(d, o);
    const size_t k = (size_t)o * SEND_VLEN + (size_t)d->nq[o]++;
    uint8_t *dst = d->stage + k * SR_DOWNSTREAM_BUF_SIZE;
    size_t off = 0;
    for (int i = 0; i < iovcnt; i++) {
        memcpy(dst + off, iov[i].iov_base, iov[i].iov_len);
        off += iov[i].iov_len;
    }
    d->siov[k] = (struct iovec){dst, bytes};
    struct msghdr *h = &d->smsg[k].msg_hdr;
    memset(h, 0, sizeof(*h));
    h->msg_name = &d->c->ds_addr[ds];
    h->msg_namelen = sizeof(struct sockaddr_in);
    h->msg_iov = &d->siov[k];
    h->msg_iovlen = 1;
}

static void on_log(void *user, int level, const char *msg, size_t len) {
    (void)user;
    sr_log_text(level, msg, len);
}

static void refresh_alive(data_thread *d) {
    const uint64_t g = atomic_load_explicit(&d->c->alive_gen, memory_order_acquire);
    if (g == d->alive_gen) return;
    d->alive_gen = g;
    for (int w = 0; w < (d->c->downstream_num + 63) / 64; w++)
        d->alive[w] = atomic_load_explicit(&d->c->alive_words[w], memory_order_relaxed);
    int rc = sr_core_set_alive(d->core, d->alive);
    if (rc) sr_log(SR_ERROR, "%s: sr_core_set_alive() failed %s", "data_pipe_thread", strerror(-rc));
}

/* A read event's batch goes to the GPU while the next one is received (sr_core_submit: slot k routes
 * while slot k^1 fills; the batch before it is walked and sent when k is submitted). A read event
 * ends with its batch in flight: the next read event completes it, or, when the loop finds nothing
 * else to do, the idle watcher does, so a lone datagram still costs about one GPU round trip. */
static void submit_batch(data_thread *d) {
    if (!d->len) return;
    refresh_alive(d);
    int rc = sr_core_submit_datagrams(d->core, d->slot, d->len, d->ends, d->nends);
    if (rc) sr_log(SR_ERROR, "%s: sr_core_submit() failed %s", "udp_read_cb", strerror(-rc));
    d->len = 0;
    d->nends = 0;
    if (sr_core_in_flight(d->core) != d->slot) {
        /* the batch was not taken (its lines are lost, as the ERROR says): complete the one in
         * flight and keep filling this slot, which no GPU work reads */
        int rc2 = sr_core_drain(d->core);
        if (rc2) sr_log(SR_ERROR, "%s: sr_core_drain() failed %s", "udp_read_cb", strerror(-rc2));
        return;
    }
    d->slot ^= 1;
    d->batch = sr_core_slot_buffer(d->core, d->slot, &d->cap);
}

static void drain(data_thread *d) {
    ev_idle_stop(d->loop, &d->idle);
    int rc = sr_core_drain(d->core);
    if (rc) sr_log(SR_ERROR, "%s: sr_core_drain() failed %s", "udp_read_cb", strerror(-rc));
}

static void idle_cb(struct ev_loop *loop, ev_idle *w, int revents) {
    (void)loop, (void)revents;
    drain((data_thread *)((char *)w - offsetof(data_thread, idle)));
}

static void route_batch(data_thread *d) {
    submit_batch(d);
    drain(d);
}

static void udp_read_cb(struct ev_loop *loop, ev_io *w, int revents) {
    (void)loop;
    data_thread *d = (data_thread *)((char *)w - offsetof(data_thread, io));
    if (EV_ERROR & revents) {
        sr_log(SR_WARN, "%s: invalid event %s", "udp_read_cb", strerror(errno));
        return;
    }
    /* Under sustained load the socket never drains: after READ_EVENT_SECONDS (checked at each full
     * batch) the event returns to the loop (the socket is still readable, so it comes straight back),
     * and the flush, ping and alive timers run in between, as they do between the reference's
     * one-datagram reads. A cap of 4 batches per event instead cost a third of the delivered lines at
     * one data thread and two senders (profiles/r04/c1_ab_r4g.jsonl). */
    int batches = 0;
    const ev_tstamp t0 = d->c->dt_yield_s > 0 ? ev_time() : 0;
    for (;;) {
        if (d->cap - d->len < (size_t)RECV_VLEN * SR_DATA_BUF_SIZE) {
            if (d->c->dt_sync) route_batch(d);
            else submit_batch(d);
            if (d->c->dt_yield && ++batches >= d->c->dt_yield) break;
            if (d->c->dt_yield_s > 0 && ev_time() - t0 >= d->c->dt_yield_s) break;
        }
        /* datagram j lands in its own 4096-byte slot after the batch's end, capped at 4095 bytes
         * like recv(fd, buffer, DATA_BUF_SIZE - 1) (sr-main.c:163), then is moved down and framed */
        for (int j = 0; j < RECV_VLEN; j++) {
            d->riov[j] = (struct iovec){d->batch + d->len + (size_t)j * SR_DATA_BUF_SIZE, SR_MAX_DATAGRAM};
            memset(&d->rmsg[j].msg_hdr, 0, sizeof(struct msghdr));
            d->rmsg[j].msg_hdr.msg_iov = &d->riov[j];
            d->rmsg[j].msg_hdr.msg_iovlen = 1;
        }
        const size_t len0 = d->len;
        int k = recvmmsg(d->sock_in, d->rmsg, RECV_VLEN, MSG_DONTWAIT, NULL);
        if (k < 0) {
            if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
                sr_log(SR_WARN, "%s: recv() failed %s", "udp_read_cb", strerror(errno));
            break;
        }
        for (int j = 0; j < k; j++) {
            size_t n = d->rmsg[j].msg_len;
            if (n == 0) continue;   /* an empty datagram has no lines (sr-main.c:170) */
            const uint8_t *src = d->batch + len0 + (size_t)j * SR_DATA_BUF_SIZE;
            uint8_t *dst = d->batch + d->len;   /* never above src: framed datagrams are <= 4096 B */
            if (dst != src) memmove(dst, src, n);
            if (dst[n - 1] != '\n') dst[n++] = '\n';   /* sr-main.c:171-173 */
            d->len += n;
            if (d->trace) {   /* "got packet" per datagram at TRACE (sr-main.c:174) */
                if (d->nends == d->ends_cap) {
                    const size_t nc = d->ends_cap ? 2 * d->ends_cap : 4096;
                    uint32_t *p = realloc(d->ends, nc * sizeof(uint32_t));
                    if (!p) {
                        d->trace = 0;   /* the lines' own TRACE messages still follow */
                        sr_log(SR_ERROR, "%s: malloc() failed %s", "udp_read_cb", strerror(errno));
                        continue;
                    }
                    d->ends = p;
                    d->ends_cap = nc;
                }
                d->ends[d->nends++] = (uint32_t)d->len;
            }
        }
        if (k < RECV_VLEN) break;   /* drained */
    }
    if (d->c->dt_sync) {
        route_batch(d);
        return;
    }
    submit_batch(d);
    ev_idle_start(d->loop, &d->idle);
}

static void flush_timer_cb(struct ev_loop *loop, ev_periodic *p, int revents) {
    (void)loop, (void)revents;
    data_thread *d = (data_thread *)((char *)p - offsetof(data_thread, flush_timer));
    route_batch(d);
    sr_core_flush_timer(d->core);
}

static void ping_timer_cb(struct ev_loop *loop, ev_periodic *p, int revents) {
    (void)loop, (void)revents;
    data_thread *d = (data_thread *)((char *)p - offsetof(data_thread, ping_timer));
    route_batch(d);
    refresh_alive(d);
    int rc = sr_core_ping(d->core);
    if (rc) sr_log(SR_ERROR, "%s: sr_core_ping() failed %s", "ping_cb", strerror(-rc));
}

/* a data thread that cannot route: the process ends (status 1) unless SR_REQUIRE_GPU=0 */
static void *thread_fail(data_thread *d, int gpu) {
    if (d->sock_in >= 0) close(d->sock_in);
    if (gpu && d->c->require_gpu) {
        fflush(stdout);
        _exit(1);
    }
    return NULL;
}

void *sr_data_thread(void *arg) {
    sr_thread *t = arg;
    sr_config *c = t->config;
    const char *fn = "data_pipe_thread";
    data_thread *d = calloc(1, sizeof(*d));
    if (!d) return NULL;
    d->t = t;
    d->c = c;
    d->sock_in = -1;
    d->loop = ev_loop_new(0);
    d->sock_in = socket(PF_INET, SOCK_DGRAM, 0);
    if (d->sock_in < 0) {
        sr_log(SR_ERROR, "%s: socket_in socket() error %s", fn, strerror(errno));
        return thread_fail(d, 0);
    }
    struct sockaddr_in addr;
    memset(&addr, 0, sizeof(addr));
    addr.sin_family = AF_INET;
    addr.sin_port = htons((uint16_t)c->data_port);
    addr.sin_addr.s_addr = INADDR_ANY;
    int one = 1;
    if (setsockopt(d->sock_in, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one)) != 0) {
        sr_log(SR_ERROR, "%s: setsockopt() failed %s", fn, strerror(errno));
        return thread_fail(d, 0);
    }
    int rcvbuf = 32 << 20;
    setsockopt(d->sock_in, SOL_SOCKET, SO_RCVBUF, &rcvbuf, sizeof(rcvbuf));
    if (bind(d->sock_in, (struct sockaddr *)&addr, sizeof(addr)) != 0) {
        sr_log(SR_ERROR, "%s: bind() failed %s", fn, strerror(errno));
        return thread_fail(d, 0);
    }
    /* bound first (datagrams queue while the GPU context opens, as they do while the reference's
     * thread starts); a thread whose GPU context cannot be opened closes its socket and ends the
     * process, so no share of the port is left unread */
    sr_core_config cc;
    memset(&cc, 0, sizeof(cc));
    cc.device = c->n_devices > 0 ? t->index % c->n_devices : 0;
    cc.max_batch_bytes = c->batch_bytes;
    cc.n_downstreams = (uint32_t)c->downstream_num;
    cc.ds_hosts = (const char *const *)c->ds_hosts;
    cc.ds_data_ports = (const char *const *)c->ds_data_ports;
    cc.ping_prefix = c->ping_prefix;
    cc.hostname = c->hostname;
    cc.data_port = c->data_port + t->index;   /* sr-init.c:57,113 */
    cc.log_level = sr_log_level;
    int rc = sr_core_open(&d->core, &cc, on_emit, on_log, on_flush, d);
    if (rc) {
        sr_log(SR_ERROR, "%s: sr_core_open() failed %s", fn, strerror(-rc));
        return thread_fail(d, 1);
    }
    d->slot = 0;
    d->batch = sr_core_slot_buffer(d->core, 0, &d->cap);
    d->trace = sr_log_level <= SR_TRACE;
    d->nout = c->socket_out_num;
    d->sock_out = calloc((size_t)d->nout, sizeof(int));
    d->smsg = calloc((size_t)d->nout * SEND_VLEN, sizeof(struct mmsghdr));
    d->siov = calloc((size_t)d->nout * SEND_VLEN, sizeof(struct iovec));
    d->stage = malloc((size_t)d->nout * SEND_VLEN * SR_DOWNSTREAM_BUF_SIZE);
    d->nq = calloc((size_t)d->nout, sizeof(int));
    d->alive = calloc((size_t)(c->downstream_num + 63) / 64, sizeof(uint64_t));
    if (!d->sock_out || !d->smsg || !d->siov || !d->stage || !d->nq || !d->alive) {
        sr_log(SR_ERROR, "%s: malloc() failed %s", fn, strerror(errno));
        return thread_fail(d, 0);
    }
    for (int i = 0; i < d->nout; i++) {
        if ((d->sock_out[i] = socket(AF_INET, SOCK_DGRAM, IPPROTO_UDP)) < 0) {
            sr_log(SR_ERROR, "%s: socket_out socket() error %s", fn, strerror(errno));
            return thread_fail(d, 0);
        }
    }
    d->alive_gen = (uint64_t)-1;
    refresh_alive(d);
    ev_io_init(&d->io, udp_read_cb, d->sock_in, EV_READ);
    ev_io_start(d->loop, &d->io);
    ev_idle_init(&d->idle, idle_cb);
    ev_periodic_init(&d->flush_timer, flush_timer_cb, 0.0, c->downstream_flush_interval, 0);
    ev_periodic_start(d->loop, &d->flush_timer);
    ev_periodic_init(&d->ping_timer, ping_timer_cb, 0.0, c->downstream_ping_interval, 0);
    ev_periodic_start(d->loop, &d->ping_timer);
    ev_run(d->loop, 0);
    sr_log(SR_ERROR, "%s: ev_loop() exited", fn);
    return NULL;
}

/* SIGHUP / SIGINT as the reference handles them (sr-init.c:177-185,290-297): a SIGHUP is logged and
 * ignored (logrotate, init scripts), a SIGINT is logged and ends the process with status 0. Here they
 * are libev signal watchers on the main thread's loop; the process exits without running the GPU
 * runtime's teardown under the data threads. */
static void on_sighup(struct ev_loop *loop, ev_signal *w, int revents) {
    (void)loop, (void)w, (void)revents;
    sr_log(SR_INFO, "%s: sighup received", "on_sighup");
}

static void on_sigint(struct ev_loop *loop, ev_signal *w, int revents) {
    (void)loop, (void)w, (void)revents;
    sr_log(SR_INFO, "%s: sigint received", "on_sigint");
    fflush(stdout);
    _exit(0);
}

int main(int argc, char *argv[]) {
    if (argc != 2) {
        fprintf(stdout, "Usage: %s config.file\n", argv[0]);
        exit(1);
    }
    static sr_config config;
    if (sr_init_config(argv[1], &config) != 0) {
        sr_log(SR_ERROR, "%s: init_config() failed", "main");
        exit(1);
    }
    /* GPU knobs outside the reference's config keys (the config file stays the reference's) */
    const char *bb = getenv("SR_BATCH_BYTES");
    config.batch_bytes = bb ? (size_t)strtoull(bb, NULL, 0) : (size_t)8 << 20;
    if (config.batch_bytes < (size_t)2 * RECV_VLEN * SR_DATA_BUF_SIZE) config.batch_bytes = (size_t)2 * RECV_VLEN * SR_DATA_BUF_SIZE;
    const char *nd = getenv("SR_DEVICES");
    config.n_devices = nd ? atoi(nd) : 1;
    const char *ds = getenv("SR_DT_SYNC"), *dy = getenv("SR_DT_YIELD"), *dys = getenv("SR_DT_YIELD_S");
    config.dt_sync = ds && ds[0] == '1';
    config.dt_yield = dy ? atoi(dy) : 0;
    config.dt_yield_s = dys ? atof(dys) : READ_EVENT_SECONDS;

    struct ev_loop *loop = ev_default_loop(0);
    const char *fn = "main";
    static ev_signal sighup_w, sigint_w;
    ev_signal_init(&sighup_w, on_sighup, SIGHUP);
    ev_signal_start(loop, &sighup_w);
    ev_signal_init(&sigint_w, on_sigint, SIGINT);
    ev_signal_start(loop, &sigint_w);
    /* a data thread whose GPU context cannot be opened ends the process (status 1) instead of leaving
     * its share of the SO_REUSEPORT traffic unread; SR_REQUIRE_GPU=0 keeps the main thread's services
     * (control port, health checks) running without data threads, for host-surface tests on CPU */
    const char *rg = getenv("SR_REQUIRE_GPU");
    config.require_gpu = !(rg && rg[0] == '0');
    int cs = socket(PF_INET, SOCK_STREAM, 0);
    if (cs < 0) {
        sr_log(SR_ERROR, "%s: socket() error %s", fn, strerror(errno));
        return 1;
    }
    struct sockaddr_in addr;
    memset(&addr, 0, sizeof(addr));
    addr.sin_family = AF_INET;
    addr.sin_port = htons((uint16_t)config.control_port);
    addr.sin_addr.s_addr = INADDR_ANY;
    int one = 1;
    setsockopt(cs, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (bind(cs, (struct sockaddr *)&addr, sizeof(addr)) != 0) {
        sr_log(SR_ERROR, "%s: bind() failed %s", fn, strerror(errno));
        return 1;
    }
    if (listen(cs, 4096) < 0) {
        sr_log(SR_ERROR, "%s: listen() error %s", fn, strerror(errno));
        return 1;
    }
    config.control_socket = cs;
    static sr_control_io control;
    memset(&control, 0, sizeof(control));
    control.health_response = config.health_check_response_buf;
    control.health_response_len = &config.health_check_response_buf_length;
    ev_io_init(&control.super, sr_control_accept_cb, cs, EV_READ);
    ev_io_start(loop, &control.super);

    static sr_health_timer ht;
    ht.config = &config;
    ev_periodic_init(&ht.super, sr_health_check_timer_cb, 0.0, config.downstream_health_check_interval, 0);
    ev_periodic_start(loop, &ht.super);

    sr_thread *threads = calloc((size_t)config.threads_num, sizeof(sr_thread));
    for (int i = 0; i < config.threads_num; i++) {
        threads[i].index = i;
        threads[i].config = &config;
        pthread_create(&threads[i].thread, NULL, sr_data_thread, &threads[i]);
    }
    ev_run(loop, 0);
    sr_log(SR_ERROR, "%s: ev_loop() exited", fn);
    return 0;
}
