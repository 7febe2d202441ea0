/*
 * sr_sink — loopback downstreams for the C1 measurement and the router's end-to-end tests: what the
 * reference's test library's StatsdMock does (statsd-router-test-lib.rb:45-167), in C so it keeps
 * up with a router at full rate.
 *
 * For downstream i it binds UDP 127.0.0.1:<base + 2i> (data) and TCP <base + 2i + 1> (health: answers
 * every "health" request with "health: up\n", sr-types.h:96). It counts datagrams, lines and bytes
 * per downstream and stops after <seconds>, or once <idle> seconds pass without data after data began.
 *
 * usage: sr_sink <base port> <n downstreams> <seconds> [idle=1.0] [dump file]
 * dump file: every datagram received, [u16 downstream][u16 length][bytes].
 * prints one JSON line when it stops; "ready" on stderr once every socket listens.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#define MAXN 64
#define VLEN 256
#define MAXCONN 64

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int bind_sock(int type, int port) {
    int s = socket(AF_INET, type, 0);
    int one = 1;
    setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (type == SOCK_DGRAM) {
        int rb = 64 << 20;
        setsockopt(s, SOL_SOCKET, SO_RCVBUF, &rb, sizeof(rb));
    }
    struct sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind(s, (struct sockaddr *)&a, sizeof(a)) != 0) {
        fprintf(stderr, "bind %d: %s\n", port, strerror(errno));
        exit(3);
    }
    if (type == SOCK_STREAM) listen(s, 64);
    fcntl(s, F_SETFL, O_NONBLOCK);
    return s;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s base_port n seconds [idle] [dump]\n", argv[0]);
        return 2;
    }
    const int base = atoi(argv[1]), n = atoi(argv[2]);
    const double secs = atof(argv[3]), idle = argc > 4 ? atof(argv[4]) : 1.0;
    FILE *dump = argc > 5 ? fopen(argv[5], "wb") : NULL;
    if (n < 1 || n > MAXN) return 2;
    int udp[MAXN], tcp[MAXN];
    for (int i = 0; i < n; i++) {
        udp[i] = bind_sock(SOCK_DGRAM, base + 2 * i);
        tcp[i] = bind_sock(SOCK_STREAM, base + 2 * i + 1);
    }
    int conn[MAXCONN], nconn = 0;
    uint64_t dg[MAXN] = {0}, lines[MAXN] = {0}, bytes[MAXN] = {0};
    static char buf[VLEN][2048];
    static struct mmsghdr m[VLEN];
    static struct iovec iov[VLEN];
    fprintf(stderr, "ready\n");
    fflush(stderr);
    const double t0 = now();
    double first = -1, last = -1;
    struct pollfd pf[2 * MAXN + MAXCONN];
    for (;;) {
        double t = now();
        if (t - t0 > secs || (last > 0 && t - last > idle)) break;
        int np = 0;
        for (int i = 0; i < n; i++) pf[np++] = (struct pollfd){udp[i], POLLIN, 0};
        for (int i = 0; i < n; i++) pf[np++] = (struct pollfd){tcp[i], POLLIN, 0};
        for (int i = 0; i < nconn; i++) pf[np++] = (struct pollfd){conn[i], POLLIN, 0};
        if (poll(pf, (nfds_t)np, 50) <= 0) continue;
        for (int i = 0; i < n; i++) {
            if (!(pf[i].revents & POLLIN)) continue;
            for (;;) {
                for (int j = 0; j < VLEN; j++) {
                    iov[j] = (struct iovec){buf[j], sizeof(buf[j])};
                    memset(&m[j].msg_hdr, 0, sizeof(m[j].msg_hdr));
                    m[j].msg_hdr.msg_iov = &iov[j];
                    m[j].msg_hdr.msg_iovlen = 1;
                }
                int r = recvmmsg(udp[i], m, VLEN, MSG_DONTWAIT, NULL);
                if (r <= 0) break;
                last = now();
                if (first < 0) first = last;
                for (int j = 0; j < r; j++) {
                    const unsigned len = m[j].msg_len;
                    dg[i]++;
                    bytes[i] += len;
                    for (unsigned q = 0; q < len; q++) lines[i] += buf[j][q] == '\n';
                    if (dump) {
                        uint16_t d = (uint16_t)i, l = (uint16_t)len;
                        fwrite(&d, 2, 1, dump);
                        fwrite(&l, 2, 1, dump);
                        fwrite(buf[j], 1, len, dump);
                    }
                }
                if (r < VLEN) break;
            }
        }
        for (int i = 0; i < n; i++) {
            if (!(pf[n + i].revents & POLLIN)) continue;
            int c = accept(tcp[i], NULL, NULL);
            if (c >= 0 && nconn < MAXCONN) {
                fcntl(c, F_SETFL, O_NONBLOCK);
                conn[nconn++] = c;
            } else if (c >= 0) {
                close(c);
            }
        }
        /* health connections (persistent, like the reference's health client keeps them): poll
         * indices were taken before any accept above, so walk the polled ones by index and compact
         * after */
        const int polled = np - 2 * n;
        for (int i = 0; i < polled; i++) {
            if (!(pf[2 * n + i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
            char req[64];
            ssize_t r = recv(conn[i], req, sizeof(req), 0);
            if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) continue;
            if (r <= 0 || send(conn[i], "health: up\n", 11, MSG_NOSIGNAL) < 0) {
                close(conn[i]);
                conn[i] = -1;
            }
        }
        int k = 0;
        for (int i = 0; i < nconn; i++)
            if (conn[i] >= 0) conn[k++] = conn[i];
        nconn = k;
    }
    if (dump) fclose(dump);
    uint64_t td = 0, tl = 0, tb = 0;
    printf("{\"downstreams\": [");
    for (int i = 0; i < n; i++) {
        printf("%s{\"datagrams\": %llu, \"lines\": %llu, \"bytes\": %llu}", i ? ", " : "", (unsigned long long)dg[i],
               (unsigned long long)lines[i], (unsigned long long)bytes[i]);
        td += dg[i], tl += lines[i], tb += bytes[i];
    }
    printf("], \"datagrams\": %llu, \"lines\": %llu, \"bytes\": %llu, \"first\": %.6f, \"last\": %.6f, "
           "\"first_abs\": %.6f, \"last_abs\": %.6f}\n",
           (unsigned long long)td, (unsigned long long)tl, (unsigned long long)tb, first > 0 ? first - t0 : -1.0,
           last > 0 ? last - t0 : -1.0, first, last);
    return 0;
}
