/*
 * sr_blast — loopback statsd load generator for config C1 (BASELINE.json configs[0]).
 *
 * The reference's own statsd-traffic-generator sends one ~19-byte datagram per libev timer tick
 * (statsd-traffic-generator.c:90-112), about 2.6 k datagrams/s at its fastest here: far too slow to
 * load a router. This sends the test/003 line shape (statsd-router-test-lib.rb:232-250
 * valid_metric(64): "statsd-cluster.count" + 'X' padding + rand(100) = a 64-byte name, then
 * ":<0..999>|c") packed whole into datagrams of at most --dgram bytes, with sendmmsg, at a target
 * rate or flat out, for a fixed time.
 *
 * usage: sr_blast <port> <seconds> <datagrams per s, 0 = max> [dgram bytes=1400] [seed=1] [pool file]
 * prints one JSON line: datagrams, lines, bytes sent, seconds.
 * With a pool file, the distinct datagrams it cycles through are written there ([u32 len][bytes]).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#define POOL 4096
#define VLEN 64

static uint64_t rng_state;
static uint64_t rnd(void) {   /* xorshift64* */
    rng_state ^= rng_state >> 12;
    rng_state ^= rng_state << 25;
    rng_state ^= rng_state >> 27;
    return rng_state * 0x2545F4914F6CDD1Dull;
}

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* valid_metric(64): a 64-byte name, then ":<counter>|c" */
static int metric(char *out) {
    char num[8];
    int nl = snprintf(num, sizeof(num), "%d", (int)(rnd() % 100));
    const char *pre = "statsd-cluster.count";
    int p = (int)strlen(pre), pad = 64 - p - nl;
    memcpy(out, pre, (size_t)p);
    memset(out + p, 'X', (size_t)pad);
    memcpy(out + p + pad, num, (size_t)nl);
    return 64 + sprintf(out + 64, ":%d|c", (int)(rnd() % 1000));
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s port seconds rate [dgram_bytes] [seed] [pool_file]\n", argv[0]);
        return 2;
    }
    const int port = atoi(argv[1]);
    const double secs = atof(argv[2]), rate = atof(argv[3]);
    const int dmax = argc > 4 ? atoi(argv[4]) : 1400;
    rng_state = 0x9E3779B97F4A7C15ull * (uint64_t)(argc > 5 ? atoll(argv[5]) : 1) + 1;
    static char pool[POOL][4096];
    static int plen[POOL], plines[POOL];
    for (int i = 0; i < POOL; i++) {
        int n = 0, k = 0;
        char line[128];
        for (;;) {
            int l = metric(line);
            if (n && n + l + 1 > dmax) break;
            if (n) pool[i][n++] = '\n';
            memcpy(pool[i] + n, line, (size_t)l);
            n += l;
            k++;
            if (n + 1 >= dmax) break;
        }
        pool[i][n++] = '\n';
        plen[i] = n;
        plines[i] = k;
    }
    if (argc > 6) {
        FILE *f = fopen(argv[6], "wb");
        for (int i = 0; f && i < POOL; i++) {
            uint32_t l = (uint32_t)plen[i];
            fwrite(&l, 4, 1, f);
            fwrite(pool[i], 1, (size_t)plen[i], f);
        }
        if (f) fclose(f);
    }
    int s = socket(AF_INET, SOCK_DGRAM, 0);
    int sb = 8 << 20;
    setsockopt(s, SOL_SOCKET, SO_SNDBUF, &sb, sizeof(sb));
    struct sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (connect(s, (struct sockaddr *)&a, sizeof(a)) != 0) return 3;
    static struct mmsghdr m[VLEN];
    static struct iovec iov[VLEN];
    uint64_t dg = 0, lines = 0, bytes = 0;
    const double t0 = now();
    double t = t0;
    int pi = 0;
    while ((t = now()) - t0 < secs) {
        if (rate > 0 && (double)dg > rate * (t - t0)) {
            usleep(50);
            continue;
        }
        for (int j = 0; j < VLEN; j++) {
            iov[j].iov_base = pool[(pi + j) % POOL];
            iov[j].iov_len = (size_t)plen[(pi + j) % POOL];
            memset(&m[j].msg_hdr, 0, sizeof(m[j].msg_hdr));
            m[j].msg_hdr.msg_iov = &iov[j];
            m[j].msg_hdr.msg_iovlen = 1;
        }
        int r = sendmmsg(s, m, VLEN, 0);
        if (r <= 0) continue;
        for (int j = 0; j < r; j++) {
            lines += (uint64_t)plines[(pi + j) % POOL];
            bytes += (uint64_t)plen[(pi + j) % POOL];
        }
        dg += (uint64_t)r;
        pi = (pi + r) % POOL;
    }
    printf("{\"datagrams\": %llu, \"lines\": %llu, \"bytes\": %llu, \"seconds\": %.6f, \"start_abs\": %.6f, "
           "\"end_abs\": %.6f}\n",
           (unsigned long long)dg, (unsigned long long)lines, (unsigned long long)bytes, t - t0, t0, t);
    return 0;
}
